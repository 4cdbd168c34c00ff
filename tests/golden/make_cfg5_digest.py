"""Reference digest of BASELINE config 5 (build container only: needs
oracle/_ref, the reference C compiled from /root/reference by oracle/Makefile).

Config 5 = an HDF5 dataset of 8 GiB uint16 (G1 + 32768, seed 12345) in 1-D
chunks of 16 Mi elements (32 MiB) through filter 32008, opts (0, 2).  Each
stored chunk is the reference filter's format (src/bshuf_h5filter.c:198-202):
u64BE uncompressed bytes || u32BE block_size*elem_size || bshuf_compress_lz4
stream.  This script computes the SHA-256 of all stored chunks concatenated in
chunk order with the reference's own bshuf_compress_lz4 and records it in
tests/golden/vectors.json["cfg5"].  Run:  python tests/golden/make_cfg5_digest.py
"""
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import Oracle, Reference  # noqa: E402

N_ELEM = 1 << 32         # 8 GiB of uint16
CHUNK = 1 << 24          # 16 Mi elements = 32 MiB


def chunk_record(codec, o, first, n):
    a = (o.gen_g1(n, first, 12345).view(np.uint16) ^ np.uint16(0x8000))  # G1 + 32768
    bs = codec.default_block_size(2)
    stream = codec.compress_lz4(a)
    hdr = int(n * 2).to_bytes(8, "big") + int(bs * 2).to_bytes(4, "big")
    return hdr, stream


def main():
    o, r = Oracle(), Reference()
    h = hashlib.sha256()
    total = 0
    for first in range(0, N_ELEM, CHUNK):
        n = min(CHUNK, N_ELEM - first)
        hdr, stream = chunk_record(r, o, first, n)
        h.update(hdr)
        h.update(stream.tobytes())
        total += len(hdr) + stream.size
    path = os.path.join(ROOT, "tests", "golden", "vectors.json")
    v = json.load(open(path))
    v["cfg5"] = dict(name="cfg5_hdf5_u16_8GiB", gen="g1+32768 uint16", seed=12345, n=N_ELEM,
                     chunk_elem=CHUNK, opts=[0, 2], stored_bytes=total, chunks_sha256=h.hexdigest())
    json.dump(v, open(path, "w"), indent=1)
    print(v["cfg5"])


if __name__ == "__main__":
    main()
