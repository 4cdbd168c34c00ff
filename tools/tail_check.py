"""Repeated encode -> decode of the 42 regression datasets through the host
C-ABI (the HDF5 filter's calls), and through the device API, reporting every
mismatch with the bytes found, the expected bytes and the stream's bytes at
the same offset.  Usage: python tools/tail_check.py ROUNDS  (GPU box)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402
from vectors import regression_cases  # noqa: E402

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
cases = regression_cases()
bad = {"host": 0, "dev": 0}
for r in range(rounds):
    for ver, name, arr, chunk, block in cases:
        stream = chunk[12:]
        raw = arr.view(np.uint8)
        enc = api.compress_lz4(arr, block)
        dec = api.decompress_lz4(stream, arr.shape, arr.dtype, block).view(np.uint8)
        if not np.array_equal(dec, raw) or enc.tobytes() != stream.tobytes():
            bad["host"] += 1
            d = np.nonzero(dec != raw)[0]
            f = int(d[0]) if d.size else -1
            print("HOST round %d %s/%s enc_ok=%s ndiff=%d first=%d got=%s want=%s stream_at=%s" % (
                r, ver, name, enc.tobytes() == stream.tobytes(), d.size, f,
                dec[f:f + 8].tobytes().hex(), raw[f:f + 8].tobytes().hex(),
                stream[f:f + 8].tobytes().hex()), flush=True)
        t = torch.from_numpy(raw.copy()).cuda()
        E = arr.dtype.itemsize
        tv = t.view(torch.uint8)
        c = api.compress_lz4_dev(tv, block) if E == 1 else None
        if c is not None:
            y = api.decompress_lz4_dev(c, tv.shape, torch.uint8, block)
            if not torch.equal(y, tv):
                bad["dev"] += 1
                print("DEV round %d %s/%s" % (r, ver, name), flush=True)
print("rounds", rounds, "bad", bad, flush=True)
