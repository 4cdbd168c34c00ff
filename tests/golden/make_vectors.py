"""Golden-vector generator (build container only: needs oracle/_ref, i.e. the
reference C compiled from /root/reference by oracle/Makefile).

Writes tests/golden/vectors.json plus small binary fixtures under
tests/golden/vectors/:
  * correlated synthetic inputs (SURVEY.md 8(d) generators G0/G1/G2 and a few
    byte patterns) -> the reference's bitshuffle output and bitshuffle+LZ4
    stream, stored whole for small cases and as SHA-256 digests for the
    BASELINE.json full-size configs (64 MiB int32 ramp, 4 GiB int16 G1,
    16 GiB float32 G2, 32 MiB G1 chunks of config 4), and for the element-size /
    block-size modes (MODES: G1 int16 bytes re-read as E = 3 / 12 elements, or
    framed with 256 KiB blocks -- bench.py's --elem-size / --block-size lines
    at 4 GiB, and the 1 GiB workload of tools/ab.py with AB_ELEM).
Inputs are regenerated from their counter-based definition at test time, so
only outputs are stored.  Run:  python tests/golden/make_vectors.py [--full]
"""
import argparse
import hashlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import Oracle, Reference  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
VEC = os.path.join(HERE, "vectors")


def sha(buf):
    return hashlib.sha256(memoryview(np.ascontiguousarray(buf)).cast("B")).hexdigest()


def make_input(o, spec):
    """Must match tests/vectors.py:make_input."""
    g, n, first, seed = spec["gen"], spec["n"], spec.get("first", 0), spec.get("seed", 12345)
    if g == "g0":
        a = o.gen_g0(n, first)
    elif g == "g1":
        a = o.gen_g1(n, first, seed)
    elif g == "g2":
        a = o.gen_g2(n, first, seed)
    elif g == "bytes_mod":
        a = (np.arange(n, dtype=np.int64) % spec["mod"]).astype(np.uint8)
    else:
        raise ValueError(g)
    if "view" in spec:
        a = a.view(np.uint8).view(np.dtype(spec["view"]))
    return a


SMALL = [
    # name, gen params, block size
    dict(name="g0_i32_64k", gen="g0", n=16384, bs=0),
    dict(name="g1_i16_256k", gen="g1", n=131072, bs=0),
    dict(name="g1_i16_odd", gen="g1", n=131072 - 13, bs=0),
    dict(name="g2_f32_256k", gen="g2", n=65536, bs=0),
    dict(name="g2_f32_bs680", gen="g2", n=65536 + 5, bs=680),
    dict(name="g1_i16_bs8", gen="g1", n=4096 + 3, bs=8),
    dict(name="g1_i16_bs64", gen="g1", n=32768 + 7, bs=64),
    dict(name="g1_E3", gen="g1", n=3 * 40000, view="V3", bs=0),
    dict(name="g1_E5", gen="g1", n=5 * 20000, view="V5", bs=0),
    dict(name="g1_E6", gen="g1", n=6 * 20000, view="V6", bs=0),
    dict(name="g1_E10", gen="g1", n=10 * 10000, view="V10", bs=0),
    dict(name="g1_E12", gen="g1", n=12 * 10000, view="V12", bs=0),
    dict(name="g1_E24", gen="g1", n=24 * 8000, view="V24", bs=0),
    dict(name="g2_E8", gen="g2", n=65536, view="u8", bs=0),
    dict(name="g2_E16", gen="g2", n=65536, view="V16", bs=0),
    # byU32 table path: bs*E >= 65547
    dict(name="g1_u32_E8_bs8200", gen="g1", n=4 * 16400 * 2, view="u8", bs=8200),
    dict(name="g2_u32_bs16400", gen="g2", n=16400 * 3 + 11, bs=16400),
    dict(name="bytes_mod251", gen="bytes_mod", mod=251, n=200000, bs=0),
    dict(name="bytes_mod3_E2", gen="bytes_mod", mod=3, n=100000, view="u2", bs=0),
]

FULL = [
    dict(name="cfg1_g0_i32_64MiB", gen="g0", n=1 << 24, bs=0, shuffle_only=True),
    dict(name="cfg2_g1_i16_4GiB", gen="g1", n=1 << 31, bs=0),
    dict(name="cfg3_g2_f32_16GiB", gen="g2", n=1 << 32, bs=0),
] + [dict(name="cfg4_g1_chunk%04d" % c, gen="g1", n=1 << 24, seed=12345 + c, bs=0)
     for c in (0, 1, 2, 3, 511, 1023)]


# G1 int16 (seed 12345) generated for n_i16 elements, its first `nbytes` bytes
# framed as `elem_size`-byte elements with block size `bs` (0 = default)
def _mode(name, n_i16, nbytes, E, bs):
    return dict(name=name, gen="g1", n=n_i16, nbytes=nbytes, elem_size=E, bs=bs)


MODES = [
    # tools/ab.py 1 GiB with AB_ELEM=E: x = int16[2**29] -> bytes[:(2**30 // E) * E]
    _mode("mode_ab_g1_1GiB_E3", 1 << 29, (1 << 30) // 3 * 3, 3, 0),
    _mode("mode_ab_g1_1GiB_E12", 1 << 29, (1 << 30) // 12 * 12, 12, 0),
    _mode("mode_g1_1GiB_E2_bs131072", 1 << 29, 1 << 30, 2, 131072),
    # bench.py --elem-size E / --block-size B at 4 GiB: n = 2**32 // E // 8 * 8
    _mode("mode_bench_g1_4GiB_E3", 1 << 31, (1 << 32) // 3 // 8 * 8 * 3, 3, 0),
    _mode("mode_bench_g1_4GiB_E12", 1 << 31, (1 << 32) // 12 // 8 * 8 * 12, 12, 0),
    _mode("mode_bench_g1_4GiB_E2_bs131072", 1 << 31, 1 << 32, 2, 131072),
]


def mode_input(o, spec):
    """The mode's input bytes viewed as its elements (must match
    tests/vectors.py:mode_input)."""
    raw = o.gen_g1(spec["n"], 0, spec.get("seed", 12345)).view(np.uint8)[: spec["nbytes"]]
    E = spec["elem_size"]
    return raw.view(np.dtype("V%d" % E)) if E != 2 else raw.view(np.int16)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--full", action="store_true", help="also compute full-size digests")
    ap.add_argument("--modes", action="store_true", help="also compute element/block-size mode digests")
    args = ap.parse_args()
    o, r = Oracle(), Reference()
    os.makedirs(VEC, exist_ok=True)
    out = {"small": [], "full": [], "modes": []}
    path = os.path.join(HERE, "vectors.json")
    if os.path.exists(path):
        old = json.load(open(path))
        for k, v in old.items():
            if k != "small":
                out[k] = v
    for spec in SMALL:
        a = make_input(o, spec)
        shuf = r.bitshuffle(a, spec["bs"])
        comp = r.compress_lz4(a, spec["bs"])
        assert o.compress_lz4(a, spec["bs"]).tobytes() == comp.tobytes(), spec["name"]
        fn = spec["name"] + ".lz4"
        comp.tofile(os.path.join(VEC, fn))
        e = dict(spec)
        e.update(dtype=a.dtype.str, elem_size=a.dtype.itemsize, size=int(a.size),
                 input_sha256=sha(a), shuffled_sha256=sha(shuf), compressed_file=fn,
                 compressed_len=int(comp.size), compressed_sha256=sha(comp))
        out["small"].append(e)
        print(e["name"], e["compressed_len"], flush=True)
    if args.full:
        out["full"] = []
        for spec in FULL:
            a = make_input(o, spec)
            e = dict(spec)
            e.update(dtype=a.dtype.str, elem_size=a.dtype.itemsize, size=int(a.size),
                     input_sha256=sha(a))
            if spec.get("shuffle_only"):
                e["shuffled_sha256"] = sha(r.bitshuffle(a, spec["bs"]))
            else:
                comp = r.compress_lz4(a, spec["bs"])
                e.update(compressed_len=int(comp.size), compressed_sha256=sha(comp))
                del comp
            del a
            out["full"].append(e)
            print(e["name"], e.get("compressed_len"), flush=True)
    if args.modes:
        out["modes"] = []
        for spec in MODES:
            a = mode_input(o, spec)
            comp = r.compress_lz4(a, spec["bs"])
            e = dict(spec)
            e.update(size=int(a.size), input_sha256=sha(a), compressed_len=int(comp.size),
                     compressed_sha256=sha(comp))
            # the 1 GiB cases: our oracle restatement must agree too
            if spec["nbytes"] <= (1 << 30):
                assert o.compress_lz4(a, spec["bs"]).tobytes() == comp.tobytes(), spec["name"]
            del comp, a
            out["modes"].append(e)
            print(e["name"], e["compressed_len"], flush=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
