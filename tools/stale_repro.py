"""Host-path stale-result experiment.

Runs the host-pointer drop-in API (bshuf_compress_lz4 / bshuf_decompress_lz4)
in many FRESH processes per transport mode and counts wrong results:
  * the reference's 42 LZ4 regression chunks (tests/golden/regression):
    decode == original and re-encode == stored bytes, PASSES times per process;
  * three 32 MiB int16 G1 chunks (different seeds, so every call's buffers hold
    the previous call's different bytes): encode must give the same bytes on
    every pass and decode must give the original.
Modes (BSHUF_HOST_XFER): kernel (default transport: k_xfer through pinned
fine-grained memory), dma (hipMemcpyAsync to/from the per-thread device
buffers, no cache maintenance), dma_fenced (dma + the round-2 256-workgroup
system-scope release/acquire kernel around every copy).

The switches exist in the DIAGNOSTIC library only: run with
BSHUF_LIB=bitshuffle_amd/libbitshuffle_mi355x_diag.so (make -C bitshuffle_amd diag).

usage: python tools/stale_repro.py [--procs N] [--passes P] mode [mode ...]
"""
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def g1(n, first, seed=12345):
    """int16 (tri>>3) - 2048 + (h & 31) - 16."""
    i = np.arange(first, first + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    p = (i % np.uint64(65536)).astype(np.int64)
    tri = np.where(p < 32768, p, 65536 - p)
    return ((tri >> 3) - 2048 + (z & np.uint64(31)).astype(np.int64) - 16).astype(np.int16)


def worker(passes):
    os.environ["BSHUF_STANDALONE_HIP"] = "1"
    import bitshuffle_amd as B
    from tests.vectors import regression_cases
    cases = regression_cases()
    big = [g1(1 << 24, k << 24, 12345 + k) for k in range(3)]
    bad = {"reg_dec": 0, "reg_enc": 0, "big_dec": 0, "big_enc": 0, "errors": 0}
    first = [None] * 3
    t0 = time.time()
    for _ in range(passes):
        for ver, name, arr, chunk, block in cases:
            stream = chunk[12:]
            try:
                if B.decompress_lz4(stream, arr.shape, arr.dtype, block).tobytes() != arr.tobytes():
                    bad["reg_dec"] += 1
                if B.compress_lz4(arr, block).tobytes() != stream.tobytes():
                    bad["reg_enc"] += 1
            except RuntimeError:
                bad["errors"] += 1
        for k, a in enumerate(big):
            try:
                c = B.compress_lz4(a).tobytes()
                if first[k] is None:
                    first[k] = c
                elif c != first[k]:
                    bad["big_enc"] += 1
                d = B.decompress_lz4(np.frombuffer(first[k], dtype=np.uint8), a.shape, a.dtype)
                if d.tobytes() != a.tobytes():
                    bad["big_dec"] += 1
            except RuntimeError:
                bad["errors"] += 1
    st = (np.zeros(2, dtype=np.uint64))
    B.lib.bshuf_host_xfer_stats(st.ctypes.data)
    bad["pieces"], bad["late_flags"] = int(st[0]), int(st[1])
    bad["seconds"] = round(time.time() - t0, 2)
    print(json.dumps(bad), flush=True)


def main():
    args = sys.argv[1:]
    if args and args[0] == "worker":
        worker(int(args[1]))
        return
    procs, passes, modes = 10, 3, []
    while args:
        a = args.pop(0)
        if a == "--procs":
            procs = int(args.pop(0))
        elif a == "--passes":
            passes = int(args.pop(0))
        else:
            modes.append(a)
    summary = {}
    for mode in modes or ["kernel"]:
        env = dict(os.environ, BSHUF_HOST_XFER=mode)
        tot = {}
        for t in range(procs):
            r = subprocess.run([sys.executable, os.path.abspath(__file__), "worker", str(passes)],
                               env=env, capture_output=True, text=True, timeout=300)
            line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else "{}"
            try:
                d = json.loads(line)
            except ValueError:
                d = {"crash": 1}
            if r.returncode:
                d["crash"] = d.get("crash", 0) + 1
            wrong = sum(d.get(k, 0) for k in ("reg_dec", "reg_enc", "big_dec", "big_enc"))
            d["procs_with_wrong"] = 1 if wrong else 0
            for k, v in d.items():
                tot[k] = round(tot.get(k, 0) + v, 2)
            print(mode, t, json.dumps(d), flush=True)
        tot["procs"] = procs
        tot["calls_per_proc"] = passes * (2 * 42 + 6)
        summary[mode] = tot
        print("SUMMARY", mode, json.dumps(tot), flush=True)
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
