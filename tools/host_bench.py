"""End-to-end rate of the drop-in host-pointer C-ABI (bshuf_compress_lz4 /
bshuf_decompress_lz4 / bshuf_bitshuffle on host buffers: H2D + kernels + D2H),
i.e. what an HDF5 filter callback or a numpy caller sees.
Usage: python tools/host_bench.py [GiB] [reps]   (GPU box)"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
n = int(gib * (1 << 30)) // 2
x = torch.empty(n, dtype=torch.int16, device="cuda")
B.synth_fill_dev(x, 1)
a = x.cpu().numpy()           # pageable host input
nbytes = a.nbytes
bound = B.compress_lz4_bound(n, 2)
comp = np.empty(bound, dtype=np.uint8)
out = np.empty_like(a)
shuf = np.empty_like(a)
res = {}
for name, fn in [
    ("compress_lz4", lambda: B.compress_lz4(a, out=comp)),
    ("decompress_lz4", lambda: B.decompress_lz4(res["_c"], a.shape, a.dtype, out=out)),
    ("bitshuffle", lambda: B.bitshuffle(a, out=shuf)),
]:
    best = None
    for r in range(reps + 1):
        t0 = time.perf_counter()
        v = fn()
        dt = time.perf_counter() - t0
        if name == "compress_lz4":
            res["_c"] = v.copy() if r == 0 else res["_c"]
        if r:
            best = dt if best is None else min(best, dt)
    res[name] = round(nbytes / best / (1 << 30), 3)
assert np.array_equal(out, a)
c = res.pop("_c")
print(json.dumps({"host_path_GiBps": res, "bytes": nbytes, "compressed": int(c.size),
                  "note": "host (pageable numpy) buffers in and out; GiB/s of uncompressed bytes, "
                          "best of %d" % reps}))
