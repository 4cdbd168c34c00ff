"""Occupancy sweep of the LZ4 kernels (diagnostic build): the LDS request is
padded so that at most w waves fit a CU (BSHUF_DIAG_WAVES / _DEC_WAVES), and
each kernel is timed at every w.  Shows whether a kernel's time follows its
resident waves (latency-bound per wave) or not (a shared unit bounds it).
Usage: python tools/occ_sweep.py [GiB] [gen] [w1,w2,...]  (on the GPU box)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("BSHUF_LIB", os.path.join(ROOT, "bitshuffle_amd", "libbitshuffle_mi355x_diag.so"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402
import bench  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
gen = int(sys.argv[2]) if len(sys.argv) > 2 else 1
ws = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "0,6,5,4,3,2").split(",")]
n = int(gib * (1 << 30)) // (2 if gen == 1 else 4)
x = torch.empty(n, dtype=torch.int16 if gen == 1 else torch.float32, device="cuda")
B.synth_fill_dev(x, gen)
c = api.compress_lz4_dev(x)
for w in ws:
    for k in ("BSHUF_DIAG_WAVES", "BSHUF_DIAG_DEC_WAVES"):
        if w:
            os.environ[k] = str(w)
        else:
            os.environ.pop(k, None)
    c = api.compress_lz4_dev(x)
    y, r = api.decompress_lz4_dev(c, x.shape, x.dtype, sync=False)
    torch.cuda.synchronize()
    B.lib.bshuf_prof_enable(1)
    bench.prof_collect(B.lib)
    for _ in range(3):
        c = api.compress_lz4_dev(x)
        y, r = api.decompress_lz4_dev(c, x.shape, x.dtype, sync=False)
    torch.cuda.synchronize()
    k = bench.prof_collect(B.lib)
    B.lib.bshuf_prof_enable(0)
    assert torch.equal(x, y)
    print("waves %d" % w, {name: round(ms / cnt, 3) for name, (cnt, ms) in k.items()
                           if name in ("k_lz4_encode", "k_lz4_decode")}, flush=True)
