"""Phase split of k_lz4_encode from the diagnostic build (BSHUF_DIAG stamps).
Usage: python tools/diag_encode.py [GiB] [gen] [elem_size]   (runs on the GPU box)"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["BSHUF_LIB"] = os.path.join(ROOT, "bitshuffle_amd", "libbitshuffle_mi355x_diag.so")
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
gen = int(sys.argv[2]) if len(sys.argv) > 2 else 1
es = int(sys.argv[3]) if len(sys.argv) > 3 else 0  # element size override (the same bytes)
n = int(gib * (1 << 30)) // (2 if gen == 1 else 4)
x = torch.empty(n, dtype=torch.int16 if gen == 1 else torch.float32, device="cuda")
B.synth_fill_dev(x, gen)
if es:
    x = x.view(torch.uint8)[: (x.numel() * x.element_size() // es) * es]
rd = B.lib.bshuf_diag_read
rd.argtypes = [ctypes.c_void_p]
buf = (ctypes.c_ulonglong * 32)()
c = api.compress_lz4_dev(x, elem_size=es or None)
torch.cuda.synchronize()
rd(buf)  # reset after warm-up
B.lib.bshuf_prof_enable(1)
c = api.compress_lz4_dev(x, elem_size=es or None)
torch.cuda.synchronize()
rd(buf)
import bench  # noqa: E402
prof = bench.prof_collect(B.lib)
v = list(buf)
names = ["search", "catch+count", "(unused)", "seq-record", "retest", "last"]
cnt = ["matches", "windows", "collision_windows", "retest_hits", "blocks", "literal_bytes",
       "searches"]
blocks = max(v[12], 1)
tot = sum(v[:6])
print("blocks", blocks, "ratio", x.numel() * x.element_size() / c.numel())
for i, nm in enumerate(names):
    print("%-12s %8.0f cyc/block  %5.1f%%" % (nm, v[i] / blocks, 100.0 * v[i] / max(tot, 1)))
print("parse cycles/block %.0f" % (tot / blocks))
kn = ["zero+transpose", "parse", "emit+copy-out", "loop/other"]
ktot = sum(v[16:20])
for i, nm in enumerate(kn):
    print("kernel %-15s %8.0f cyc/block  %5.1f%%" % (nm, v[16 + i] / blocks, 100.0 * v[16 + i] / max(ktot, 1)))
for i, nm in enumerate(cnt):
    print("%-18s %8.2f per block" % (nm, v[8 + i] / blocks))
print("kernel ms", {k: round(t / c_, 3) for k, (c_, t) in prof.items()})
