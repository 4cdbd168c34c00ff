"""Decoder time split from the diagnostic build's ablations (wrong output,
timing only): 0 full, 8 no inverse transpose/stores, 64 no sequence
execution, 72 neither, 1024 no literal copies, 2048 no match copies; then
k_lz4_decode's s_memtime phase split of a full decode (cycles per block,
summed over waves; the clock reads themselves add a little to every phase).
Usage: python tools/diag_decode.py [GiB] [gen] [variant]"""
import ctypes
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
if len(sys.argv) > 3:
    assert B.lib.bshuf_set_variant(int(sys.argv[3])) == 0
n = int(gib * (1 << 30)) // (2 if gen == 1 else 4)
x = torch.empty(n, dtype=torch.int16 if gen == 1 else torch.float32, device="cuda")
B.synth_fill_dev(x, gen)
c = api.compress_lz4_dev(x)
abl = B.lib.bshuf_diag_set_ablation
abl.argtypes = [ctypes.c_int]
for v in (0, 8, 64, 72, 1024, 2048, 0):
    abl(v)
    y, r = api.decompress_lz4_dev(c, x.shape, x.dtype, sync=False)
    torch.cuda.synchronize()
    B.lib.bshuf_prof_enable(1)
    bench.prof_collect(B.lib)
    for _ in range(3):
        y, r = api.decompress_lz4_dev(c, x.shape, x.dtype, sync=False)
    torch.cuda.synchronize()
    k = bench.prof_collect(B.lib)
    B.lib.bshuf_prof_enable(0)
    print("ablation %2d" % v, {name: round(ms / cnt, 3) for name, (cnt, ms) in k.items() if ms / cnt > 0.02})
abl(0)

rd = B.lib.bshuf_diag_read_dec
rd.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
buf = (ctypes.c_ulonglong * 16)()
rd(buf)
y, r = api.decompress_lz4_dev(c, x.shape, x.dtype, sync=False)
torch.cuda.synchronize()
rd(buf)
blocks = max(1, buf[8 + 3])
names = ["fields", "literals", "matches", "untranspose+store", "next record", "other"]
tot = sum(buf[i] for i in range(6))
for i, nm in enumerate(names):
    print("%-18s %8d cyc/block %5.1f%%" % (nm, buf[i] // blocks, 100.0 * buf[i] / max(1, tot)))
print("blocks %d  sequences/block %.1f  batches/block %.1f  coop matches/block %.1f" % (
    blocks, buf[8] / blocks, buf[9] / blocks, buf[10] / blocks))
