"""Time kernel variants WITHOUT output checks (ablations produce wrong bytes).
Usage: python tools/ablate.py dec|enc 0,2,10,... [GiB] [gen]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402
import bench  # noqa: E402

what = sys.argv[1]
variants = [int(v) for v in sys.argv[2].split(",")]
gib = float(sys.argv[3]) if len(sys.argv) > 3 else 2.0
gen = int(sys.argv[4]) if len(sys.argv) > 4 else 1
dt = torch.int16 if gen == 1 else torch.float32
n = int(gib * (1 << 30)) // (2 if gen == 1 else 4)
x = torch.empty(n, dtype=dt, device="cuda")
B.synth_fill_dev(x, gen)
B.lib.bshuf_set_variant(0)
c = api.compress_lz4_dev(x)
offs = None
res = {}
for rnd in range(2):
    for v in variants:
        B.lib.bshuf_set_variant(v)
        B.lib.bshuf_prof_enable(1)
        bench.prof_collect(B.lib)
        for _ in range(3):
            if what == "dec":
                api.decompress_lz4_dev(c, x.shape, x.dtype, sync=False)
            else:
                api.compress_lz4_dev(x, sync=False)
        torch.cuda.synchronize()
        k = bench.prof_collect(B.lib)
        B.lib.bshuf_prof_enable(0)
        name = "k_lz4_decode" if what == "dec" else "k_lz4_encode"
        cnt, ms = k[name]
        res.setdefault(v, []).append(ms / cnt)
B.lib.bshuf_set_variant(0)
for v, xs in res.items():
    print("%s variant %3d  %8.3f ms" % (what, v, sum(xs) / len(xs)))
