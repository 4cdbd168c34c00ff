"""A/B kernel variants in one process: python tools/ab.py 0,1 [GiB] [gen] [reps]
Every variant must produce byte-identical streams (checked against variant 0)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402
import bench  # noqa: E402

variants = [int(v) for v in sys.argv[1].split(",")]
gib = float(sys.argv[2]) if len(sys.argv) > 2 else 2.0
gen = int(sys.argv[3]) if len(sys.argv) > 3 else 1
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 3
dt = torch.int16 if gen == 1 else torch.float32
n = int(gib * (1 << 30)) // (2 if gen == 1 else 4)
x = torch.empty(n, dtype=dt, device="cuda")
B.synth_fill_dev(x, gen)
# AB_ELEM=E: the same bytes as E-byte elements (odd element sizes)
es = int(os.environ.get("AB_ELEM", "0"))
if es:
    x = x.view(torch.uint8)[: (x.numel() * x.element_size() // es) * es]
kw = {"elem_size": es} if es else {}
shape = (x.numel() // es,) if es else x.shape
ref = None
res = {}
for rnd in range(2):  # interleave rounds to average out clock drift
    for v in variants:
        B.lib.bshuf_set_variant(v)
        c = api.compress_lz4_dev(x, **kw)
        y = api.decompress_lz4_dev(c, shape, x.dtype, **kw)
        torch.cuda.synchronize()
        if ref is None:
            ref = c.clone()
        assert c.numel() == ref.numel() and torch.equal(c, ref), "variant %d differs" % v
        assert torch.equal(x.view(torch.uint8), y.view(torch.uint8)), "variant %d round trip" % v
        B.lib.bshuf_prof_enable(1)
        bench.prof_collect(B.lib)
        for _ in range(reps):
            c = api.compress_lz4_dev(x, **kw)
            y = api.decompress_lz4_dev(c, shape, x.dtype, **kw)
        torch.cuda.synchronize()
        k = bench.prof_collect(B.lib)
        B.lib.bshuf_prof_enable(0)
        for name, (cnt, ms) in k.items():
            res.setdefault((v, name), []).append(ms / cnt)
B.lib.bshuf_set_variant(0)
for (v, name), xs in sorted(res.items()):
    if xs and max(xs) > 0.05:
        print("variant %d %-20s %8.3f ms (rounds: %s)" % (v, name, sum(xs) / len(xs),
                                                       " ".join("%.3f" % t for t in xs)))
