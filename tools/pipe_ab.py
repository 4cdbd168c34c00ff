"""Wall-clock A/B of whole compress / decompress calls (device-resident),
e.g. pipelined launches on and off: python tools/pipe_ab.py 1048576,0 [GiB] [gen] [reps]
(variant 1048576 = kNoPipe).  Streams are checked identical across variants."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402

variants = [int(v) for v in sys.argv[1].split(",")]
gib = float(sys.argv[2]) if len(sys.argv) > 2 else 4.0
gen = int(sys.argv[3]) if len(sys.argv) > 3 else 1
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 5
dt = torch.int16 if gen == 1 else torch.float32
n = int(gib * (1 << 30)) // (2 if gen == 1 else 4)
x = torch.empty(n, dtype=dt, device="cuda")
B.synth_fill_dev(x, gen)
es = x.element_size()
comp = torch.empty(B.compress_lz4_bound(n, es, 0), dtype=torch.uint8, device="cuda")
ws_e = api.compress_lz4_workspace(n, es, 0, device=x.device)
ws_d = api.decompress_lz4_workspace(comp.numel(), n, es, 0, device=x.device)
res = torch.empty(1, dtype=torch.int64, device="cuda")
y = torch.empty_like(x)
ref = None
out = {}
for rnd in range(3):
    for v in variants:
        assert B.lib.bshuf_set_variant(v) == 0
        api.compress_lz4_dev(x, out=comp, workspace=ws_e, result=res, sync=False)
        c = int(res.item())
        h = comp[:c].clone()
        if ref is None:
            ref = h
        assert torch.equal(h, ref), "variant %d stream differs" % v
        api.decompress_lz4_dev(comp[:c], x.shape, x.dtype, out=y, workspace=ws_d, result=res, sync=False)
        torch.cuda.synchronize()
        assert torch.equal(x, y), "variant %d round trip" % v
        t0 = time.perf_counter()
        for _ in range(reps):
            api.compress_lz4_dev(x, out=comp, workspace=ws_e, result=res, sync=False)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(reps):
            api.decompress_lz4_dev(comp[:c], x.shape, x.dtype, out=y, workspace=ws_d, result=res, sync=False)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        out.setdefault(v, []).append(((t1 - t0) / reps * 1e3, (t2 - t1) / reps * 1e3))
B.lib.bshuf_set_variant(0)
for v, xs in out.items():
    e = sorted(t[0] for t in xs)[len(xs) // 2]
    d = sorted(t[1] for t in xs)[len(xs) // 2]
    print("variant %8d  compress %.3f ms  decompress %.3f ms  round trip %.3f ms  (%.1f GiB/s)  rounds %s" % (
        v, e, d, e + d, gib / ((e + d) / 1e3), " ".join("%.2f/%.2f" % t for t in xs)), flush=True)
