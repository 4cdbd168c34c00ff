"""One timing sample of the codec library named by BSHUF_LIB (or the default):
python tools/ab_one.py GiB gen reps -> one JSON line {kernel: avg ms, ..., "sha": stream digest}.
tools/ab_libs.sh alternates libraries over fresh processes with it."""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402
import bench  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
gen = int(sys.argv[2]) if len(sys.argv) > 2 else 1
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
dt = torch.int16 if gen == 1 else torch.float32
n = int(gib * (1 << 30)) // (2 if gen == 1 else 4)
x = torch.empty(n, dtype=dt, device="cuda")
B.synth_fill_dev(x, gen)
# AB_ELEM=E: the same bytes as E-byte elements (odd element sizes)
es = int(os.environ.get("AB_ELEM", "0"))
if es:
    x = x.view(torch.uint8)[: (x.numel() * x.element_size() // es) * es]
kw = {"elem_size": es} if es else {}
# AB_BS=elements: explicit block size (e.g. 131072 for 256 KiB int16 blocks)
if int(os.environ.get("AB_BS", "0")):
    kw["block_size"] = int(os.environ["AB_BS"])
shape = (x.numel() // es,) if es else x.shape
c = api.compress_lz4_dev(x, **kw)
y = api.decompress_lz4_dev(c, shape, x.dtype, **kw)
torch.cuda.synchronize()
assert torch.equal(x.view(torch.uint8), y.view(torch.uint8))
h = hashlib.sha256(c.cpu().numpy().tobytes()).hexdigest()[:16]
B.lib.bshuf_prof_enable(1)
bench.prof_collect(B.lib)
for _ in range(reps):
    c = api.compress_lz4_dev(x, **kw)
    y = api.decompress_lz4_dev(c, shape, x.dtype, **kw)
torch.cuda.synchronize()
k = bench.prof_collect(B.lib)
out = {name: round(ms / cnt, 4) for name, (cnt, ms) in k.items() if ms / cnt > 0.02}
out["sha"] = h
out["lib"] = os.path.basename(os.environ.get("BSHUF_LIB", "default"))
print(json.dumps(out), flush=True)
