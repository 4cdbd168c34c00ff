"""Run one device-resident compress (+ optionally decompress) of G1 data, for
profilers.  Usage: python tools/run_codec_once.py [GiB] [enc|dec|both]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
what = sys.argv[2] if len(sys.argv) > 2 else "both"
n = int(gib * (1 << 30)) // 2
x = torch.empty(n, dtype=torch.int16, device="cuda")
B.synth_fill_dev(x, 1)
c = api.compress_lz4_dev(x)
if what in ("dec", "both"):
    y = api.decompress_lz4_dev(c, x.shape, x.dtype)
    assert torch.equal(x, y)
torch.cuda.synchronize()
print("ok", c.numel())
