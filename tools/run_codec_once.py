"""Run one device-resident compress (+ optionally decompress) of synthetic
data, for profilers.  Usage:
    python tools/run_codec_once.py [GiB] [enc|dec|both] [gen]
gen 1 (default) = int16 G1 (config 2's data, seed 12345), 2 = float32 G2
(config 3's data), 8 = uniformly random int16 (every block all-miss: only
search windows), 9 = zeros (one search, one block-long match).  BSHUF_VARIANT=v selects a byte-identical A/B variant."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bitshuffle_amd as B  # noqa: E402
from bitshuffle_amd import api  # noqa: E402

gib = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
what = sys.argv[2] if len(sys.argv) > 2 else "both"
gen = int(sys.argv[3]) if len(sys.argv) > 3 else 1
dt = torch.float32 if gen == 2 else torch.int16
n = int(gib * (1 << 30)) // torch.empty(0, dtype=dt).element_size()
if os.environ.get("BSHUF_VARIANT"):  # byte-identical A/B variant (bshuf_set_variant)
    assert B.lib.bshuf_set_variant(int(os.environ["BSHUF_VARIANT"])) == 0
x = torch.empty(n, dtype=dt, device="cuda")
if gen == 8:
    x.copy_(torch.randint(-32768, 32767, (n,), dtype=torch.int16,
                          generator=torch.Generator().manual_seed(7)).to("cuda"))
elif gen == 9:
    x.zero_()
else:
    B.synth_fill_dev(x, gen)
c = api.compress_lz4_dev(x)
if what in ("dec", "both"):
    y = api.decompress_lz4_dev(c, x.shape, x.dtype)
    assert torch.equal(x.view(torch.uint8), y.view(torch.uint8))
torch.cuda.synchronize()
print("ok", c.numel())
