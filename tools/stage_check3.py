import os, sys
sys.path.insert(0, os.getcwd())
import numpy as np
import bitshuffle_amd as B
from oracle import Oracle
o = Oracle()
arrs = [(o.gen_g1(1 << 24, k << 24).view(np.uint16) ^ np.uint16(0x8000)) for k in range(3)]
encs = [o.compress_lz4(a) for a in arrs]
for k in range(3):
    d = B.decompress_lz4(encs[k], arrs[k].shape, arrs[k].dtype)
    bad = np.nonzero(d != arrs[k])[0]
    print("dec-only", k, len(bad), bad[:5], flush=True)
for k in range(3):
    c = B.compress_lz4(arrs[k])
    print("enc", k, c.tobytes() == encs[k].tobytes(), flush=True)
for k in range(3):
    d = B.decompress_lz4(encs[k], arrs[k].shape, arrs[k].dtype)
    bad = np.nonzero(d != arrs[k])[0]
    print("dec", k, len(bad), bad[:5], (bad.max() if len(bad) else None), flush=True)
