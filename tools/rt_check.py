import os, sys; sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bitshuffle_amd as b, torch, numpy as np
print("HIP", b.using_HIP(), "torch", torch.cuda.is_available())
x = torch.arange(100000, dtype=torch.int16, device="cuda")
c = b.compress_lz4_dev(x)
d = b.decompress_lz4_dev(c.clone(), x.shape, x.dtype)
print("dev roundtrip", torch.equal(d, x), c.numel())
a = np.arange(100000, dtype=np.int16)
print("host match", b.compress_lz4(a).tobytes() == c.cpu().numpy().tobytes())
