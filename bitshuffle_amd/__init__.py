"""bitshuffle_amd -- MI355X-native bitshuffle + LZ4 (drop-in for kiyo-masui/bitshuffle).

Python mirror of the reference's module API (bitshuffle/__init__.py:24-35,
bitshuffle/ext.pyx:311-505): same function names, argument meaning and error
behaviour, backed by the HIP/gfx950 C-ABI library libbitshuffle_mi355x.so
(built in-tree by bitshuffle_amd/Makefile).  There is no CPU fallback: if the
library or a HIP device is missing, calls raise.

Host (numpy) functions
    bitshuffle(arr, block_size=0)            -> array, same shape/dtype
    bitunshuffle(arr, block_size=0)          -> array
    compress_lz4(arr, block_size=0)          -> uint8 array (framed stream)
    decompress_lz4(arr, shape, dtype, block_size=0) -> array
Device (torch CUDA/HIP tensor) functions, no host round trip
    bitshuffle_dev / bitunshuffle_dev / compress_lz4_dev / decompress_lz4_dev
    compress_lz4_batch_dev / decompress_lz4_batch_dev  (many streams per launch)
"""
from ._lib import (  # noqa: F401
    LIB_PATH,
    BshufError,
    lib,
    using_AVX2,
    using_AVX512,
    using_HIP,
    using_NEON,
    using_SSE2,
)
from .api import (  # noqa: F401
    bitshuffle,
    bitshuffle_dev,
    bitunshuffle,
    bitunshuffle_dev,
    compress_lz4,
    compress_lz4_batch_dev,
    compress_lz4_bound,
    compress_lz4_dev,
    decompress_lz4,
    decompress_lz4_batch_dev,
    decompress_lz4_dev,
    default_block_size,
    synth_fill_dev,
)

__version__ = "0.6.0"
__zstd__ = False

__all__ = [
    "__version__",
    "bitshuffle",
    "bitunshuffle",
    "using_NEON",
    "using_SSE2",
    "using_AVX2",
    "using_AVX512",
    "using_HIP",
    "compress_lz4",
    "decompress_lz4",
    "bitshuffle_dev",
    "bitunshuffle_dev",
    "compress_lz4_dev",
    "decompress_lz4_dev",
    "compress_lz4_batch_dev",
    "decompress_lz4_batch_dev",
]
