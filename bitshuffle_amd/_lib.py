"""Loader for libbitshuffle_mi355x.so and the C-ABI prototypes of include/*.h."""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("BSHUF_LIB") or os.path.join(HERE, "libbitshuffle_mi355x.so")
PLUGIN_PATH = os.path.join(HERE, "libh5bshuf_mi355x.so")

_vp = ctypes.c_void_p
_sz = ctypes.c_size_t
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_int = ctypes.c_int

# name -> (restype, argtypes); every symbol the headers in include/ declare.
PROTOTYPES = {
    # include/bitshuffle_core.h
    "bshuf_using_SSE2": (_int, []),
    "bshuf_using_NEON": (_int, []),
    "bshuf_using_AVX2": (_int, []),
    "bshuf_using_AVX512": (_int, []),
    "bshuf_using_HIP": (_int, []),
    "bshuf_default_block_size": (_sz, [_sz]),
    "bshuf_bitshuffle": (_i64, [_vp, _vp, _sz, _sz, _sz]),
    "bshuf_bitunshuffle": (_i64, [_vp, _vp, _sz, _sz, _sz]),
    "bshuf_bitshuffle_dev": (_i64, [_vp, _vp, _sz, _sz, _sz, _vp]),
    "bshuf_bitunshuffle_dev": (_i64, [_vp, _vp, _sz, _sz, _sz, _vp]),
    # include/bitshuffle.h
    "bshuf_compress_lz4_bound": (_sz, [_sz, _sz, _sz]),
    "bshuf_compress_lz4": (_i64, [_vp, _vp, _sz, _sz, _sz]),
    "bshuf_decompress_lz4": (_i64, [_vp, _vp, _sz, _sz, _sz]),
    "bshuf_compress_lz4_dev_workspace": (_sz, [_sz, _sz, _sz]),
    "bshuf_decompress_lz4_dev_workspace": (_sz, [_sz, _sz, _sz, _sz]),
    "bshuf_lz4_dev_nblocks": (_sz, [_sz, _sz, _sz]),
    "bshuf_compress_lz4_dev": (_i64, [_vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, _vp, _vp]),
    "bshuf_decompress_lz4_dev": (_i64, [_vp, _sz, _vp, _sz, _sz, _sz, _vp, _sz, _vp, _vp, _vp]),
    "bshuf_decompress_lz4_dev_dlen": (_i64, [_vp, _vp, _sz, _vp, _sz, _sz, _sz, _vp, _sz, _vp, _vp,
                                             _vp]),
    "bshuf_lz4_block_index_dev": (_i64, [_vp, _sz, _sz, _sz, _sz, _vp, _sz, _vp, _vp, _vp]),
    "bshuf_compress_lz4_batch_dev_workspace": (_sz, [_vp, _sz, _sz, _sz]),
    "bshuf_compress_lz4_batch_dev": (_i64, [_vp, _vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, _vp, _vp]),
    "bshuf_decompress_lz4_batch_dev_workspace": (_sz, [_vp, _vp, _sz, _sz, _sz]),
    "bshuf_decompress_lz4_batch_dev": (_i64, [_vp, _vp, _vp, _vp, _sz, _sz, _sz, _vp, _sz, _vp, _vp]),
    "bshuf_decompress_lz4_batch_dev_dlen": (_i64, [_vp, _vp, _vp, _vp, _vp, _sz, _sz, _sz, _vp, _sz,
                                                   _vp, _vp]),
    "bshuf_synth_fill_dev": (_i64, [_vp, _sz, _int, _u64, _u64, _vp]),
    "bshuf_prof_enable": (None, [_int]),
    "bshuf_prof_only": (None, [ctypes.c_char_p]),
    "bshuf_set_variant": (_int, [_int]),
    "bshuf_prof_collect": (_sz, [ctypes.c_char_p, _sz]),
    "bshuf_host_poison": (_i64, [_int]),
    # include/bitshuffle_internals.h (the reference's Cython hooks)
    **{n: (_i64, [_vp, _vp, _sz, _sz]) for n in (
        "bshuf_copy", "bshuf_trans_byte_elem_scal", "bshuf_trans_bit_byte_scal",
        "bshuf_trans_bitrow_eight", "bshuf_trans_bit_elem_scal", "bshuf_trans_byte_bitrow_scal",
        "bshuf_shuffle_bit_eightelem_scal", "bshuf_untrans_bit_elem_scal", "bshuf_trans_bit_elem",
        "bshuf_untrans_bit_elem")},
    **{"bshuf_%s_%s" % (f, isa): (_i64, [_vp, _vp, _sz, _sz])
       for isa, fs in (("SSE", ("trans_byte_elem", "trans_bit_byte", "trans_bit_elem",
                                 "trans_byte_bitrow", "shuffle_bit_eightelem", "untrans_bit_elem")),
                       ("NEON", ("trans_byte_elem", "trans_bit_byte", "trans_bit_elem",
                                  "trans_byte_bitrow", "shuffle_bit_eightelem", "untrans_bit_elem")),
                       ("AVX", ("trans_bit_byte", "trans_bit_elem", "trans_byte_bitrow",
                                 "shuffle_bit_eightelem", "untrans_bit_elem")),
                       ("AVX512", ("trans_bit_byte", "trans_bit_elem", "shuffle_bit_eightelem",
                                    "untrans_bit_elem")))
       for f in fs},
    "bshuf_host_xfer_stats": (None, [_vp]),
}


class BshufError(RuntimeError):
    """Raised with the library's negative error code as args[1]."""


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _share_torch_hip_runtime():
    """torch ships its own libamdhip64.so (SONAME libamdhip64.so.7, the same
    SONAME as /opt/rocm's).  Loading torch first makes the dynamic linker bind
    this library to that already-loaded runtime, so tensors allocated by torch
    and kernels launched here live in ONE HIP runtime (two runtimes in one
    process do not see each other's devices/allocations)."""
    if os.environ.get("BSHUF_STANDALONE_HIP"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def _load():
    _share_torch_hip_runtime()
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            "bitshuffle_amd: %s is missing -- build it with `make -C %s` "
            "(hipcc, gfx950). There is no CPU fallback." % (LIB_PATH, HERE))
    L = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in PROTOTYPES.items():
        f = getattr(L, name)
        f.restype = res
        f.argtypes = args
    return L


lib = _load()


def using_SSE2():
    return bool(lib.bshuf_using_SSE2())


def using_NEON():
    return bool(lib.bshuf_using_NEON())


def using_AVX2():
    return bool(lib.bshuf_using_AVX2())


def using_AVX512():
    return bool(lib.bshuf_using_AVX512())


def using_HIP():
    return bool(lib.bshuf_using_HIP())
