"""TEST INFRASTRUCTURE ONLY -- ctypes access to the CPU oracle.

`Oracle` wraps oracle/liboracle.so (our from-scratch restatement of the
reference's hot path, oracle/bshuf_oracle.c) and `Reference` wraps
oracle/_ref/libbshuf_ref.so (the reference C compiled by oracle/Makefile from
/root/reference sources).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product package bitshuffle_amd
never does.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libbshuf_ref.so")
REF_SCALAR_SO = os.path.join(HERE, "_ref", "libbshuf_ref_scalar.so")

_c_void_p = ctypes.c_void_p
_c_size = ctypes.c_size_t
_c_i64 = ctypes.c_int64


def build():
    """Compile liboracle.so (and _ref/ when /root/reference is present)."""
    subprocess.check_call(["make", "-s", "-C", HERE])


def _ptr(a):
    return a.ctypes.data_as(_c_void_p)


class _Codec:
    """Common numpy-level API over a bshuf-style C library (prefix pfx)."""

    def __init__(self, path, pfx):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        self.lib = ctypes.CDLL(path)
        self.path = path
        for name in ("bitshuffle", "bitunshuffle", "compress_lz4", "decompress_lz4"):
            f = getattr(self.lib, pfx + name)
            f.restype = _c_i64
            f.argtypes = [_c_void_p, _c_void_p, _c_size, _c_size, _c_size]
            setattr(self, "_" + name, f)
        f = getattr(self.lib, pfx + "compress_lz4_bound")
        f.restype = _c_size
        f.argtypes = [_c_size, _c_size, _c_size]
        self._bound = f
        f = getattr(self.lib, pfx + "default_block_size")
        f.restype = _c_size
        f.argtypes = [_c_size]
        self._dbs = f

    def default_block_size(self, elem_size):
        return int(self._dbs(elem_size))

    def compress_lz4_bound(self, size, elem_size, block_size=0):
        return int(self._bound(size, elem_size, block_size))

    @staticmethod
    def _flat(arr):
        arr = np.ascontiguousarray(arr)
        return arr, arr.view(np.uint8).reshape(-1)

    def bitshuffle(self, arr, block_size=0):
        arr, flat = self._flat(arr)
        out = np.empty_like(arr)
        n = self._bitshuffle(_ptr(flat), _ptr(out), arr.size, arr.dtype.itemsize, block_size)
        if n < 0:
            raise RuntimeError("bitshuffle failed %d" % n, n)
        return out

    def bitunshuffle(self, arr, block_size=0):
        arr, flat = self._flat(arr)
        out = np.empty_like(arr)
        n = self._bitunshuffle(_ptr(flat), _ptr(out), arr.size, arr.dtype.itemsize, block_size)
        if n < 0:
            raise RuntimeError("bitunshuffle failed %d" % n, n)
        return out

    def compress_lz4(self, arr, block_size=0):
        arr, flat = self._flat(arr)
        bound = self.compress_lz4_bound(arr.size, arr.dtype.itemsize, block_size)
        out = np.empty(max(bound, 1), dtype=np.uint8)
        n = self._compress_lz4(_ptr(flat), _ptr(out), arr.size, arr.dtype.itemsize, block_size)
        if n < 0:
            raise RuntimeError("compress_lz4 failed %d" % n, n)
        return out[:n].copy()

    def decompress_lz4(self, buf, shape, dtype, block_size=0):
        dtype = np.dtype(dtype)
        buf = np.ascontiguousarray(buf, dtype=np.uint8)
        out = np.empty(shape, dtype=dtype)
        size = int(np.prod(shape))
        n = self._decompress_lz4(_ptr(buf), _ptr(out), size, dtype.itemsize, block_size)
        if n < 0:
            raise RuntimeError("decompress_lz4 failed %d" % n, n)
        if n != buf.size:
            raise RuntimeError("consumed %d of %d bytes" % (n, buf.size), n)
        return out


class Oracle(_Codec):
    """Our CPU restatement (bshuf_oracle.c)."""

    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            build()
        super().__init__(path, "orc_")
        L = self.lib
        L.orc_trans_bit_elem.argtypes = [_c_void_p, _c_void_p, _c_size, _c_size]
        L.orc_untrans_bit_elem.argtypes = [_c_void_p, _c_void_p, _c_size, _c_size]
        L.orc_lz4_compress_block.restype = ctypes.c_int
        L.orc_lz4_compress_block.argtypes = [_c_void_p, ctypes.c_int, _c_void_p]
        L.orc_lz4_decompress_block.restype = ctypes.c_int
        L.orc_lz4_decompress_block.argtypes = [_c_void_p, ctypes.c_int, _c_void_p, ctypes.c_int]
        for g in ("orc_gen_g1_i16", "orc_gen_g2_f32"):
            getattr(L, g).argtypes = [_c_void_p, _c_size, _c_size, ctypes.c_uint64]
        L.orc_gen_g0_ramp_i32.argtypes = [_c_void_p, _c_size, _c_size]

    def lz4_compress_block(self, data):
        data = np.ascontiguousarray(data, dtype=np.uint8)
        out = np.empty(data.size + data.size // 255 + 16, dtype=np.uint8)
        n = self.lib.orc_lz4_compress_block(_ptr(data), data.size, _ptr(out))
        return out[:n].copy()

    def lz4_decompress_block(self, comp, capacity):
        comp = np.ascontiguousarray(comp, dtype=np.uint8)
        out = np.empty(max(capacity, 1), dtype=np.uint8)
        n = self.lib.orc_lz4_decompress_block(_ptr(comp), comp.size, _ptr(out), capacity)
        if n < 0:
            raise RuntimeError("lz4 decode error %d" % n, n)
        return out[:n].copy()

    def gen_g0(self, n, first=0):
        out = np.empty(n, dtype=np.int32)
        self.lib.orc_gen_g0_ramp_i32(_ptr(out), n, first)
        return out

    def gen_g1(self, n, first=0, seed=12345):
        out = np.empty(n, dtype=np.int16)
        self.lib.orc_gen_g1_i16(_ptr(out), n, first, seed)
        return out

    def gen_g2(self, n, first=0, seed=12345):
        out = np.empty(n, dtype=np.float32)
        self.lib.orc_gen_g2_f32(_ptr(out), n, first, seed)
        return out


class Reference(_Codec):
    """The reference C (oracle/_ref), compiled from /root/reference sources."""

    def __init__(self, path=REF_SO):
        super().__init__(path, "bshuf_")
        self.lib.LZ4_decompress_safe.restype = ctypes.c_int
        self.lib.LZ4_decompress_safe.argtypes = [_c_void_p, _c_void_p, ctypes.c_int, ctypes.c_int]

    def lz4_decompress_block(self, comp, capacity):
        """LZ4 1.10.0's LZ4_decompress_safe (lz4/lz4.c:2451) on one raw block."""
        comp = np.ascontiguousarray(comp, dtype=np.uint8)
        out = np.empty(max(capacity, 1), dtype=np.uint8)
        n = self.lib.LZ4_decompress_safe(_ptr(comp), _ptr(out), comp.size, capacity)
        if n < 0:
            raise RuntimeError("lz4 decode error %d" % n, n)
        return out[:n].copy()


def reference_available(path=REF_SO):
    return os.path.exists(path)
