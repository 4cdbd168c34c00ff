"""Caller-owned memory from a trimming stream-ordered pool.

DESIGN.md §4.2: in round 2 the host path produced wrong bytes when its
workspace came from ROCm's default stream-ordered pool, which hands freed
memory back to the OS at every synchronisation (release threshold 0) and maps
new memory at the next hipMallocAsync.  The library's own calls no longer use
that pool -- but a caller of the *_dev entry points may pass such memory for
`in`, `out` and `ws` (e.g. PyTorch with backend:hipMallocAsync), as the
HDF5 filter's buffers are caller-owned (reference src/bshuf_h5filter.c:171-234).

This test makes every call run on freshly mapped memory: in, out, ws, the
result word and the block offsets are hipMallocAsync'd from the device's
DEFAULT pool, freed with hipFreeAsync after the call, and the pool is trimmed
to zero (hipMemPoolTrimTo) before the next call.  Every stream is compared
with the oracle, every decode with the input.  Run once, deterministically.
"""
import ctypes

import numpy as np
import pytest

from tests.vectors import regression_cases

pytestmark = pytest.mark.gpu

H2D, D2H = 1, 2


@pytest.fixture(scope="module")
def hip():
    import torch  # noqa: F401  (torch's HIP runtime is the one the library binds)
    import bitshuffle_amd
    assert bitshuffle_amd.using_HIP()
    h = ctypes.CDLL("libamdhip64.so.7")
    vp, sz = ctypes.c_void_p, ctypes.c_size_t
    h.hipMallocAsync.argtypes = [ctypes.POINTER(vp), sz, vp]
    h.hipFreeAsync.argtypes = [vp, vp]
    h.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
    h.hipStreamCreate.argtypes = [ctypes.POINTER(vp)]
    h.hipStreamSynchronize.argtypes = [vp]
    h.hipDeviceGetDefaultMemPool.argtypes = [ctypes.POINTER(vp), ctypes.c_int]
    h.hipMemPoolTrimTo.argtypes = [vp, sz]
    return h


class PoolMem:
    """hipMallocAsync / hipFreeAsync from the default pool on one stream."""

    def __init__(self, hip):
        self.hip = hip
        self.s = ctypes.c_void_p()
        assert hip.hipStreamCreate(ctypes.byref(self.s)) == 0
        self.pool = ctypes.c_void_p()
        assert hip.hipDeviceGetDefaultMemPool(ctypes.byref(self.pool), 0) == 0
        self.live = []

    def alloc(self, n):
        p = ctypes.c_void_p()
        assert self.hip.hipMallocAsync(ctypes.byref(p), max(int(n), 1), self.s) == 0
        self.live.append(p)
        return p

    def put(self, arr):
        arr = np.ascontiguousarray(arr)
        p = self.alloc(arr.nbytes)
        assert self.hip.hipMemcpyAsync(p, arr.ctypes.data, arr.nbytes, H2D, self.s) == 0
        return p

    def get(self, p, n, dtype=np.uint8):
        out = np.empty(int(n) // np.dtype(dtype).itemsize, dtype=dtype)
        assert self.hip.hipMemcpyAsync(out.ctypes.data, p, out.nbytes, D2H, self.s) == 0
        assert self.hip.hipStreamSynchronize(self.s) == 0
        return out

    def release(self):
        """free everything, synchronise, return the pool's memory to the OS"""
        for p in self.live:
            assert self.hip.hipFreeAsync(p, self.s) == 0
        self.live = []
        assert self.hip.hipStreamSynchronize(self.s) == 0
        assert self.hip.hipMemPoolTrimTo(self.pool, 0) == 0


def test_dev_calls_on_freshly_mapped_pool_memory(hip, oracle):
    import bitshuffle_amd as B
    lib = B.lib
    m = PoolMem(hip)
    cases = [(arr, block) for _, _, arr, _, block in regression_cases()]
    cases += [(oracle.gen_g1(37 * 4096 + 1003, 0, 77), 0), (oracle.gen_g2(9 * 2048 + 5, 0, 78), 0),
              (oracle.gen_g1(5 * 4096 + 8, 0, 79).view(np.uint8), 64)]
    checked = 0
    for arr, block in cases:
        arr = np.ascontiguousarray(arr)
        n, E = arr.size, arr.dtype.itemsize
        want = oracle.compress_lz4(arr, block)
        nb = max(int(lib.bshuf_lz4_dev_nblocks(n, E, block)), 1)
        # encode, everything freshly mapped
        din = m.put(arr.view(np.uint8))
        bound = int(lib.bshuf_compress_lz4_bound(n, E, block))
        dout = m.alloc(bound)
        wsb = int(lib.bshuf_compress_lz4_dev_workspace(n, E, block))
        ws = m.alloc(wsb)
        res = m.alloc(8)
        offs = m.alloc(8 * nb)
        rc = lib.bshuf_compress_lz4_dev(din, dout, n, E, block, ws, wsb, res, offs, m.s)
        assert rc == 0, (n, E, block, rc)
        got_n = int(m.get(res, 8, np.int64)[0])
        assert got_n == want.size, ("encode length", n, E, block, got_n, want.size)
        got = m.get(dout, got_n)
        assert got.tobytes() == want.tobytes(), ("encode bytes", n, E, block)
        enc_offs = m.get(offs, 8 * nb, np.uint64)
        m.release()
        # decode (parallel index rebuild), everything freshly mapped
        for with_offs in (False, True):
            dc = m.put(want)
            dd = m.alloc(arr.nbytes)
            wsb = int(lib.bshuf_decompress_lz4_dev_workspace(want.size, n, E, block))
            ws = m.alloc(wsb)
            res = m.alloc(8)
            doffs = m.put(enc_offs) if with_offs else None
            rc = lib.bshuf_decompress_lz4_dev(dc, want.size, dd, n, E, block, ws, wsb, res, doffs, m.s)
            assert rc == 0, (n, E, block, rc)
            got_n = int(m.get(res, 8, np.int64)[0])
            assert got_n == want.size, ("decode consumed", n, E, block, with_offs, got_n)
            back = m.get(dd, arr.nbytes)
            assert back.tobytes() == arr.view(np.uint8).tobytes(), ("decode bytes", n, E, block, with_offs)
            m.release()
        checked += 1
    assert checked == len(cases) >= 45
