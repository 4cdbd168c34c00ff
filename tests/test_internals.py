"""The reference's internal transpose steps (include/bitshuffle_internals.h;
the symbols its Cython module links, bitshuffle/ext.pyx:56-86) on the GPU,
against the reference's own numpy definitions (tests/test_ext.py:672-716),
against the same-named functions of the compiled reference (oracle/_ref), and
composed as the reference composes them (src/bitshuffle_core.c:276-296,
369-387)."""
import ctypes

import numpy as np
import pytest

from tests.test_oracle import trans_bit_byte_np, trans_bit_elem_np, trans_byte_elem_np

pytestmark = pytest.mark.gpu

STEPS = ["bshuf_copy", "bshuf_trans_byte_elem_scal", "bshuf_trans_bit_byte_scal",
         "bshuf_trans_bitrow_eight", "bshuf_trans_bit_elem_scal", "bshuf_trans_byte_bitrow_scal",
         "bshuf_shuffle_bit_eightelem_scal", "bshuf_untrans_bit_elem_scal",
         "bshuf_trans_bit_elem", "bshuf_untrans_bit_elem"]


@pytest.fixture(scope="module")
def lib():
    import bitshuffle_amd
    assert bitshuffle_amd.using_HIP()
    return bitshuffle_amd.lib


def call(lib, name, arr):
    arr = np.ascontiguousarray(arr)
    out = np.empty_like(arr)
    r = getattr(lib, name)(arr.ctypes.data, out.ctypes.data, arr.size, arr.dtype.itemsize)
    return r, out.view(np.uint8).reshape(-1)


def dtypes():
    return [np.dtype(t) for t in (np.uint8, np.int16, np.int32, np.int64)] + \
        [np.dtype("V3"), np.dtype("V5"), np.dtype("V12"), np.dtype("V24")]


def test_internal_steps_known_answers(lib):
    rng = np.random.default_rng(3)
    for dt in dtypes():
        for n in (8, 64, 1024, 4096 + 8):
            a = rng.integers(0, 200, n * dt.itemsize, dtype=np.uint8).view(dt)
            r, got = call(lib, "bshuf_trans_byte_elem_scal", a)
            assert r == a.nbytes and got.tobytes() == trans_byte_elem_np(a).tobytes(), (dt, n)
            r, got = call(lib, "bshuf_trans_bit_byte_scal", a)
            assert r == a.nbytes and got.tobytes() == trans_bit_byte_np(a).tobytes(), (dt, n)
            for name in ("bshuf_trans_bit_elem", "bshuf_trans_bit_elem_scal"):
                r, got = call(lib, name, a)
                assert r == a.nbytes and got.tobytes() == trans_bit_elem_np(a).tobytes(), (dt, n)
            for name in ("bshuf_untrans_bit_elem", "bshuf_untrans_bit_elem_scal"):
                r, back = call(lib, name, got.view(dt))
                assert r == a.nbytes and back.tobytes() == a.tobytes(), (dt, n)
            r, cp = call(lib, "bshuf_copy", a)
            assert r == a.nbytes and cp.tobytes() == a.tobytes()


def test_internal_steps_compose_like_the_reference(lib):
    rng = np.random.default_rng(4)
    for dt in dtypes():
        a = rng.integers(0, 256, 2048 * dt.itemsize, dtype=np.uint8).view(dt)
        _, x = call(lib, "bshuf_trans_byte_elem_scal", a)
        _, y = call(lib, "bshuf_trans_bit_byte_scal", x.view(dt))
        _, z = call(lib, "bshuf_trans_bitrow_eight", y.view(dt))
        _, want = call(lib, "bshuf_trans_bit_elem", a)
        assert z.tobytes() == want.tobytes(), dt
        _, u = call(lib, "bshuf_trans_byte_bitrow_scal", want.view(dt))
        _, v = call(lib, "bshuf_shuffle_bit_eightelem_scal", u.view(dt))
        assert v.tobytes() == a.tobytes(), dt


def test_internal_steps_match_compiled_reference(lib):
    from oracle import Reference, reference_available
    if not reference_available():
        pytest.skip("oracle/_ref not built")
    ref = Reference().lib
    rng = np.random.default_rng(5)
    for name in STEPS:
        f = getattr(ref, name)
        f.restype = ctypes.c_int64
        f.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t]
        for dt in dtypes():
            for n in (16, 800, 4096):
                a = np.ascontiguousarray(rng.integers(0, 256, n * dt.itemsize, dtype=np.uint8).view(dt))
                want = np.empty_like(a)
                rw = f(a.ctypes.data, want.ctypes.data, a.size, dt.itemsize)
                rg, got = call(lib, name, a)
                assert rg == rw, (name, dt, n, rg, rw)
                assert got.tobytes() == want.view(np.uint8).tobytes(), (name, dt, n)
    # sizes that are not a multiple of 8: the same error / remainder handling
    for name in STEPS:
        f = getattr(ref, name)
        a = np.ascontiguousarray(rng.integers(0, 256, 13 * 3, dtype=np.uint8).view("V3"))
        want = np.zeros_like(a)
        rw = f(a.ctypes.data, want.ctypes.data, a.size, 3)
        rg, got = call(lib, name, a)
        assert rg == rw, (name, rg, rw)
        if rw >= 0:
            assert got.tobytes() == want.view(np.uint8).tobytes(), name


def test_cpu_simd_variants_report_missing_isa(lib):
    a = np.arange(64, dtype=np.uint16)
    for isa, code in (("SSE", -11), ("AVX", -12), ("NEON", -13), ("AVX512", -14)):
        from bitshuffle_amd._lib import PROTOTYPES
        names = [n for n in PROTOTYPES if n.endswith("_" + isa) and "_using_" not in n]
        assert names
        for n in names:
            r, _ = call(lib, n, a)
            assert r == code, (n, r)
