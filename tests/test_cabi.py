"""CPU tests of the drop-in boundary: the HIP library loads, exports every
symbol include/*.h declares, and its host-only logic matches the reference.
No compute call is made without a GPU -- except to check that compute entry
points fail loudly (-70) instead of falling back to a CPU path."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(ROOT, "include")


def declared_symbols():
    names = set()
    for fn in os.listdir(INCLUDE):
        if not fn.endswith(".h"):
            continue
        src = open(os.path.join(INCLUDE, fn)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"//[^\n]*", "", src)
        for m in re.finditer(r"\b(bshuf_\w+|H5PLget_\w+)\s*\(", src):
            names.add(m.group(1))
        for m in re.finditer(r"extern\s+H5Z_class_t\s+(\w+)", src):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    import bitshuffle_amd
    from bitshuffle_amd._lib import PLUGIN_PATH, PROTOTYPES
    out = subprocess.check_output(["nm", "-D", "--defined-only", bitshuffle_amd.LIB_PATH]).decode()
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    if os.path.exists(PLUGIN_PATH):
        out = subprocess.check_output(["nm", "-D", "--defined-only", PLUGIN_PATH]).decode()
        exported |= set(l.split()[-1] for l in out.splitlines() if l.strip())
    want = declared_symbols()
    assert "bshuf_compress_lz4" in want and "bshuf_bitshuffle" in want
    missing = sorted(want - exported)
    assert not missing, missing
    # the ctypes prototype table covers the whole core ABI
    core = {n for n in want if n.startswith("bshuf_") and "h5" not in n.lower()}
    assert core <= set(PROTOTYPES), sorted(core - set(PROTOTYPES))


def test_host_logic_matches_reference(oracle):
    import bitshuffle_amd as B
    for e in [1, 2, 3, 4, 5, 8, 16, 63, 64, 65, 100, 1000]:
        assert B.default_block_size(e) == oracle.default_block_size(e)
    for size, e, bs in [(0, 2, 0), (100, 2, 0), (4096 * 3 + 77, 2, 0), (12345, 3, 64),
                        (10 ** 9, 4, 0), (2 ** 31, 2, 0), (1000, 8, 8200)]:
        assert B.compress_lz4_bound(size, e, bs) == oracle.compress_lz4_bound(size, e, bs)
    # reference quirk: bad block size -> (size_t)-81 (src/bitshuffle.c:222)
    assert B.lib.bshuf_compress_lz4_bound(100, 2, 12) == ctypes.c_size_t(-81).value


def test_isa_probes():
    import bitshuffle_amd as B
    assert not (B.using_SSE2() or B.using_AVX2() or B.using_AVX512() or B.using_NEON())


def test_bad_block_size_before_device():
    import bitshuffle_amd as B
    with pytest.raises(RuntimeError) as ei:
        B.bitshuffle(np.arange(64, dtype=np.int16), 12)
    assert ei.value.args[1] == -81


def test_no_cpu_fallback_without_gpu():
    import bitshuffle_amd as B
    if B.using_HIP():
        pytest.skip("HIP device present")
    for f in (B.bitshuffle, B.bitunshuffle, B.compress_lz4):
        with pytest.raises(RuntimeError) as ei:
            f(np.arange(1024, dtype=np.int16))
        assert ei.value.args[1] == -70


def test_one_block_hooks_limit_before_device():
    """bitshuffle_internals.h: the one-block bit-transpose hooks run the whole
    array as one block; above 2^30 bytes or elem_size 65536 they return -71
    before touching any memory (NULL pointers are never dereferenced)."""
    import bitshuffle_amd as B
    for name in ("bshuf_trans_bit_elem", "bshuf_trans_bit_elem_scal", "bshuf_untrans_bit_elem",
                 "bshuf_untrans_bit_elem_scal"):
        f = getattr(B.lib, name)
        assert f(None, None, 1 << 31, 1) == -71, name
        assert f(None, None, (1 << 30) // 4 + 8, 4) == -71, name
        assert f(None, None, 8, 65537) == -71, name
        assert f(None, None, 9, 1) == -80, name
    assert B.lib.bshuf_trans_bit_byte_scal(None, None, 1 << 31, 1) == -71
