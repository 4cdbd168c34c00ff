"""CPU checks of the two-phase decoder's logic (no GPU needed):

* the host build of the scan state machine the GPU runs
  (bitshuffle_amd/csrc/lz4_scan.h via libbshuf_hostcheck.so) accepts and
  rejects exactly what the oracle's LZ4_decompress_safe restatement does, with
  the same error position and decoded length;
* the lane model of phase 2 (tests/exec_model.py) rebuilds every accepted
  block byte for byte from the scan's token positions.
"""
import ctypes
import os

import numpy as np
import pytest

from tests.exec_model import exec_block
from tests.test_oracle import corrupt_lz4_blocks

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTCHECK = os.path.join(ROOT, "bitshuffle_amd", "libbshuf_hostcheck.so")


@pytest.fixture(scope="module")
def scan():
    if not os.path.exists(HOSTCHECK):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "bitshuffle_amd"),
                               HOSTCHECK])
    lib = ctypes.CDLL(HOSTCHECK)
    fn = lib.bshuf_hostcheck_scan
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p,
                   ctypes.POINTER(ctypes.c_int)]

    def run(comp, n):
        comp = np.ascontiguousarray(comp, dtype=np.uint8)
        pos = np.zeros(comp.size // 3 + 2, dtype=np.uint32)
        cnt = ctypes.c_int(0)
        r = fn(comp.ctypes.data, comp.size, n, pos.ctypes.data, ctypes.byref(cnt))
        return r, pos[:cnt.value].copy()
    return run


def _oracle(oracle, comp, n):
    try:
        return "ok", oracle.lz4_decompress_block(comp, n)
    except RuntimeError as e:
        return "err", e.args[1]


def _blocks(oracle):
    """Valid blocks of the benchmark generators (bit-shuffled G1/G2 planes:
    long literal runs, long matches, many short sequences) and odd data."""
    out = []
    for arr in [oracle.gen_g1(4096 * 6), oracle.gen_g2(2048 * 6)]:
        sh = oracle.bitshuffle(arr).view(np.uint8)
        out += [sh[i:i + 8192] for i in range(0, sh.size, 8192)]
    rng = np.random.default_rng(3)
    for n in [64, 100, 777, 4096, 8192]:
        out.append((np.arange(n) % 3).astype(np.uint8))
        out.append(np.repeat(rng.integers(0, 256, n // 40 + 1), 40)[:n].astype(np.uint8))
        out.append((np.arange(n) * 7 % 251).astype(np.uint8))
    return out


def test_scan_and_exec_model_rebuild_valid_blocks(oracle, scan):
    for d in _blocks(oracle):
        comp = oracle.lz4_compress_block(d)
        r, pos = scan(comp, d.size)
        assert r == d.size
        assert exec_block(comp, pos, d.size).tobytes() == d.tobytes()


def test_scan_matches_oracle_on_corrupt_blocks(oracle, scan):
    checked = accepted = 0
    for comp, cap in corrupt_lz4_blocks(oracle, seed=31, per_base=25):
        if cap == 0:
            continue
        want = _oracle(oracle, comp, cap)
        r, pos = scan(comp, cap)
        if want[0] == "err":
            assert r == want[1], (comp.size, cap, r, want[1])
        else:
            assert r == want[1].size, (comp.size, cap, r, want[1].size)
            if r == cap:  # the GPU executes only blocks that decode to exactly n bytes
                assert exec_block(comp, pos, cap).tobytes() == want[1].tobytes()
                accepted += 1
        checked += 1
    assert checked > 1000 and accepted > 50
