"""AddressSanitizer + UBSan runs of the CPU-side C and C++ (SURVEY.md 5:
sanitizers on the host paths), built by tests/asan/Makefile:

* the oracle's framed codec and transposes, and the host build of the GPU
  decoder's scan state machine (bitshuffle_amd/csrc/lz4_scan.h) on valid and
  corrupted exact-size records (tests/asan/asan_driver.cpp);
* the HDF5 filter-32008 source (bitshuffle_amd/csrc/h5filter.c) loaded by the
  real HDF5 library through HDF5_PLUGIN_PATH from an ASan-built harness,
  with the oracle serving the C-ABI (tests/asan/h5_oracle_backend.c): the
  reference's 42 regression chunks and a multi-chunk round trip.

No GPU: the GPU library itself is exercised by the -m gpu suite.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDF5 = "/opt/conda"

needs_gcc = pytest.mark.skipif(shutil.which("gcc") is None or shutil.which("g++") is None,
                               reason="no gcc/g++")


@pytest.fixture(scope="module")
def asan_dir(tmp_path_factory):
    out = str(tmp_path_factory.mktemp("asan"))
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "tests", "asan"), "OUT=" + out])
    return out


def _clean(r):
    text = r.stdout + r.stderr
    assert "AddressSanitizer" not in text and "runtime error" not in text, text[-4000:]
    assert r.returncode == 0, text[-4000:]
    return text


@needs_gcc
def test_asan_oracle_and_scan(asan_dir):
    r = subprocess.run([os.path.join(asan_dir, "asan_driver")], capture_output=True, text=True,
                       timeout=300, env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1"))
    text = _clean(r)
    assert ", 0 failures" in text


@needs_gcc
@pytest.mark.skipif(not os.path.exists(os.path.join(HDF5, "include", "hdf5.h")),
                    reason="HDF5 headers not available")
def test_asan_h5filter(asan_dir):
    exe = os.path.join(asan_dir, "h5_harness_asan")
    # libhdf5 itself is not instrumented and keeps global state until exit:
    # leak reports would be its, not the filter's
    env = dict(os.environ, HDF5_PLUGIN_PATH=os.path.join(asan_dir, "plug"),
               ASAN_OPTIONS="detect_leaks=0")
    r = subprocess.run([exe, "regress", os.path.join(ROOT, "tests", "golden", "regression"),
                        os.path.join(asan_dir, "regress.h5")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert "regress 42/42" in _clean(r)
    r = subprocess.run([exe, "roundtrip", os.path.join(asan_dir, "rt.h5"), str(3 * 65536 + 777),
                        str(65536)], capture_output=True, text=True, timeout=300, env=env)
    assert '"match": true' in _clean(r)
