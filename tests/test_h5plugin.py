"""HDF5 filter-32008 plugin, driven through the real HDF5 C library with the
plugin loaded dynamically (HDF5_PLUGIN_PATH) -- the reference's
tests/test_h5filter.py / test_h5plugin.py / test_regression.py coverage,
without h5py (not installed here).  HDF5 1.10 comes from /opt/conda."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDF5 = "/opt/conda"
PLUGIN_DIR = os.path.join(ROOT, "bitshuffle_amd")
needs_hdf5 = pytest.mark.skipif(not os.path.exists(os.path.join(HDF5, "include", "hdf5.h")),
                                reason="HDF5 headers not available")


def harness(tmp_path_factory):
    exe = str(tmp_path_factory.mktemp("h5") / "h5_harness")
    subprocess.check_call(["gcc", "-O2", "-I", HDF5 + "/include", os.path.join(ROOT, "tests", "h5_harness.c"),
                           "-L", HDF5 + "/lib", "-lhdf5", "-Wl,-rpath," + HDF5 + "/lib", "-o", exe])
    return exe


def env():
    e = dict(os.environ)
    e["HDF5_PLUGIN_PATH"] = PLUGIN_DIR
    return e


@needs_hdf5
def test_harness_builds_and_plugin_present(tmp_path_factory):
    assert os.path.exists(os.path.join(PLUGIN_DIR, "libh5bshuf_mi355x.so"))
    assert os.path.exists(harness(tmp_path_factory))


@needs_hdf5
@pytest.mark.gpu
def test_regression_chunks_through_hdf5(tmp_path_factory):
    exe = harness(tmp_path_factory)
    out = str(tmp_path_factory.mktemp("h5") / "regress.h5")
    r = subprocess.run([exe, "regress", os.path.join(ROOT, "tests", "golden", "regression"), out],
                       env=env(), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "regress 42/42" in r.stdout


@needs_hdf5
@pytest.mark.gpu
def test_roundtrip_and_h5dump(tmp_path_factory):
    exe = harness(tmp_path_factory)
    out = str(tmp_path_factory.mktemp("h5") / "rt.h5")
    r = subprocess.run([exe, "roundtrip", out, str(3 * (1 << 20) + 777), str(1 << 20)], env=env(),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert '"match": true' in r.stdout
    # an external HDF5 tool decodes it through the plugin and exits cleanly
    # (reference tests/test_h5plugin.py:49-52; dlclose at exit must not crash)
    h5dump = os.path.join(HDF5, "bin", "h5dump")
    if os.path.exists(h5dump):
        for _ in range(3):
            d = subprocess.run([h5dump, "-d", "/data", "-s", "0", "-c", "8", out], env=env(),
                               capture_output=True, text=True, timeout=120)
            assert d.returncode == 0, d.stderr
            assert "DATA" in d.stdout
