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


def _dump_chunks(exe, path, dset="data"):
    p = subprocess.Popen([exe, "chunks", path, dset], env=env(), stdout=subprocess.PIPE,
                         stderr=subprocess.PIPE)
    return p


@needs_hdf5
@pytest.mark.gpu
def test_config5_stored_chunks_match_oracle(tmp_path_factory, oracle):
    """BASELINE config 5 layout (uint16 = G1 + 32768 in 32 MiB chunks, filter
    opts (0, 2)) at 3 chunks: every chunk HDF5 stored through the plugin equals
    the reference filter's u64BE nbytes || u32BE block bytes ||
    bshuf_compress_lz4(chunk) (src/bshuf_h5filter.c:198-202), byte for byte."""
    import numpy as np
    exe = harness(tmp_path_factory)
    out = str(tmp_path_factory.mktemp("h5") / "cfg5s.h5")
    chunk, n = 1 << 24, 3 << 24
    r = subprocess.run([exe, "roundtrip", out, str(n), str(chunk)], env=env(), capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0 and '"match": true' in r.stdout, r.stdout + r.stderr
    p = _dump_chunks(exe, out)
    raw, err = p.communicate(timeout=300)
    assert p.returncode == 0, err
    pos = 0
    for first in range(0, n, chunk):
        a = oracle.gen_g1(chunk, first, 12345).view(np.uint16) ^ np.uint16(0x8000)
        want = (int(chunk * 2).to_bytes(8, "big") + int(4096 * 2).to_bytes(4, "big")
                + oracle.compress_lz4(a).tobytes())
        assert raw[pos:pos + len(want)] == want, first
        pos += len(want)
    assert pos == len(raw)


@needs_hdf5
@pytest.mark.gpu
@pytest.mark.slow
def test_config5_full_8GiB_digest(tmp_path_factory):
    """BASELINE config 5 at full size: 8 GiB uint16 written and read back
    through the plugin, and the SHA-256 of all 256 stored chunks equals the
    digest of the reference's own chunks (tests/golden/make_cfg5_digest.py)."""
    import hashlib
    import json
    from tests.vectors import load_vectors
    cfg = load_vectors()["cfg5"]
    exe = harness(tmp_path_factory)
    out = str(tmp_path_factory.mktemp("h5") / "cfg5.h5")
    r = subprocess.run([exe, "roundtrip", out, str(cfg["n"]), str(cfg["chunk_elem"])], env=env(),
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout + r.stderr
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["match"] is True and line["stored_bytes"] == cfg["stored_bytes"], line
    p = _dump_chunks(exe, out)
    h, total = hashlib.sha256(), 0
    while True:
        b = p.stdout.read(1 << 24)
        if not b:
            break
        h.update(b)
        total += len(b)
    assert p.wait(timeout=300) == 0
    assert total == cfg["stored_bytes"]
    assert h.hexdigest() == cfg["chunks_sha256"]
