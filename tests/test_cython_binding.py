"""The reference's UNCHANGED Cython binding (bitshuffle/ext.pyx) builds against
libbitshuffle_mi355x.so and imports: every symbol its `cdef extern` blocks name
(ext.pyx:23-86, including the internal transpose hooks of :56-86) resolves in
this library.  THIS CONTAINER ONLY: the reference source is read from
/root/reference into a temporary directory (it never enters the repo and never
travels to the GPU box); skipped where it or Cython is absent."""
import os
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_PYX = "/root/reference/bitshuffle/ext.pyx"
LIBDIR = os.path.join(ROOT, "bitshuffle_amd")

SETUP = textwrap.dedent("""
    import numpy
    from Cython.Build import cythonize
    from setuptools import Extension, setup
    ext = Extension("ext", ["ext.pyx"],
                    include_dirs=[{inc!r}, numpy.get_include()],
                    library_dirs=[{lib!r}], libraries=["bitshuffle_mi355x"],
                    runtime_library_dirs=[{lib!r}])
    setup(name="ext", ext_modules=cythonize([ext], compile_time_env={{"ZSTD_SUPPORT": False}},
                                              language_level=3, quiet=True))
""")

PROBE = textwrap.dedent("""
    import numpy as np
    import ext
    print("version", ext.__version__)
    print("isa", ext.using_SSE2(), ext.using_AVX2(), ext.using_NEON())
    try:
        ext.bitshuffle(np.arange(64, dtype=np.int16))
        print("call ok")
    except RuntimeError as e:
        print("call error", e)
""")


@pytest.mark.skipif(not os.path.exists(REF_PYX), reason="reference source not in this container")
def test_reference_cython_ext_builds_and_imports(tmp_path):
    pytest.importorskip("Cython")
    lib = os.path.join(LIBDIR, "libbitshuffle_mi355x.so")
    assert os.path.exists(lib), "build the library first (make -C bitshuffle_amd)"
    (tmp_path / "ext.pyx").write_bytes(open(REF_PYX, "rb").read())
    (tmp_path / "setup.py").write_text(SETUP.format(inc=os.path.join(ROOT, "include"), lib=LIBDIR))
    r = subprocess.run([sys.executable, "setup.py", "build_ext", "--inplace"], cwd=tmp_path,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, BSHUF_STANDALONE_HIP="1")
    p = subprocess.run([sys.executable, "-c", PROBE], cwd=tmp_path, capture_output=True, text=True,
                       timeout=120, env=env)
    assert p.returncode == 0, p.stderr[-3000:]
    out = p.stdout
    assert "version 0.6.0" in out
    assert "isa False False False" in out
    # this container has no GPU: the call must fail loudly (-70), never fall
    # back to a CPU path; on an MI355X it succeeds
    assert ("call error" in out and "-70" in out) or "call ok" in out, out
