"""Golden fixtures: the reference's regression chunks and the reference-made
vectors of tests/golden/vectors.json (see tests/golden/make_vectors.py)."""
import hashlib
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def sha(buf):
    return hashlib.sha256(memoryview(np.ascontiguousarray(buf)).cast("B")).hexdigest()


def regression_cases():
    """(version, name, original array, stored chunk bytes, block_size) for the 42
    LZ4 datasets of tests/data/regression_{0.1.3,0.4.0}.h5."""
    d = os.path.join(GOLDEN, "regression")
    out = []
    for line in open(os.path.join(d, "MANIFEST")):
        f = line.split()
        ver, name, E, n = f[0], f[1], int(f[2]), int(f[3])
        orig = np.fromfile(os.path.join(d, "%s__%s.orig" % (ver, name)), dtype=np.uint8)
        chunk = np.fromfile(os.path.join(d, "%s__%s.chunk" % (ver, name)), dtype=np.uint8)
        bsb = int.from_bytes(chunk[8:12].tobytes(), "big")
        arr = orig.view(np.dtype("V%d" % E)) if E > 1 else orig.copy()
        assert arr.size == n
        out.append((ver, name, arr, chunk, bsb // E))
    return out


def load_vectors():
    return json.load(open(os.path.join(GOLDEN, "vectors.json")))


def make_input(o, spec):
    """Regenerate a vector's input from its counter-based definition
    (identical to tests/golden/make_vectors.py:make_input)."""
    g, n, first, seed = spec["gen"], spec["n"], spec.get("first", 0), spec.get("seed", 12345)
    if g == "g0":
        a = o.gen_g0(n, first)
    elif g == "g1":
        a = o.gen_g1(n, first, seed)
    elif g == "g2":
        a = o.gen_g2(n, first, seed)
    elif g == "bytes_mod":
        a = (np.arange(n, dtype=np.int64) % spec["mod"]).astype(np.uint8)
    else:
        raise ValueError(g)
    if "view" in spec:
        a = a.view(np.uint8).view(np.dtype(spec["view"]))
    return a


def compressed(spec):
    return np.fromfile(os.path.join(GOLDEN, "vectors", spec["compressed_file"]), dtype=np.uint8)
