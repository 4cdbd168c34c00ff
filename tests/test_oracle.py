"""CPU tests: the oracle against the reference's golden vectors, and the
lane-vectorised model of the HIP encoder against the oracle."""
import os

import numpy as np
import pytest

from tests.vectors import compressed, load_vectors, make_input, regression_cases, sha


# Known-answer definitions restated from the reference's tests
# (tests/test_ext.py:672-716): pure numpy, LSB-first bit numbering.
def trans_byte_elem_np(arr):
    itemsize = arr.dtype.itemsize
    b = arr.view(np.uint8).reshape(-1, itemsize)
    return np.ascontiguousarray(b.T).reshape(-1)


def trans_bit_byte_np(arr):
    bits = np.unpackbits(arr.view(np.uint8)).reshape(-1, 8)[:, ::-1]
    return np.packbits(np.ascontiguousarray(bits.T).reshape(-1, 8)[:, ::-1].reshape(-1))


def trans_bit_elem_np(arr):
    n, itemsize = arr.size, arr.dtype.itemsize
    bits = np.unpackbits(arr.view(np.uint8)).reshape(-1, 8)[:, ::-1].reshape(n, itemsize * 8)
    out = np.ascontiguousarray(bits.T).reshape(-1, 8)[:, ::-1]
    return np.packbits(out.reshape(-1))


def test_regression_chunks(oracle):
    cases = regression_cases()
    assert len(cases) == 42
    for ver, name, arr, chunk, block in cases:
        assert int.from_bytes(chunk[:8].tobytes(), "big") == arr.nbytes
        stream = chunk[12:]
        assert oracle.compress_lz4(arr, block).tobytes() == stream.tobytes(), (ver, name)
        assert oracle.decompress_lz4(stream, arr.shape, arr.dtype, block).tobytes() == \
            arr.tobytes(), (ver, name)


def test_golden_vectors(oracle):
    v = load_vectors()
    assert len(v["small"]) >= 15
    for spec in v["small"]:
        a = make_input(oracle, spec)
        assert sha(a) == spec["input_sha256"], spec["name"]
        assert sha(oracle.bitshuffle(a, spec["bs"])) == spec["shuffled_sha256"], spec["name"]
        ref = compressed(spec)
        assert sha(ref) == spec["compressed_sha256"]
        assert oracle.compress_lz4(a, spec["bs"]).tobytes() == ref.tobytes(), spec["name"]
        assert oracle.decompress_lz4(ref, a.shape, a.dtype, spec["bs"]).tobytes() == a.tobytes()


@pytest.mark.parametrize("dtype", ["u1", "u2", "u4", "u8", "V3", "V5", "V12"])
def test_known_answer_transposes(oracle, dtype):
    rng = np.random.default_rng(3)
    dt = np.dtype(dtype)
    arr = rng.integers(0, 200, 1024 * dt.itemsize, dtype=np.uint8).view(dt)
    out = np.empty(arr.nbytes, dtype=np.uint8)
    oracle.lib.orc_trans_bit_elem(arr.ctypes.data, out.ctypes.data, arr.size, dt.itemsize)
    assert out.tobytes() == trans_bit_elem_np(arr).tobytes()
    # trans_bit_elem == trans_bit_byte(trans_byte_elem(.)) restricted to a block
    assert trans_bit_byte_np(trans_byte_elem_np(arr)).size == arr.nbytes
    back = np.empty_like(out)
    oracle.lib.orc_untrans_bit_elem(out.ctypes.data, back.ctypes.data, arr.size, dt.itemsize)
    assert back.tobytes() == arr.view(np.uint8).tobytes()


def test_default_block_size(oracle):
    # format-stable values (src/bitshuffle_core.c:2038-2046)
    assert [oracle.default_block_size(e) for e in (1, 2, 3, 4, 8, 64, 100)] == \
        [8192, 4096, 2728, 2048, 1024, 128, 128]


def test_tail_and_partial_block(oracle):
    rng = np.random.default_rng(11)
    arr = rng.integers(0, 1000, 4096 + 64 + 5, dtype=np.int16)
    enc = oracle.compress_lz4(arr)
    # raw tail: the last 5 elements verbatim
    assert enc[-10:].tobytes() == arr[-5:].tobytes()
    assert oracle.decompress_lz4(enc, arr.shape, arr.dtype).tobytes() == arr.tobytes()


def test_wave_model_matches_oracle(oracle):
    """The HIP encoder's wave-parallel parse (tests/wave_model.py) is the
    reference's greedy parse: check on collision-heavy and correlated blocks."""
    from tests.wave_model import encode_block, sched
    seq, p, step, nb = [], 0, 1, 64
    for _ in range(2000):
        seq.append(p)
        p += step
        step = nb >> 6
        nb += 1
    assert list(sched(np.arange(2000))) == seq
    rng = np.random.default_rng(5)
    blocks = [rng.integers(0, 256, 700, dtype=np.uint8), np.zeros(300, np.uint8),
              (np.arange(2000) % 3).astype(np.uint8), rng.integers(0, 3, 1500, dtype=np.uint8),
              (np.arange(4096) % 65 * 37 % 256).astype(np.uint8)]
    sh = oracle.bitshuffle(oracle.gen_g1(8192)).view(np.uint8)
    blocks += [sh[:8192], sh[8192:]]
    for b in blocks:
        assert encode_block(b) == oracle.lz4_compress_block(b).tobytes()


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle",
                                                    "_ref", "libbshuf_ref.so")),
                    reason="oracle/_ref not built (needs /root/reference)")
def test_oracle_vs_compiled_reference(oracle):
    from oracle import Reference
    ref = Reference()
    rng = np.random.default_rng(9)
    for E in [1, 2, 3, 4, 6, 8, 16]:
        for n in [0, 5, 8, 100, 3001, 20000]:
            for block in [0, 8, 128, 680]:
                d = (rng.integers(0, 3, n * E).cumsum() % 256).astype(np.uint8)
                arr = d.view(np.dtype("V%d" % E)) if E > 1 else d
                assert oracle.bitshuffle(arr, block).tobytes() == ref.bitshuffle(arr, block).tobytes()
                assert oracle.compress_lz4(arr, block).tobytes() == \
                    ref.compress_lz4(arr, block).tobytes()


def _lz4_outcome(codec, comp, cap):
    try:
        return ("ok", codec.lz4_decompress_block(comp, cap).tobytes())
    except RuntimeError as e:
        return ("err", e.args[1])


def corrupt_lz4_blocks(oracle, seed=11, per_base=40):
    """Valid LZ4 blocks of assorted sizes plus seeded corruptions of them:
    random bytes, 0/15/255 bytes, truncations, extensions."""
    rng = np.random.default_rng(seed)
    bases = []
    for n in [16, 40, 63, 64, 65, 80, 100, 300, 1000, 4096, 8192]:
        for kind in range(4):
            if kind == 0:
                d = rng.integers(0, 256, n, dtype=np.uint8)
            elif kind == 1:
                d = np.repeat(rng.integers(0, 3, n // 5 + 1), 5)[:n].astype(np.uint8)
            elif kind == 2:
                d = (rng.integers(-1, 2, n).cumsum() % 7).astype(np.uint8)
            else:
                d = np.zeros(n, dtype=np.uint8)
                d[rng.integers(0, n, max(n // 50, 1))] = rng.integers(0, 256, max(n // 50, 1))
            bases.append((d, oracle.lz4_compress_block(d)))
    cases = []
    for d, c in bases:
        n = d.size
        cases.append((c, n))
        cases.append((c, n + 1))
        cases.append((c, max(n - 1, 0)))
        for _ in range(per_base):
            x = c.copy()
            kind = rng.integers(0, 6)
            if kind <= 2 and x.size:
                k = int(rng.integers(1, 4))
                idx = rng.integers(0, x.size, k)
                x[idx] = [rng.integers(0, 256), 255, 0x0F, 0xF0, 0][kind] if kind else \
                    rng.integers(0, 256, k)
            elif kind == 3 and x.size > 1:
                x = x[:int(rng.integers(1, x.size))]
            elif kind == 4:
                x = np.concatenate([x, rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)])
            else:
                x = rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8)
            cases.append((x, n))
    return cases


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(__file__), "..", "oracle",
                                                    "_ref", "libbshuf_ref.so")),
                    reason="oracle/_ref not built (needs /root/reference)")
def test_lz4_decoder_matches_reference_on_corrupt_blocks(oracle):
    """Pins the oracle's LZ4_decompress_safe restatement (accept/reject,
    error position, output) against the compiled reference, on valid blocks
    and ~1900 seeded corruptions of them."""
    from oracle import Reference
    ref = Reference()
    diffs = []
    cases = corrupt_lz4_blocks(oracle)
    nerr = 0
    for comp, cap in cases:
        a, b = _lz4_outcome(oracle, comp, cap), _lz4_outcome(ref, comp, cap)
        nerr += a[0] == "err"
        if a != b:
            diffs.append((comp.size, cap, a[0], a[1] if a[0] == "err" else len(a[1]),
                          b[0], b[1] if b[0] == "err" else len(b[1])))
    assert not diffs, diffs[:10]
    assert nerr > len(cases) // 3  # the corruptions do exercise the error paths
