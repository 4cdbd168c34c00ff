"""Parity of the HIP path (through the C-ABI) with the reference.

Checked against: the reference's 42 LZ4 regression chunks, the
reference-generated vectors of tests/golden/vectors.json, the CPU oracle on
seeded random/odd/edge inputs, and at BASELINE sizes against SHA-256 digests
of the reference's own output.  Integer/byte work: every comparison is
bit-exact.
"""
import numpy as np
import pytest

from tests.vectors import compressed, load_vectors, make_input, regression_cases, sha

pytestmark = pytest.mark.gpu

DTYPES = {1: np.uint8, 2: np.uint16, 4: np.uint32, 8: np.uint64}


def view_e(data, E):
    data = np.ascontiguousarray(data, dtype=np.uint8)
    return data.view(DTYPES[E]) if E in DTYPES else data.view(np.dtype("V%d" % E))


@pytest.fixture(scope="module")
def bs():
    import bitshuffle_amd
    assert bitshuffle_amd.using_HIP(), "no HIP device: the GPU suite must run on MI355X"
    return bitshuffle_amd


@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available()
    return torch


# ------------------------------------------------------------------ transpose
@pytest.mark.parametrize("E", [1, 2, 3, 4, 5, 6, 8, 10, 12, 16, 24])
def test_bitshuffle_matches_oracle(bs, oracle, E):
    rng = np.random.default_rng(100 + E)
    for n in [0, 1, 7, 8, 9, 64, 100, 1000, 4097, 33000]:
        for block in [0, 8, 64, 680, 2048]:
            arr = view_e(rng.integers(0, 256, n * E, dtype=np.uint8), E)
            want = oracle.bitshuffle(arr, block)
            got = bs.bitshuffle(arr, block)
            assert got.tobytes() == want.tobytes(), (E, n, block)
            back = bs.bitunshuffle(got, block)
            assert back.tobytes() == arr.tobytes(), (E, n, block)


def test_bitshuffle_golden_and_known_answer(bs, oracle):
    from tests.test_oracle import trans_bit_elem_np
    for spec in load_vectors()["small"]:
        a = make_input(oracle, spec)
        assert sha(bs.bitshuffle(a, spec["bs"])) == spec["shuffled_sha256"], spec["name"]
    rng = np.random.default_rng(7)
    for dt in [np.int8, np.int16, np.int32, np.int64, np.dtype("V3"), np.dtype("V12")]:
        dt = np.dtype(dt)
        arr = rng.integers(0, 200, 1024 * dt.itemsize, dtype=np.uint8).view(dt)
        # a single block covering the whole array == trans_bit_elem of test_ext.py:702-716
        got = bs.bitshuffle(arr, arr.size)
        assert got.tobytes() == trans_bit_elem_np(arr).tobytes(), dt


def test_bitshuffle_bad_block_size(bs):
    with pytest.raises(RuntimeError) as ei:
        bs.bitshuffle(np.arange(100, dtype=np.int16), 12)
    assert ei.value.args[1] == -81


# ------------------------------------------------------------------ LZ4 stream
def test_regression_chunks_encode_decode(bs):
    """The 42 stored LZ4 chunks of the reference's regression files
    (tests/test_regression.py:24-42): decode to `original`, and re-encoding
    `original` reproduces the stored bytes exactly."""
    cases = regression_cases()
    assert len(cases) == 42
    for ver, name, arr, chunk, block in cases:
        stream = chunk[12:]
        dec = bs.decompress_lz4(stream, arr.shape, arr.dtype, block)
        assert dec.tobytes() == arr.tobytes(), (ver, name)
        enc = bs.compress_lz4(arr, block)
        assert enc.tobytes() == stream.tobytes(), (ver, name)


def test_golden_vectors_encode_decode(bs, oracle):
    for spec in load_vectors()["small"]:
        a = make_input(oracle, spec)
        ref = compressed(spec)
        enc = bs.compress_lz4(a, spec["bs"])
        assert enc.size == spec["compressed_len"], spec["name"]
        assert enc.tobytes() == ref.tobytes(), spec["name"]
        dec = bs.decompress_lz4(ref, a.shape, a.dtype, spec["bs"])
        assert dec.tobytes() == a.tobytes(), spec["name"]


@pytest.mark.parametrize("kind", ["random", "runs", "periodic", "walk", "zeros"])
def test_lz4_matches_oracle(bs, oracle, kind):
    rng = np.random.default_rng(hash(kind) & 0xFFFF)
    for E in [1, 2, 4, 8, 3, 12]:
        for n in [1, 8, 13, 64, 200, 1000, 5000, 40000]:
            nbytes = n * E
            if kind == "random":
                d = rng.integers(0, 256, nbytes, dtype=np.uint8)
            elif kind == "runs":
                d = np.repeat(rng.integers(0, 4, nbytes // 7 + 1), 7)[:nbytes].astype(np.uint8)
            elif kind == "periodic":
                d = (np.arange(nbytes) % (1 + (n % 13)) * 29).astype(np.uint8)
            elif kind == "walk":
                d = (rng.integers(-2, 3, nbytes).cumsum() % 256).astype(np.uint8)
            else:
                d = np.zeros(nbytes, dtype=np.uint8)
            arr = view_e(d, E)
            for block in [0, 64, 8]:
                want = oracle.compress_lz4(arr, block)
                got = bs.compress_lz4(arr, block)
                assert got.tobytes() == want.tobytes(), (kind, E, n, block)
                back = bs.decompress_lz4(got, arr.shape, arr.dtype, block)
                assert back.tobytes() == arr.tobytes(), (kind, E, n, block)


def test_odd_e_deferred_copyout_alternating(bs, oracle):
    """Odd element sizes stage each block's raw bytes at the END of the hash
    table's LDS while the previous block's record still waits at its start
    (deferred copy-out); an incompressible record would overlap them and is
    flushed first.  Blocks alternate between incompressible, compressible and
    zero bytes so both orders meet, through the host API and the default
    blocks (8 KiB or just below)."""
    rng = np.random.default_rng(3)
    for E in [3, 5, 7, 12]:
        bs_bytes = (8192 // E) // 8 * 8 * E
        parts = []
        for k in range(14):
            kind = (k * 7 // 3) % 3
            if kind == 0:
                parts.append(rng.integers(0, 256, bs_bytes, dtype=np.uint8))
            elif kind == 1:
                parts.append((rng.integers(-2, 3, bs_bytes).cumsum() % 7).astype(np.uint8))
            else:
                parts.append(np.zeros(bs_bytes, dtype=np.uint8))
        d = np.concatenate(parts + [rng.integers(0, 256, 5 * E, dtype=np.uint8)])
        arr = view_e(d, E)
        want = oracle.compress_lz4(arr)
        got = bs.compress_lz4(arr)
        assert got.tobytes() == want.tobytes(), E
        back = bs.decompress_lz4(got, arr.shape, arr.dtype)
        assert back.tobytes() == arr.tobytes(), E


def _with_variant(bs, variant, fn):
    try:
        assert bs.lib.bshuf_set_variant(variant) == 0
        return fn()
    finally:
        bs.lib.bshuf_set_variant(0)


def test_variant_knob_rejects_ablations(bs):
    """Only byte-identical variants are accepted (and only for the calling
    thread); timing ablations are not in the product library."""
    for v in (1, 48, 68, 3, -1, 576):
        assert bs.lib.bshuf_set_variant(v) == -71
    assert bs.lib.bshuf_set_variant(0) == 0


@pytest.mark.parametrize("variant", [128, 2, 4, 8, 16, 32, 64, 512, 2048, 4096, 8192, 16384, 24576, 40960, 57344, 65536, 319488, 172032, 450560, 2793472, 3072000])
def test_encoder_alternate_paths_match_oracle(bs, oracle, variant):
    """Byte-identical alternate paths (elem_size 2): 128 the insert/
    read-back search window (the fallback when the LDS-atomic lane-order
    self-check fails), 8192 the hand-scheduled re-test chain (asm, VGPR-buffered
    descriptors) without its offset-2 shortcut (40960 = the default), 65536 the
    compiled re-test chain (round 3's default), 2 the inline emitter (also the overflow path of the
    descriptor emitter), 4 the one-group-per-lane transpose, 8 the re-test
    table lookup by lane 0's returning exchange (the default: plain LDS ops by
    every lane); decoder record access: 16 straight from global memory with
    each record's lines touched two blocks ahead, 32 the same without the
    touch, 64 staged in an LDS buffer of its own (the default decodes each
    record in place at the end of its block's LDS buffer); 512 every search
    window with per-lane validity masks (the default runs full windows
    without them); 2048 the re-test's
    4-byte test as its own readfirstlane compare before the count; 4096 each record
    copied out at the end of its own block (the default defers it behind the
    next block's transpose)."""
    rng = np.random.default_rng(128)
    cases = [oracle.gen_g1(3 * 4096 + 1005),
             (rng.integers(-2, 3, 50000).cumsum() % 97).astype(np.int16),
             np.repeat(rng.integers(0, 4, 9000), 7).astype(np.int16),
             rng.integers(0, 1 << 16, 20000).astype(np.uint16)]

    def run():
        for arr in cases:
            for block in [0, 64, 2048]:
                want = oracle.compress_lz4(arr, block)
                got = bs.compress_lz4(arr, block)
                assert got.tobytes() == want.tobytes(), (arr.size, block)
                back = bs.decompress_lz4(got, arr.shape, arr.dtype, block)
                assert back.tobytes() == arr.tobytes(), (arr.size, block)
    _with_variant(bs, variant, run)


@pytest.mark.parametrize("variant", [8192, 16384, 24576, 40960, 57344, 65536, 319488, 172032, 450560, 2793472, 3072000])
def test_encoder_variant_all_element_sizes(bs, oracle, variant):
    """A variant that applies to every element size (8192: the hand-scheduled
    re-test chain) on the oracle matrix of test_lz4_matches_oracle plus the
    reference's regression chunks and the batch API."""
    def run():
        for kind in ("random", "runs", "periodic", "walk", "zeros"):
            rng = np.random.default_rng(hash(kind) & 0xFFFF)
            for E in [1, 2, 4, 8, 3, 12]:
                for n in [13, 200, 5000, 40000]:
                    nbytes = n * E
                    if kind == "random":
                        d = rng.integers(0, 256, nbytes, dtype=np.uint8)
                    elif kind == "runs":
                        d = np.repeat(rng.integers(0, 4, nbytes // 7 + 1), 7)[:nbytes].astype(np.uint8)
                    elif kind == "periodic":
                        d = (np.arange(nbytes) % (1 + (n % 13)) * 29).astype(np.uint8)
                    elif kind == "walk":
                        d = (rng.integers(-2, 3, nbytes).cumsum() % 256).astype(np.uint8)
                    else:
                        d = np.zeros(nbytes, dtype=np.uint8)
                    arr = view_e(d, E)
                    for block in [0, 64]:
                        want = oracle.compress_lz4(arr, block)
                        got = bs.compress_lz4(arr, block)
                        assert got.tobytes() == want.tobytes(), (kind, E, n, block)
        for ver, name, arr, chunk, block in regression_cases():
            assert bs.compress_lz4(arr, block).tobytes() == chunk[12:].tobytes(), (ver, name)
        for gen in (oracle.gen_g1, oracle.gen_g2):
            a = gen(20 * 4096 + 1005)
            assert bs.compress_lz4(a).tobytes() == oracle.compress_lz4(a).tobytes()
    _with_variant(bs, variant, run)


def _lz4_len(v):
    out = bytearray()
    while v >= 255:
        out.append(255)
        v -= 255
    out.append(v)
    return out


def _crafted_block(rng, n, oracle):
    """One LZ4 record decoding to n bytes, from random sequences weighted to
    the decoder's hard cases: offsets 0-8 (periodic fills, incl. the
    offset 0 LZ4_decompress_safe accepts), matches reading the output of the
    sequence just before (batch breaks), long matches and literal runs, length
    extensions.  Checked against the oracle's decoder."""
    while True:
        pay = bytearray()
        op = 0
        hist = []
        while True:
            lit = int(rng.choice([0, 0, 0, 1, 2, 3, 7, 14, 15, 16, 17, 33, 64, 300]))
            ml = int(rng.choice([4, 5, 6, 7, 8, 11, 15, 16, 17, 18, 19, 20, 33, 63, 64, 65, 127, 300, 1000]))
            if op + lit + ml > n - 12:
                break
            avail = op + lit
            kind = rng.integers(0, 4)
            if kind == 0:
                off = int(rng.integers(0, 9))
            elif kind == 1 and hist:
                off = max(1, avail - hist[-1] - int(rng.integers(0, 3)))  # into the previous match
            elif kind == 2:
                off = int(rng.integers(1, 40))
            else:
                off = int(rng.integers(1, max(2, avail)))
            if off > avail or off > 65535:
                off = min(avail, 65535)
            if avail == 0:
                lit, avail, off = 1, op + 1, 1
            tok = (min(lit, 15) << 4) | min(ml - 4, 15)
            pay.append(tok)
            if lit >= 15:
                pay += _lz4_len(lit - 15)
            pay += bytes(rng.integers(0, 4, lit, dtype=np.uint8) * 37)
            pay += bytes([off & 255, off >> 8])
            if ml - 4 >= 15:
                pay += _lz4_len(ml - 4 - 15)
            hist.append(avail)
            op = avail + ml
        last = n - op
        pay.append(min(last, 15) << 4)
        if last >= 15:
            pay += _lz4_len(last - 15)
        pay += bytes(rng.integers(0, 256, last, dtype=np.uint8))
        try:
            oracle.lz4_decompress_block(np.frombuffer(bytes(pay), np.uint8), n)
        except RuntimeError:
            continue
        return bytes(pay)


@pytest.mark.parametrize("E", [1, 4])
def test_decoder_crafted_sequences_match_oracle(bs, oracle, E):
    """Streams of hand-built LZ4 records (not what the encoder emits): every
    decoder match path -- per-lane and wave copies, periods 0/1/2/3/4/other,
    matches reading the previous sequence's output (batch breaks), long
    lengths -- against the oracle's LZ4_decompress_safe restatement.  Blocks
    whose in-place margin fails take the decoder's global-record path."""
    rng = np.random.default_rng(4242 + E)
    nbytes = 8192
    frames = bytearray()
    for _ in range(40):
        pay = _crafted_block(rng, nbytes, oracle)
        frames += len(pay).to_bytes(4, "big") + pay
    buf = np.frombuffer(bytes(frames), np.uint8)
    shape, dt = (40 * nbytes // E,), DTYPES[E]
    want = oracle.decompress_lz4(buf, shape, dt, nbytes // E)

    got = bs.decompress_lz4(buf, shape, dt, nbytes // E)
    assert got.tobytes() == want.tobytes()


def _record(payload):
    return np.frombuffer(len(payload).to_bytes(4, "big") + bytes(payload), dtype=np.uint8)


# corrupt single-block payloads (4096 x u8, or 2048 x u16); each hits one
# LZ4_decompress_safe check at a specific position
_BAD_PAYLOADS = {
    "litlen_run_to_end": [0xF0, 255, 255, 255],
    "litlen_run_to_end_long": [0xF0] + [255] * 70,
    "matchlen_run_to_end": [0x1F, 7, 1, 0, 255, 255],
    "matchlen_run_to_end_long": [0x1F, 7, 1, 0] + [255] * 80,
    "offset_zero": [0x10, 7, 0, 0, 0x00],
    "offset_past_start": [0x20, 7, 8, 3, 0, 0x00],
    "literals_truncated": [0x50, 1, 2],
    "offset_truncated": [0x10, 7, 1],
    "output_short": [0x30, 1, 2, 3],
    "match_past_end": [0x1F, 7, 1, 0, 255, 255, 255, 255, 255, 255, 255, 255, 255, 255,
                       255, 255, 255, 255, 255, 255, 100, 0x00],
    "literals_past_end": [0xF0, 255] * 1 + [255] * 16 + [10] + [0] * 8,
    "empty_token_run": [0x00, 1, 0],
}


@pytest.mark.parametrize("name", sorted(_BAD_PAYLOADS))
def test_decompress_error_codes_match_oracle(bs, oracle, name):
    """The error code of a corrupt record equals the oracle's (r - 1000 with r
    LZ4_decompress_safe's -(position)-1, or -91)."""
    for dtype, n in [(np.uint8, 4096), (np.uint16, 2048)]:
        buf = _record(_BAD_PAYLOADS[name])
        with pytest.raises(RuntimeError) as want:
            oracle.decompress_lz4(buf, (n,), dtype)
        with pytest.raises(RuntimeError) as got:
            bs.decompress_lz4(buf, (n,), dtype)
        assert got.value.args[1] == want.value.args[1], (name, dtype)


def test_decompress_corrupt_blocks_match_oracle(bs, oracle):
    """Seeded corruptions of valid LZ4 blocks (tests/test_oracle.py pins the
    oracle's LZ4_decompress_safe restatement to the compiled reference on the
    same generator): the GPU accepts exactly what the oracle accepts, with the
    same output, and rejects the rest with the same error code."""
    from tests.test_oracle import corrupt_lz4_blocks
    checked = 0
    for comp, cap in corrupt_lz4_blocks(oracle, seed=23, per_base=12):
        # (records longer than LZ4_compressBound(block) -- no compressor emits
        # one -- are rejected with -91 by design)
        if cap == 0 or cap % 8 or cap > 8192 or comp.size > cap + cap // 255 + 16:
            continue
        buf = _record(comp)
        try:
            want = ("ok", oracle.decompress_lz4(buf, (cap,), np.uint8).tobytes())
        except RuntimeError as e:
            want = ("err", e.args[1])
        try:
            got = ("ok", bs.decompress_lz4(buf, (cap,), np.uint8).tobytes())
        except RuntimeError as e:
            got = ("err", e.args[1])
        assert got == want, (comp.size, cap, got[0], want[0],
                             got[1] if got[0] == "err" else None,
                             want[1] if want[0] == "err" else None)
        checked += 1
    assert checked > 300


def test_lz4_u32_table_path(bs, oracle):
    """Blocks of >= 65547 bytes switch LZ4 to the byU32 table + hash5
    (lz4/lz4.c:1389-1393, 785-795)."""
    g1 = oracle.gen_g1(1 << 19)
    for arr, block in [(g1.view(np.uint64), 8200), (g1, 40000), (g1, 32768 + 8),
                       (oracle.gen_g2(1 << 17), 16400)]:
        want = oracle.compress_lz4(arr, block)
        got = bs.compress_lz4(arr, block)
        assert got.tobytes() == want.tobytes(), (arr.dtype, block)
        back = bs.decompress_lz4(got, arr.shape, arr.dtype, block)
        assert back.tobytes() == arr.tobytes()


def test_decompress_errors(bs, oracle):
    arr = oracle.gen_g1(10000)
    enc = oracle.compress_lz4(arr)
    bad = enc.copy()
    bad[4 + 20] ^= 0xFF  # corrupt the first block's payload
    with pytest.raises(RuntimeError):
        out = bs.decompress_lz4(bad, arr.shape, arr.dtype)
        assert out.tobytes() != arr.tobytes()
        raise RuntimeError("corrupt stream decoded to different data")
    with pytest.raises(RuntimeError):
        bs.decompress_lz4(enc[:-1], arr.shape, arr.dtype)  # consumed != buffer size


def _block_header_positions(enc, nblocks):
    pos, out = 0, []
    for _ in range(nblocks):
        out.append(pos)
        pos += 4 + int.from_bytes(enc[pos:pos + 4].tobytes(), "big")
    return out


def test_device_decode_truncated_and_corrupt_headers(bs, oracle, torch):
    """The device decoder WITHOUT block offsets (parallel index rebuild) on
    truncated streams and on corrupted block headers: every read stays inside
    in_nbytes and the call reports an error instead of decoding; where the
    host drop-in path sees the same bytes (a corrupt last header) both return
    the same code."""
    a = oracle.gen_g1(20 * 4096 + 1000 + 3)
    enc = oracle.compress_lz4(a)
    nb = 21
    hdr = _block_header_positions(enc, nb)
    bad = [enc[:-1], enc[:hdr[7] + 2], enc[:hdr[12]], enc[:len(enc) // 2], enc[:3]]
    for k, val in [(5, 0), (5, 0xFFFFFFFF), (5, None), (nb - 1, 0), (nb - 1, 9000)]:
        e = enc.copy()
        if val is None:  # off by one
            val = int.from_bytes(e[hdr[k]:hdr[k] + 4].tobytes(), "big") + 1
        e[hdr[k]:hdr[k] + 4] = np.frombuffer(int(val).to_bytes(4, "big"), dtype=np.uint8)
        bad.append(e)
    for i, buf in enumerate(bad):
        t = torch.from_numpy(np.ascontiguousarray(buf)).cuda()
        with pytest.raises(RuntimeError) as dev:
            bs.decompress_lz4_dev(t, a.shape, torch.int16)
        torch.cuda.synchronize()
        if i >= len(bad) - 2:  # corrupt LAST header: host walk == device index
            # (no padding: the host walk stages only the implausible header,
            # never payload bytes past it)
            with pytest.raises(RuntimeError) as host:
                bs.decompress_lz4(np.ascontiguousarray(buf), a.shape, a.dtype)
            assert host.value.args[1] == dev.value.args[1], i
    # a zero-length last header: the reference's LZ4_decompress_safe returns -1
    # for srcSize 0 without reading anything (-1001 from bshuf_decompress_lz4),
    # so the oracle pins the host and device codes there
    zero_last = bad[len(bad) - 2]
    with pytest.raises(RuntimeError) as want:
        oracle.decompress_lz4(np.ascontiguousarray(zero_last), a.shape, a.dtype)
    with pytest.raises(RuntimeError) as host:
        bs.decompress_lz4(np.ascontiguousarray(zero_last), a.shape, a.dtype)
    assert want.value.args[1] == host.value.args[1] == -1001


# ------------------------------------------------------------------ device API
def test_device_api_roundtrip_and_index(bs, oracle, torch):
    for spec in load_vectors()["small"]:
        a = make_input(oracle, spec)
        ref = compressed(spec)
        t = torch.from_numpy(a.view(np.uint8).copy()).cuda()
        off = torch.empty(max(1, bs.lib.bshuf_lz4_dev_nblocks(a.size, a.dtype.itemsize, spec["bs"])),
                          dtype=torch.int64, device="cuda")
        # element count / size come from the original dtype
        out = torch.empty(bs.compress_lz4_bound(a.size, a.dtype.itemsize, spec["bs"]),
                          dtype=torch.uint8, device="cuda")
        res = torch.empty(1, dtype=torch.int64, device="cuda")
        import ctypes
        rc = bs.lib.bshuf_compress_lz4_dev(ctypes.c_void_p(t.data_ptr()),
                                           ctypes.c_void_p(out.data_ptr()), a.size,
                                           a.dtype.itemsize, spec["bs"], None, 0,
                                           ctypes.c_void_p(res.data_ptr()),
                                           ctypes.c_void_p(off.data_ptr()), None)
        assert rc == 0
        n = int(res.item())
        assert n == ref.size, spec["name"]
        assert out[:n].cpu().numpy().tobytes() == ref.tobytes(), spec["name"]
        # decode with the parallel index rebuild (no offsets)
        dec = torch.empty(a.size * a.dtype.itemsize, dtype=torch.uint8, device="cuda")
        rc = bs.lib.bshuf_decompress_lz4_dev(ctypes.c_void_p(out.data_ptr()), n,
                                             ctypes.c_void_p(dec.data_ptr()), a.size,
                                             a.dtype.itemsize, spec["bs"], None, 0,
                                             ctypes.c_void_p(res.data_ptr()), None, None)
        assert rc == 0
        assert int(res.item()) == n, spec["name"]
        assert dec.cpu().numpy().tobytes() == a.view(np.uint8).tobytes(), spec["name"]
        # decode with the encoder's offsets
        dec.zero_()
        rc = bs.lib.bshuf_decompress_lz4_dev(ctypes.c_void_p(out.data_ptr()), n,
                                             ctypes.c_void_p(dec.data_ptr()), a.size,
                                             a.dtype.itemsize, spec["bs"], None, 0,
                                             ctypes.c_void_p(res.data_ptr()),
                                             ctypes.c_void_p(off.data_ptr()), None)
        assert rc == 0 and int(res.item()) == n
        assert dec.cpu().numpy().tobytes() == a.view(np.uint8).tobytes(), spec["name"]


def test_device_synth_matches_cpu_generators(bs, oracle, torch):
    for gen, dt, ref in [(0, torch.int32, oracle.gen_g0), (1, torch.int16, oracle.gen_g1),
                         (2, torch.float32, oracle.gen_g2)]:
        t = torch.empty(100003, dtype=dt, device="cuda")
        bs.synth_fill_dev(t, gen, first=12345678)
        want = ref(100003, 12345678) if gen == 0 else ref(100003, 12345678, 12345)
        assert t.cpu().numpy().tobytes() == want.tobytes(), gen


# ------------------------------------------------------------------ full size
@pytest.mark.slow
def test_full_size_digests(bs, torch):
    """BASELINE configs 1-4 at full size vs SHA-256 of the reference's output
    (tests/golden/vectors.json 'full'): the 64 MiB ramp, six 32 MiB chunks of
    config 4, 4 GiB int16 G1 and 16 GiB float32 G2 (2**32 elements, a 6.9 GB
    stream: > 2**31-element and > 4 GiB offsets), plus decode round trips."""
    import hashlib
    full = {e["name"]: e for e in load_vectors()["full"]}

    def digest(t):
        h = hashlib.sha256()
        step = 1 << 28
        for i in range(0, t.numel(), step):
            h.update(t[i:i + step].cpu().numpy().tobytes())
        return h.hexdigest()

    e = full["cfg1_g0_i32_64MiB"]
    x = torch.empty(e["size"], dtype=torch.int32, device="cuda")
    bs.synth_fill_dev(x, 0)
    assert digest(x.view(torch.uint8)) == e["input_sha256"]
    y = bs.bitshuffle_dev(x)
    assert digest(y.view(torch.uint8)) == e["shuffled_sha256"]
    assert torch.equal(bs.bitunshuffle_dev(y), x)
    del x, y

    names = ["cfg4_g1_chunk%04d" % c for c in (0, 1, 2, 3, 511, 1023)]
    for name in names + ["cfg2_g1_i16_4GiB", "cfg3_g2_f32_16GiB"]:
        e = full[name]
        g2 = e["gen"] == "g2"
        x = torch.empty(e["size"], dtype=torch.float32 if g2 else torch.int16, device="cuda")
        bs.synth_fill_dev(x, 2 if g2 else 1, seed=e.get("seed", 12345))
        c = bs.compress_lz4_dev(x)
        assert c.numel() == e["compressed_len"], name
        assert digest(c) == e["compressed_sha256"], name
        d = bs.decompress_lz4_dev(c.clone(), x.shape, x.dtype)
        assert torch.equal(d, x), name
        del x, c, d
        torch.cuda.empty_cache()


def test_device_api_unaligned_pointers(bs, oracle, torch):
    """Device entry points on pointers that are NOT 16-byte aligned (odd
    offsets into larger allocations) give the same bytes."""
    import ctypes
    a = oracle.gen_g1(3 * 4096 + 517)
    want = oracle.compress_lz4(a)
    nbytes = a.nbytes
    for off_in, off_out in [(1, 3), (7, 0), (0, 5), (2, 2)]:
        src = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
        src[off_in:off_in + nbytes] = torch.from_numpy(a.view(np.uint8).copy()).cuda()
        bound = bs.compress_lz4_bound(a.size, 2)
        dst = torch.zeros(bound + 64, dtype=torch.uint8, device="cuda")
        res = torch.zeros(1, dtype=torch.int64, device="cuda")
        rc = bs.lib.bshuf_compress_lz4_dev(ctypes.c_void_p(src.data_ptr() + off_in),
                                           ctypes.c_void_p(dst.data_ptr() + off_out), a.size, 2, 0,
                                           None, 0, ctypes.c_void_p(res.data_ptr()), None, None)
        assert rc == 0
        n = int(res.item())
        assert dst[off_out:off_out + n].cpu().numpy().tobytes() == want.tobytes(), (off_in, off_out)
        back = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
        rc = bs.lib.bshuf_decompress_lz4_dev(ctypes.c_void_p(dst.data_ptr() + off_out), n,
                                             ctypes.c_void_p(back.data_ptr() + off_in), a.size, 2,
                                             0, None, 0, ctypes.c_void_p(res.data_ptr()), None, None)
        assert rc == 0 and int(res.item()) == n
        assert back[off_in:off_in + nbytes].cpu().numpy().tobytes() == a.view(np.uint8).tobytes()
        sh = torch.zeros(nbytes + 64, dtype=torch.uint8, device="cuda")
        r = bs.lib.bshuf_bitshuffle_dev(ctypes.c_void_p(src.data_ptr() + off_in),
                                        ctypes.c_void_p(sh.data_ptr() + off_out), a.size, 2, 0, None)
        torch.cuda.synchronize()
        assert r == nbytes
        assert sh[off_out:off_out + nbytes].cpu().numpy().tobytes() == oracle.bitshuffle(a).tobytes()


# --------------------------------------------------------- pipelined encode
NO_PIPE = 1 << 20  # bshuf_set_variant bit: encode without segments / side stream


def test_pipelined_encode_matches_oracle(bs, oracle, torch):
    """Encodes of >= 65536 blocks run as 4 parse segments with each segment's
    offset scan + compaction on a side stream (launch.h).  Single stream:
    65536 + 3 full blocks (not a multiple of 4), a partial block and a raw
    tail, caller workspace and ws = NULL; batch: 19 streams of uneven sizes
    whose segment boundaries fall inside streams.  Every stream equals the
    oracle's and the unsegmented (NO_PIPE) encode's, offsets included."""
    import ctypes
    n = (65536 + 3) * 4096 + 1005 + 5
    a = oracle.gen_g1(n, 0, 4321)
    want = oracle.compress_lz4(a)
    x = torch.from_numpy(a).cuda()
    nb = int(bs.lib.bshuf_lz4_dev_nblocks(n, 2, 0))
    got = {}
    for v in (0, NO_PIPE):
        def run():
            outs = []
            for ws in (True, False):
                out = torch.empty(bs.compress_lz4_bound(n, 2, 0), dtype=torch.uint8, device="cuda")
                res = torch.empty(1, dtype=torch.int64, device="cuda")
                off = torch.zeros(nb, dtype=torch.int64, device="cuda")
                wsb = int(bs.lib.bshuf_compress_lz4_dev_workspace(n, 2, 0))
                w = torch.empty(wsb, dtype=torch.uint8, device="cuda") if ws else None
                rc = bs.lib.bshuf_compress_lz4_dev(
                    ctypes.c_void_p(x.data_ptr()), ctypes.c_void_p(out.data_ptr()), n, 2, 0,
                    ctypes.c_void_p(w.data_ptr()) if ws else None, wsb if ws else 0,
                    ctypes.c_void_p(res.data_ptr()), ctypes.c_void_p(off.data_ptr()), None)
                assert rc == 0
                c = int(res.item())
                outs.append((out[:c].cpu().numpy().tobytes(), off.cpu().numpy().copy()))
            return outs
        got[v] = _with_variant(bs, v, run)
    for v in got:
        for enc, off in got[v]:
            assert enc == want.tobytes(), v
            assert np.array_equal(off, got[NO_PIPE][0][1]), v
    del x
    # batch above the threshold: uneven streams
    sizes = [(3000 + 577 * i) * 4096 + 37 * i for i in range(19)]
    arrs = [oracle.gen_g1(m, 7 * i, 99 + i) for i, m in enumerate(sizes)]
    xs = [torch.from_numpy(q).cuda() for q in arrs]
    nblk = sum(int(bs.lib.bshuf_lz4_dev_nblocks(q.size, 2, 0)) for q in arrs)
    assert nblk >= 65536
    res = {}
    for v in (0, NO_PIPE):
        def runb():
            offs = torch.zeros(nblk, dtype=torch.int64, device="cuda")
            outs = bs.compress_lz4_batch_dev(xs, 0, offsets=offs)
            return [o.cpu().numpy().tobytes() for o in outs], offs.cpu().numpy()
        res[v] = _with_variant(bs, v, runb)
    for q, enc in zip(arrs, res[0][0]):
        assert enc == oracle.compress_lz4(q).tobytes(), q.size
    assert res[0][0] == res[NO_PIPE][0]
    assert np.array_equal(res[0][1], res[NO_PIPE][1])


# ------------------------------------------------------------------ batch API
def test_device_length_entry_points(bs, oracle, torch):
    """bshuf_decompress_lz4_dev_dlen / _batch_dev_dlen: the stream length is a
    DEVICE int64 (the compress result word), the buffer only its capacity.
    Oracle streams (partial block + raw tail, E = 2 and 3, several block
    sizes) decode exactly with the same result as the host-length entry
    point; a negative length (upstream error) comes back unchanged; a length
    past the capacity is clamped to it; corrupt bytes give the host-length
    decoder's code."""
    for E, n, block in [(2, 9 * 4096 + 13, 0), (2, 300000 + 5, 0), (3, 40000 + 3, 0),
                        (2, 5 * 2048 + 7, 2048), (1, 100, 0), (2, 0, 0)]:
        raw = oracle.gen_g1((n * E + 1) // 2, 0, 12345).view(np.uint8)[: n * E]
        a = view_e(raw, E)
        want = oracle.compress_lz4(a, block)
        cap = bs.compress_lz4_bound(n, E, block)
        buf = torch.zeros(max(cap, 1), dtype=torch.uint8, device="cuda")
        x = torch.from_numpy(raw.copy()).cuda()
        _, res = bs.compress_lz4_dev(x, block_size=block, out=buf, sync=False, elem_size=E)
        y, r = bs.decompress_lz4_dev(buf, (n,), torch.uint8, block_size=block, sync=False,
                                     elem_size=E, length=res)
        assert int(res.item()) == want.size and int(r.item()) == want.size, (E, n, block)
        assert buf[: want.size].cpu().numpy().tobytes() == want.tobytes()
        assert y.cpu().numpy().tobytes() == raw.tobytes(), (E, n, block)
        # same through the convenience path (sync: checks consumed == length)
        y2 = bs.decompress_lz4_dev(buf, (n,), torch.uint8, block_size=block, elem_size=E, length=res)
        assert torch.equal(y2, y)
    # negative length word: returned as the result, nothing decoded
    a = oracle.gen_g1(3 * 4096 + 11)
    enc = oracle.compress_lz4(a)
    buf = torch.from_numpy(enc.copy()).cuda()
    neg = torch.tensor([-81], dtype=torch.int64, device="cuda")
    _, r = bs.decompress_lz4_dev(buf, a.shape, torch.int16, sync=False, length=neg)
    assert int(r.item()) == -81
    # length past the capacity: clamped to the buffer (= the exact stream here)
    big = torch.tensor([enc.size + 12345], dtype=torch.int64, device="cuda")
    y, r = bs.decompress_lz4_dev(buf, a.shape, torch.int16, sync=False, length=big)
    assert int(r.item()) == enc.size and y.cpu().numpy().tobytes() == a.tobytes()
    # a corrupt stream: the ORACLE's code for the same bytes (and the
    # host-length device decoder's)
    bad = enc.copy()
    bad[4 + 40] ^= 0x5A  # inside block 0's payload
    bad[-30:] = 0        # and the tail end
    with pytest.raises(RuntimeError) as orc:
        oracle.decompress_lz4(bad, a.shape, np.int16)
    bbuf = torch.from_numpy(bad).cuda()
    with pytest.raises(RuntimeError) as single:
        bs.decompress_lz4_dev(bbuf, a.shape, torch.int16)
    ln = torch.tensor([bad.size], dtype=torch.int64, device="cuda")
    _, r = bs.decompress_lz4_dev(bbuf, a.shape, torch.int16, sync=False, length=ln)
    assert int(r.item()) == orc.value.args[1] == single.value.args[1]
    # a payload-only corruption the decoder itself rejects (not the walk)
    bad2 = enc.copy()
    bad2[4:4 + 8] = 0xFF  # block 0: token 0xFF + 255-runs: literal length past the block
    with pytest.raises(RuntimeError) as orc2:
        oracle.decompress_lz4(bad2, a.shape, np.int16)
    _, r = bs.decompress_lz4_dev(torch.from_numpy(bad2).cuda(), a.shape, torch.int16, sync=False,
                                 length=torch.tensor([bad2.size], dtype=torch.int64, device="cuda"))
    assert int(r.item()) == orc2.value.args[1]
    # batch: capacities from the bound, lengths from the compress results
    sizes = [3 * 4096 + 1005, 0, 17, 4096, 9 * 4096 + 13, 123457]
    arrs = [oracle.gen_g1(m, 1000 * i, 12345 + i) for i, m in enumerate(sizes)]
    for block in (0, 2048):
        xs = [torch.from_numpy(v.copy()).cuda() for v in arrs]
        outs, res = bs.compress_lz4_batch_dev(xs, block, sync=False)
        dec, dres = bs.decompress_lz4_batch_dev(outs, [v.shape for v in arrs], torch.int16, block,
                                                sync=False, lengths=res)
        want = [oracle.compress_lz4(v, block).size for v in arrs]
        assert res.cpu().tolist() == want and dres.cpu().tolist() == want, block
        for v, d in zip(arrs, dec):
            assert d.cpu().numpy().tobytes() == v.tobytes(), (v.size, block)
        # one upstream error in the batch: only that stream reports it
        res2 = res.clone()
        res2[2] = -91
        _, dres = bs.decompress_lz4_batch_dev(outs, [v.shape for v in arrs], torch.int16, block,
                                              sync=False, lengths=res2)
        got = dres.cpu().tolist()
        assert got[2] == -91 and [g for i, g in enumerate(got) if i != 2] == \
            [w for i, w in enumerate(want) if i != 2]


def test_batch_api_matches_oracle(bs, oracle, torch):
    """bshuf_*_lz4_batch_dev: streams of different lengths (partial blocks,
    raw tails, an empty one, one smaller than a block) in ONE launch each way;
    every stream equals the oracle's own stream, the per-block offsets equal a
    header walk of each stream, and the decode restores every input."""
    rng = np.random.default_rng(4)
    sizes = [3 * 4096 + 1005, 0, 17, 4096, 9 * 4096 + 13, 5000, 123457]
    arrs = []
    for i, n in enumerate(sizes):
        if i % 2:
            arrs.append(oracle.gen_g1(n, 1000 * i, 12345 + i))
        else:
            arrs.append((rng.integers(-2, 3, n).cumsum() % 97).astype(np.int16))
    for block in (0, 64, 2048):
        xs = [torch.from_numpy(a.copy()).cuda() for a in arrs]
        nblk = sum(int(bs.lib.bshuf_lz4_dev_nblocks(a.size, 2, block)) for a in arrs)
        offs = torch.zeros(max(nblk, 1), dtype=torch.int64, device="cuda")
        outs = bs.compress_lz4_batch_dev(xs, block, offsets=offs)
        k = 0
        host_offs = offs.cpu().numpy()
        for a, o in zip(arrs, outs):
            want = oracle.compress_lz4(a, block)
            got = o.cpu().numpy()
            assert got.tobytes() == want.tobytes(), (a.size, block)
            nb = int(bs.lib.bshuf_lz4_dev_nblocks(a.size, 2, block))
            pos = 0
            for j in range(nb):
                assert host_offs[k + j] == pos, (a.size, block, j)
                pos += 4 + int.from_bytes(want[pos:pos + 4].tobytes(), "big")
            k += nb
        dec = bs.decompress_lz4_batch_dev([o.clone() for o in outs], [a.shape for a in arrs],
                                          torch.int16, block)
        for a, d in zip(arrs, dec):
            assert d.cpu().numpy().tobytes() == a.tobytes(), (a.size, block)


def test_batch_api_isolates_corrupt_stream(bs, oracle, torch):
    """A corrupted stream in a batch fails alone, with the single-stream
    decoder's error code; its neighbours decode correctly."""
    arrs = [oracle.gen_g1(6 * 4096 + 77, 0, 12345 + i) for i in range(5)]
    encs = [oracle.compress_lz4(a) for a in arrs]
    bad = encs[2].copy()
    bad[4 + 40] ^= 0x5A  # inside block 0's payload
    bad[-30:] = 0        # and the tail end
    bufs = [torch.from_numpy(e.copy()).cuda() for e in encs]
    bufs[2] = torch.from_numpy(bad).cuda()
    outs, res = bs.decompress_lz4_batch_dev(bufs, [a.shape for a in arrs], torch.int16, sync=False)
    res = res.cpu().tolist()
    with pytest.raises(RuntimeError) as single:
        bs.decompress_lz4_dev(bufs[2], arrs[2].shape, torch.int16)
    assert res[2] < 0 and res[2] == single.value.args[1]
    for i in (0, 1, 3, 4):
        assert res[i] == encs[i].size
        assert outs[i].cpu().numpy().tobytes() == arrs[i].tobytes()


@pytest.mark.slow
def test_batch_config4_digests(bs, torch):
    """BASELINE config 4: 32 MiB G1 chunks (seed 12345 + chunk id) compressed
    as ONE batch equal the reference's digests (chunks 0-3, 511, 1023), and
    the batch decoder restores them."""
    full = {e["name"]: e for e in load_vectors()["full"]}
    names = ["cfg4_g1_chunk%04d" % c for c in (0, 1, 2, 3, 511, 1023)]
    xs = []
    for name in names:
        e = full[name]
        x = torch.empty(e["size"], dtype=torch.int16, device="cuda")
        bs.synth_fill_dev(x, 1, seed=e["seed"])
        xs.append(x)
    outs = bs.compress_lz4_batch_dev(xs)
    import hashlib
    for name, o in zip(names, outs):
        e = full[name]
        assert o.numel() == e["compressed_len"], name
        assert hashlib.sha256(o.cpu().numpy().tobytes()).hexdigest() == e["compressed_sha256"], name
    dec = bs.decompress_lz4_batch_dev(outs, [x.shape for x in xs], torch.int16)
    for x, d in zip(xs, dec):
        assert torch.equal(x, d)


# ------------------------------------------------------------------ large blocks
@pytest.mark.parametrize("block_bytes", [96 << 10, 143 << 10, 256 << 10, 1 << 20])
def test_large_blocks_match_oracle(bs, oracle, torch, block_bytes):
    """Every block size the reference accepts (any multiple of 8 elements,
    src/bitshuffle_core.c:1894-1897): blocks above the LDS-resident kernels'
    budget (decoder from ~81 KiB, encoder from ~144 KiB) take the global-memory
    path; streams equal the oracle's and decode back, through the host API,
    the device API (with the parallel index rebuild) and the batch API."""
    rng = np.random.default_rng(block_bytes & 0xFFFF)
    for E, dt in [(2, np.int16), (8, np.uint64), (1, np.uint8)]:
        block = block_bytes // E
        n = 2 * block + block // 3 // 8 * 8 + 5
        if E == 2:
            a = oracle.gen_g1(n, 77, 999)
        else:
            a = (rng.integers(-3, 4, n * E).cumsum() % 251).astype(np.uint8).view(dt)
        want = oracle.compress_lz4(a, block)
        got = bs.compress_lz4(a, block)
        assert got.tobytes() == want.tobytes(), (E, block)
        back = bs.decompress_lz4(want, a.shape, a.dtype, block)
        assert back.tobytes() == a.tobytes(), (E, block)
        t = torch.from_numpy(a.view(np.uint8).copy()).cuda()  # raw bytes: the C-ABI gets E
        import ctypes
        out = torch.empty(bs.compress_lz4_bound(a.size, E, block), dtype=torch.uint8, device="cuda")
        res = torch.empty(1, dtype=torch.int64, device="cuda")
        rc = bs.lib.bshuf_compress_lz4_dev(ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(out.data_ptr()),
                                           a.size, E, block, None, 0, ctypes.c_void_p(res.data_ptr()),
                                           None, None)
        assert rc == 0 and int(res.item()) == want.size, (E, block)
        assert out[:want.size].cpu().numpy().tobytes() == want.tobytes()
        dec = torch.empty(a.nbytes, dtype=torch.uint8, device="cuda")
        rc = bs.lib.bshuf_decompress_lz4_dev(ctypes.c_void_p(out.data_ptr()), want.size,
                                             ctypes.c_void_p(dec.data_ptr()), a.size, E, block, None, 0,
                                             ctypes.c_void_p(res.data_ptr()), None, None)
        assert rc == 0 and int(res.item()) == want.size, (E, block, int(res.item()))
        assert dec.cpu().numpy().tobytes() == a.view(np.uint8).tobytes(), (E, block)
    # batch API (falls back to one stream at a time for such blocks)
    xs = [torch.from_numpy(oracle.gen_g1(3 * (block_bytes // 2) + 11, i, 5 + i)).cuda() for i in range(2)]
    outs = bs.compress_lz4_batch_dev(xs, block_bytes // 2)
    for x, o in zip(xs, outs):
        assert o.cpu().numpy().tobytes() == oracle.compress_lz4(x.cpu().numpy(), block_bytes // 2).tobytes()
    dec = bs.decompress_lz4_batch_dev(outs, [x.shape for x in xs], torch.int16, block_bytes // 2)
    for x, d in zip(xs, dec):
        assert torch.equal(x, d)


# ------------------------------------------------------------------ reference dtypes
# The element sizes of the reference's own test matrix (tests/test_ext.py:19-28:
# S3..S48 and complex128) beyond the ones above, plus E = 64 (the first size
# whose default block is BSHUF_MIN_RECOMMEND_BLOCK = 128 elements,
# src/bitshuffle_core.c:2038-2046) and E = 1024, whose DEFAULT block is
# 128 KiB: byU32 table in the encoder, the large-block decoder.
REF_E = [7, 9, 11, 16, 48, 64, 1024]


def _ref_e_input(E, kind, nblk_default):
    """A whole number of default blocks, a partial block and a raw tail."""
    bs_def = max(8192 // E // 8 * 8, 128)
    n = nblk_default * bs_def + (bs_def // 3) // 8 * 8 + 5
    rng = np.random.default_rng(1000 * E + len(kind))
    if kind == "random":  # as the reference's own test data: randint(0, 200)
        d = rng.integers(0, 200, n * E, dtype=np.uint8)
    else:  # a slowly varying byte walk: long LZ4 matches after the transpose
        d = (rng.integers(-2, 3, n * E).cumsum() % 251).astype(np.uint8)
    return view_e(d, E), n, bs_def


@pytest.mark.parametrize("E", REF_E)
def test_reference_dtypes_transpose(bs, oracle, E):
    arr, n, bs_def = _ref_e_input(E, "walk", 2)
    for block in [0, 8, bs_def // 2 // 8 * 8 or 8]:
        want = oracle.bitshuffle(arr, block)
        got = bs.bitshuffle(arr, block)
        assert got.tobytes() == want.tobytes(), (E, block)
        assert bs.bitunshuffle(got, block).tobytes() == arr.tobytes(), (E, block)


@pytest.mark.parametrize("E", REF_E)
def test_reference_dtypes_lz4_host(bs, oracle, E):
    """Host C-ABI (bshuf_compress_lz4 / bshuf_decompress_lz4), default and
    explicit block sizes, random and correlated bytes, vs the oracle."""
    assert bs.default_block_size(E) == max(8192 // E // 8 * 8, 128)
    for kind in ("random", "walk"):
        arr, n, bs_def = _ref_e_input(E, kind, 2)
        for block in [0, 64, bs_def // 2 // 8 * 8 or 8]:
            want = oracle.compress_lz4(arr, block)
            got = bs.compress_lz4(arr, block)
            assert got.tobytes() == want.tobytes(), (E, kind, block)
            back = bs.decompress_lz4(got, arr.shape, arr.dtype, block)
            assert back.tobytes() == arr.tobytes(), (E, kind, block)


@pytest.mark.parametrize("E", REF_E)
def test_reference_dtypes_lz4_device_and_batch(bs, oracle, torch, E):
    """The same element sizes through the device C-ABI (parallel index rebuild
    on decode) and the batch C-ABI, default block size (block_size = 0) and one
    explicit block size, vs the oracle."""
    streams = [_ref_e_input(E, "walk", k)[0] for k in (2, 1)] + [_ref_e_input(E, "random", 1)[0]]
    for block in (0, 64):
        wants = [oracle.compress_lz4(a, block) for a in streams]
        for a, want in zip(streams, wants):
            t = torch.from_numpy(a.view(np.uint8).copy()).cuda()
            c = bs.compress_lz4_dev(t, block, elem_size=E)
            assert c.cpu().numpy().tobytes() == want.tobytes(), (E, block, a.size)
            d = bs.decompress_lz4_dev(c.clone(), a.shape, None, block, elem_size=E)
            assert d.cpu().numpy().tobytes() == a.view(np.uint8).tobytes(), (E, block, a.size)
        xs = [torch.from_numpy(a.view(np.uint8).copy()).cuda() for a in streams]
        outs = bs.compress_lz4_batch_dev(xs, block, elem_size=E)
        for o, want in zip(outs, wants):
            assert o.cpu().numpy().tobytes() == want.tobytes(), (E, block, "batch")
        dec = bs.decompress_lz4_batch_dev(outs, [a.shape for a in streams], None, block, elem_size=E)
        for a, d in zip(streams, dec):
            assert d.cpu().numpy().tobytes() == a.view(np.uint8).tobytes(), (E, block, "batch")
