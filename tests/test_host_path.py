"""Host-pointer drop-in path and device workspaces from POISONED state.

Every call below starts from buffers that hold non-zero garbage: the calling
thread's cached device buffers and pinned staging slots (bshuf_host_poison),
the previous call's different bytes, and caller-provided device workspaces /
result words / outputs filled with random bytes.  Any read of a word the call
did not write first (stale or uninitialised) shows up as a wrong result on the
first run -- deterministically, not 1 run in 40.
"""
import threading

import numpy as np
import pytest

from tests.vectors import regression_cases

pytestmark = pytest.mark.gpu

POISON = [0xA5, 0xFF, 0x01, 0x5A, 0x80, 0x7F]


@pytest.fixture(scope="module")
def bs():
    import bitshuffle_amd
    assert bitshuffle_amd.using_HIP(), "no HIP device: the GPU suite must run on MI355X"
    return bitshuffle_amd


def _poison(bs, v):
    assert bs.lib.bshuf_host_poison(v) == 0


def test_host_calls_from_poisoned_buffers(bs, oracle):
    cases = regression_cases()
    arrays = [oracle.gen_g1(n, 7 * n) for n in (1 << 20, 3 * 4096 + 1000 + 5, 77)]
    arrays += [oracle.gen_g2(50_000 + 3), oracle.gen_g1(4096 * 9).view(np.uint8)]
    i = 0
    for rep in range(2):
        for ver, name, arr, chunk, block in cases[rep::4]:
            _poison(bs, POISON[i % len(POISON)])
            i += 1
            assert bs.compress_lz4(arr, block).tobytes() == chunk[12:].tobytes(), (ver, name)
            _poison(bs, POISON[i % len(POISON)])
            i += 1
            dec = bs.decompress_lz4(chunk[12:], arr.shape, arr.dtype, block)
            assert dec.tobytes() == arr.tobytes(), (ver, name)
        for a in arrays:
            want = oracle.compress_lz4(a)
            _poison(bs, POISON[i % len(POISON)])
            i += 1
            got = bs.compress_lz4(a)
            assert got.tobytes() == want.tobytes(), (a.dtype, a.size)
            _poison(bs, POISON[i % len(POISON)])
            i += 1
            assert bs.decompress_lz4(want, a.shape, a.dtype).tobytes() == a.tobytes()
            _poison(bs, POISON[i % len(POISON)])
            i += 1
            assert bs.bitshuffle(a).tobytes() == oracle.bitshuffle(a).tobytes()
            _poison(bs, POISON[i % len(POISON)])
            i += 1
            assert bs.bitunshuffle(oracle.bitshuffle(a)).tobytes() == a.tobytes()


def test_host_back_to_back_different_sizes(bs, oracle):
    """No poisoning between calls: each call's buffers hold the previous,
    LONGER call's bytes, so a stale tail or an unwritten result word shows."""
    sizes = [1 << 21, (1 << 21) - 3, 40_000, 4096 * 2 + 8 * 3 + 1, 4096, 9, 0]
    for rep in range(2):
        for n in sizes:
            a = oracle.gen_g1(n, 1000 * n + rep)
            want = oracle.compress_lz4(a)
            got = bs.compress_lz4(a)
            assert got.tobytes() == want.tobytes(), n
            assert bs.decompress_lz4(want, a.shape, a.dtype).tobytes() == a.tobytes(), n


def test_device_calls_with_poisoned_workspaces(bs, oracle):
    import torch
    g = torch.Generator(device="cuda").manual_seed(5)
    for n, E in [(3 * 4096 + 1000 + 5, 2), (1 << 19, 2), (20_003, 4), (513, 1)]:
        raw = oracle.gen_g1(n * E).view(np.uint8)[: n * E]
        a = np.ascontiguousarray(raw).view({1: np.uint8, 2: np.int16, 4: np.int32}[E])
        want = oracle.compress_lz4(a)
        t = torch.from_numpy(a.copy()).cuda()

        def garbage(nbytes):
            return torch.randint(0, 256, (max(nbytes, 256),), dtype=torch.uint8, device="cuda",
                                 generator=g)

        ws = garbage(bs.lib.bshuf_compress_lz4_dev_workspace(t.numel(), t.element_size(), 0))
        out = garbage(bs.compress_lz4_bound(t.numel(), t.element_size()))
        res = torch.full((1,), 0x5A5A5A5A5A5A, dtype=torch.int64, device="cuda")
        c = bs.compress_lz4_dev(t, out=out, workspace=ws, result=res)
        assert c.cpu().numpy().tobytes() == want.tobytes(), (n, E)
        cw = torch.from_numpy(want.copy()).cuda()
        wsd = garbage(bs.lib.bshuf_decompress_lz4_dev_workspace(cw.numel(), t.numel(),
                                                                t.element_size(), 0))
        outd = torch.from_numpy(np.frombuffer(
            np.random.default_rng(n).integers(0, 256, a.nbytes, dtype=np.uint8).tobytes(),
            dtype=a.dtype).copy()).cuda()
        res.fill_(-12345)
        y = bs.decompress_lz4_dev(cw, t.shape, t.dtype, out=outd, workspace=wsd, result=res)
        assert torch.equal(y, t), (n, E)


def test_batch_with_poisoned_workspace(bs, oracle):
    import torch
    arrs = [oracle.gen_g1(n, 31 * n) for n in (4096 * 5 + 11, 777, 4096 * 2, 0, 100_000)]
    ts = [torch.from_numpy(a.copy()).cuda() for a in arrs]
    import ctypes
    sizes = [t.numel() for t in ts]
    arr = (ctypes.c_size_t * len(sizes))(*sizes)
    wsb = bs.lib.bshuf_compress_lz4_batch_dev_workspace(ctypes.cast(arr, ctypes.c_void_p), len(sizes), 2, 0)
    for fill in (0xFF, 0x00, 0x77):
        ws = torch.full((max(wsb, 256),), fill, dtype=torch.uint8, device="cuda")
        outs = bs.compress_lz4_batch_dev(ts, workspace=ws)
        for a, o in zip(arrs, outs):
            assert o.cpu().numpy().tobytes() == oracle.compress_lz4(a).tobytes()
        back = bs.decompress_lz4_batch_dev(outs, [a.shape for a in arrs], torch.int16)
        for t, b in zip(ts, back):
            assert torch.equal(t, b)


def test_host_threads_release_their_buffers(bs, oracle):
    """Each host thread's stream, device buffers and pinned slots are freed
    when the thread exits: 24 short-lived threads leave device memory flat."""
    import torch
    a = oracle.gen_g1(1 << 22)
    want = oracle.compress_lz4(a)
    errors = []

    def run():
        try:
            if bs.compress_lz4(a).tobytes() != want.tobytes():
                errors.append("enc")
            if bs.decompress_lz4(want, a.shape, a.dtype).tobytes() != a.tobytes():
                errors.append("dec")
        except Exception as e:  # pragma: no cover - reported below
            errors.append(repr(e))

    def one_round():
        th = [threading.Thread(target=run) for _ in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    one_round()
    torch.cuda.synchronize()
    free0 = torch.cuda.mem_get_info()[0]
    for _ in range(6):
        one_round()
    torch.cuda.synchronize()
    free1 = torch.cuda.mem_get_info()[0]
    assert not errors, errors[:3]
    # each thread holds ~in + out + workspace (~30 MiB here): 24 leaked
    # threads would take > 600 MiB
    assert free0 - free1 < 128 << 20, (free0 - free1) >> 20
