"""One stream split across two ranks on the GPU (bitshuffle_amd/split.py):
two processes share cuda:0 (gloo for the one all-gather of piece lengths),
each compresses its shard with the device codec; the pieces joined in rank
order must equal the single-call device stream of the whole input (itself
checked against the oracle at this size) and each piece must decode on the
device to its shard."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

@pytest.fixture(scope="module")
def torch():
    import torch
    assert torch.cuda.is_available()
    return torch


SIZE = 3 * 1024 * 1024 + 4096 * 3 + 1005  # int16 elements: blocks split 2 ways + partial + tail


def _worker(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bitshuffle_amd as B
        from bitshuffle_amd.split import (compress_lz4_split, decompress_lz4_split, gather_stream,
                                          shard_bounds)
        x = torch.empty(SIZE, dtype=torch.int16, device="cuda")
        B.synth_fill_dev(x, 1)
        s, e = shard_bounds(SIZE, 2, world)[rank]
        piece, off, total, lengths = compress_lz4_split(x[s:e].contiguous())
        stream = gather_stream(piece, lengths)
        back = decompress_lz4_split(piece, (e - s,), torch.int16)
        ok = bool(torch.equal(back, x[s:e]))
        whole = None
        if rank == 0:
            whole = B.compress_lz4_dev(x).cpu().numpy().tobytes()
        q.put((rank, off, total, lengths, None if stream is None else stream.numpy().tobytes(),
               whole, ok))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_split_stream_on_device_equals_single_stream():
    from oracle import Oracle
    o = Oracle()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        res = sorted((q.get(timeout=150) for _ in range(2)), key=lambda r: r[0])
    finally:
        for p in procs:
            p.join(timeout=60)
    r0 = res[0]
    assert r0[5] == o.compress_lz4(o.gen_g1(SIZE)).tobytes()  # single device stream == oracle
    assert r0[4] == r0[5]  # joined pieces == the single stream
    assert r0[2] == len(r0[5]) and r0[3] == res[1][3] and res[1][1] == r0[3][0]
    assert r0[6] and res[1][6]


def test_split_stream_from_block_index(torch):
    """A whole device stream split by its block index (block_index_dev): the
    index equals the encoder's own offsets, and every rank's byte range
    decodes to its shard."""
    import bitshuffle_amd as B
    from bitshuffle_amd.api import block_index_dev
    from bitshuffle_amd.split import decompress_lz4_split, split_stream
    x = torch.empty(SIZE, dtype=torch.int16, device="cuda")
    B.synth_fill_dev(x, 1)
    nb = int(B.lib.bshuf_lz4_dev_nblocks(SIZE, 2, 0))
    enc_offs = torch.empty(nb, dtype=torch.int64, device="cuda")
    c = B.compress_lz4_dev(x, offsets=enc_offs)
    assert torch.equal(block_index_dev(c, SIZE, 2), enc_offs)
    for world in (2, 3, 5):
        for (s, e), (b0, b1) in split_stream(c, SIZE, 2, world):
            y = decompress_lz4_split(c[b0:b1], (e - s,), torch.int16)
            assert torch.equal(y, x[s:e]), (world, s, e)
    bad = c.clone()
    bad[4096] ^= 0x55
    bad[0:4] = 0  # first record length 0: the walk cannot tile the stream
    with pytest.raises(B.BshufError):
        block_index_dev(bad, SIZE, 2)


@pytest.mark.parametrize("size,worlds", [(3 * 4096 + 5, (4, 5)), (2 * 4096 + 3, (3, 4)), (5, (2,))])
def test_split_stream_tail_only_rank(torch, size, worlds):
    """size % bs < 8 and more ranks than blocks: the last rank owns only the
    raw tail (no record); its byte range is the stream's last (size % 8) * E
    bytes (src/bitshuffle_core.c:1909-1926).  Stream checked against the oracle."""
    import bitshuffle_amd as B
    from oracle import Oracle
    from bitshuffle_amd.split import decompress_lz4_split, split_stream
    x = torch.empty(size, dtype=torch.int16, device="cuda")
    B.synth_fill_dev(x, 1)
    c = B.compress_lz4_dev(x)
    assert c.cpu().numpy().tobytes() == Oracle().compress_lz4(x.cpu().numpy()).tobytes()
    for world in worlds:
        rng = split_stream(c, size, 2, world)
        assert rng[-1][1] == (c.numel() - (size % 8) * 2, c.numel()) or size // 4096 >= world
        assert rng[0][1][0] == 0 and all(rng[i][1][1] == rng[i + 1][1][0] for i in range(world - 1))
        for (s, e), (b0, b1) in rng:
            y = decompress_lz4_split(c[b0:b1], (e - s,), torch.int16)
            assert torch.equal(y, x[s:e]), (world, s, e)


def _rccl_worker(port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        import bitshuffle_amd as B
        from bitshuffle_amd.split import (compress_lz4_split, decompress_lz4_split, gather_stream,
                                          shard_bounds)
        size = 3 * 4096 + 5
        x = torch.empty(size, dtype=torch.int16, device="cuda")
        B.synth_fill_dev(x, 1)
        s, e = shard_bounds(size, 2, 1)[0]
        piece, off, total, lengths = compress_lz4_split(x[s:e].contiguous())
        stream = gather_stream(piece, lengths)
        back = decompress_lz4_split(piece, (e - s,), torch.int16)
        q.put((dist.get_backend(), off, total, lengths, stream.numpy().tobytes(),
               B.compress_lz4_dev(x).cpu().numpy().tobytes(), bool(torch.equal(back, x))))
    finally:
        dist.destroy_process_group()


def test_split_collectives_on_rccl_world1():
    """The RCCL ("nccl" backend) branch of split.py's collectives on device
    tensors -- the all-gather of piece lengths and the gather to rank 0 -- at
    world 1 (one GPU on this box; the gloo tests above cover worlds 2-5)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    try:
        backend, off, total, lengths, stream, whole, ok = q.get(timeout=150)
    finally:
        p.join(timeout=60)
    assert backend == "nccl" and off == 0 and lengths == [len(whole)] and total == len(whole)
    assert stream == whole and ok
