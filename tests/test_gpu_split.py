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
