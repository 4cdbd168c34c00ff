"""One stream split across ranks (bitshuffle_amd/split.py):
shard bounds, the offset scan, and world-2/3 gloo runs on the CPU with the
oracle as the codec -- the pieces joined in rank order must be the oracle's
stream of the whole input byte for byte, and each piece must decode to its
shard.  The device codec at world 2 is in tests/test_gpu_split.py."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from bitshuffle_amd.split import shard_bounds, stream_offsets


def test_shard_bounds_whole_blocks_and_tail():
    size, E, bs = 10 * 4096 + 1005, 2, 4096
    b = shard_bounds(size, E, 3, bs)
    assert b[0][0] == 0 and b[-1][1] == size
    assert all(b[i][1] == b[i + 1][0] for i in range(2))
    assert all((e - s) % bs == 0 for s, e in b[:-1])
    assert [(e - s) // bs for s, e in b[:-1]] == [4, 3]  # 10 blocks: 4, 3, 3 + partial + tail
    # default block size, fewer blocks than ranks: leading ranks empty-or-whole
    b = shard_bounds(3 * 4096 + 7, 2, 8)
    assert [e - s for s, e in b][:3] == [4096, 4096, 4096] and b[-1] == (3 * 4096, 3 * 4096 + 7)
    assert sum(e - s for s, e in b) == 3 * 4096 + 7
    with pytest.raises(ValueError):
        shard_bounds(100, 2, 2, 12)


def test_stream_offsets():
    assert stream_offsets([5, 0, 7]) == ([0, 5, 5], 12)
    with pytest.raises(ValueError):
        stream_offsets([3, -91])


def _oracle_codec():
    from oracle import Oracle
    o = Oracle()
    return (lambda a, bs: o.compress_lz4(a, bs),
            lambda p, shape, dt, bs: o.decompress_lz4(np.asarray(p), shape, dt, bs))


def _worker(rank, world, port, size, bs, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from oracle import Oracle
        from bitshuffle_amd.split import compress_lz4_split, decompress_lz4_split, gather_stream
        whole = Oracle().gen_g1(size)
        s, e = shard_bounds(size, 2, world, bs)[rank]
        codec = _oracle_codec()
        piece, off, total, lengths = compress_lz4_split(whole[s:e], bs, codec=codec)
        stream = gather_stream(piece, lengths)
        back = decompress_lz4_split(piece, (e - s,), np.int16, bs, codec=codec)
        q.put((rank, off, total, lengths, None if stream is None else stream.numpy().tobytes(),
               bool(np.array_equal(back, whole[s:e]))))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,size,bs", [(2, 9 * 4096 + 1005, 4096), (3, 2 * 4096 + 13, 4096),
                                           (3, 20 * 512 + 3, 512), (4, 3 * 4096 + 5, 4096)])
def test_split_stream_equals_single_stream(world, size, bs):
    from oracle import Oracle
    want = Oracle().compress_lz4(Oracle().gen_g1(size), bs).tobytes()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, size, bs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
    lengths = res[0][3]
    assert sum(lengths) == len(want) and all(r[2] == len(want) for r in res)
    assert [r[1] for r in res] == stream_offsets(lengths)[0]
    assert res[0][4] == want  # joined pieces == the single stream, byte for byte
    assert all(r[5] for r in res)  # every piece decodes to its shard


@pytest.mark.parametrize("size,worlds", [
    (9 * 4096 + 1005, (1, 2, 3, 4, 12)),
    # size % bs < 8: no partial block, the last rank owns only the raw tail
    # whenever the world exceeds the block count
    (3 * 4096 + 5, (1, 2, 3, 4, 5, 7)),
    (2 * 4096 + 3, (2, 3, 4)),
    (5, (1, 2, 3)),  # no block at all: the stream is the raw tail
])
def test_piece_ranges_from_block_index(size, worlds):
    """Byte ranges from a block index equal the compress-side piece offsets
    (oracle stream, its record headers walked on the host as the index)."""
    from oracle import Oracle
    from bitshuffle_amd.split import piece_ranges
    o = Oracle()
    bs = 4096
    x = o.gen_g1(size)
    stream = o.compress_lz4(x, bs)
    offs, p = [], 0
    for _ in range(size // bs + (1 if size % bs >= 8 else 0)):
        offs.append(p)
        p += 4 + int.from_bytes(stream[p:p + 4].tobytes(), "big")
    for world in worlds:
        bounds = shard_bounds(size, 2, world, bs)
        pieces = [o.compress_lz4(x[s:e], bs).size if e > s else 0 for s, e in bounds]
        want_offs, total = stream_offsets(pieces)
        got = piece_ranges(offs, bounds, stream.size, 2, bs)
        assert [g[0] for g in got] == want_offs and got[-1][1] == total == stream.size
        assert [g[1] - g[0] for g in got] == pieces
        # every piece decodes to its shard, and the pieces join to the stream
        for (s, e), (b0, b1) in zip(bounds, got):
            if e > s:
                back = o.decompress_lz4(stream[b0:b1], (e - s,), np.int16, bs)
                assert np.array_equal(back, x[s:e])


def test_compress_split_rejects_ragged_shard():
    """A rank other than the last must hold whole blocks; a torch.chunk-style
    split would make pieces that do not join into one stream."""
    import torch.distributed as dist
    from bitshuffle_amd import split as sp
    if dist.is_initialized():
        pytest.skip("needs no default group")
    orig = (dist.is_initialized, dist.get_rank, dist.get_world_size)
    dist.is_initialized = lambda: True
    dist.get_rank = lambda group=None: 0
    dist.get_world_size = lambda group=None: 2
    try:
        with pytest.raises(ValueError, match="whole number"):
            sp.compress_lz4_split(np.zeros(4096 + 8, np.int16), 4096, codec=_oracle_codec())
    finally:
        dist.is_initialized, dist.get_rank, dist.get_world_size = orig
