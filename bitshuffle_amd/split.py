"""One bitshuffle+LZ4 stream split across ranks (last bullet).

A framed stream is its blocks' records in block order, then the partial
block's record, then the raw `size % 8` tail (`bshuf_blocked_wrap_fun`,
src/bitshuffle_core.c:1877-1931; `bshuf_compress_lz4_block`,
src/bitshuffle.c:36-79).  Blocks are independent, so when every rank but the
last holds a whole number of blocks of the input, each rank compresses its
shard on its own GPU with the ordinary device call and the shards' streams,
concatenated in rank order, ARE the single stream of the whole input, byte for
byte.  The only exchange is one all-gather of the per-rank compressed byte
counts; its exclusive scan is each rank's offset in the stream.  Decoding runs
the same way backwards: rank r decodes bytes [offset_r, offset_r + length_r)
as a stream of its own shard's size.  A stream whose piece boundaries were
not kept (read back from a file, say) is split with its block index
(`piece_ranges` over `block_index_dev`, the decoder's parallel header walk
alone): rank r's piece starts at its first block's offset.

`shard_bounds` splits the blocks as evenly as possible; the last rank also
takes the partial block and the tail (the reference's layout puts them at the
end).  A rank may own nothing (fewer blocks than ranks): it compresses nothing
and its piece is empty.

The codec is the device API (`compress_lz4_dev` / `decompress_lz4_dev`) unless
a caller passes its own pair (the CPU tests pass the oracle's, as the
checker).  Collectives go through `torch.distributed` on the default group:
RCCL (backend "nccl") for device tensors, gloo on the CPU.
"""
from .api import default_block_size

__all__ = ["shard_bounds", "stream_offsets", "compress_lz4_split", "decompress_lz4_split",
           "gather_stream", "piece_ranges", "split_stream"]


def shard_bounds(size, elem_size, world, block_size=0):
    """[(start, end)] element ranges of the `world` shards of a `size`-element
    input: whole blocks, split as evenly as possible (the first `nblk % world`
    ranks one block more), the last rank also the partial block and tail."""
    if world < 1:
        raise ValueError("world must be >= 1")
    bs = block_size or default_block_size(elem_size)
    if bs <= 0 or bs % 8:
        raise ValueError("block_size must be a positive multiple of 8")
    nblk = size // bs
    per, extra = divmod(nblk, world)
    out, start = [], 0
    for r in range(world):
        end = start + (per + (1 if r < extra else 0)) * bs
        if r == world - 1:
            end = size
        out.append((start, end))
        start = end
    return out


def stream_offsets(lengths):
    """Exclusive scan of the per-rank compressed byte counts: (offsets, total)."""
    offs, acc = [], 0
    for n in lengths:
        if n < 0:
            raise ValueError("a rank reported error %d" % n)
        offs.append(acc)
        acc += int(n)
    return offs, acc


def _all_lengths(n, group=None, device=None):
    """All ranks' int64 values of n (one all-gather of one int64 per rank)."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return [int(n)]
    world = dist.get_world_size(group)
    if dist.get_backend(group) == "nccl":
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    else:
        dev = torch.device("cpu")
    mine = torch.tensor([int(n)], dtype=torch.int64, device=dev)
    allv = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(allv, mine, group=group)
    return [int(v) for v in allv.cpu().tolist()]


def compress_lz4_split(shard, block_size=0, elem_size=None, group=None, codec=None):
    """Compress this rank's shard (see `shard_bounds`) of one stream.

    Returns (piece, offset, total, lengths): this rank's bytes of the single
    stream, where they start in it, its total length, and every rank's piece
    length.  Collective over `group` (every rank must call it)."""
    import torch.distributed as dist
    rank, world = ((dist.get_rank(group), dist.get_world_size(group))
                   if dist.is_available() and dist.is_initialized() else (0, 1))
    if rank != world - 1:
        esz = elem_size if elem_size is not None else (
            shard.element_size() if hasattr(shard, "element_size") else shard.dtype.itemsize)
        nel = (shard.numel() * shard.element_size() // esz) if hasattr(shard, "numel") else shard.size
        bs = block_size or default_block_size(esz)
        if nel % bs:
            raise ValueError("rank %d of %d holds %d elements, not a whole number of %d-element "
                             "blocks: the joined pieces would not be one stream (use shard_bounds)"
                             % (rank, world, nel, bs))
    if codec is None:
        import torch
        from .api import compress_lz4_dev
        n = shard.numel() if elem_size is None else shard.numel() * shard.element_size() // elem_size
        if n == 0:
            piece = torch.empty(0, dtype=torch.uint8, device=shard.device)
        else:
            piece = compress_lz4_dev(shard, block_size, elem_size=elem_size)
        length, dev = piece.numel(), piece.device
    else:
        piece = codec[0](shard, block_size)
        length, dev = len(piece), None
    lengths = _all_lengths(length, group, dev)
    offs, total = stream_offsets(lengths)
    return piece, offs[rank], total, lengths


def decompress_lz4_split(piece, shape, dtype, block_size=0, elem_size=None, codec=None):
    """Decode this rank's piece of a split stream into its shard (shape /
    dtype of the shard; `elem_size` as in decompress_lz4_dev).  No exchange:
    the piece boundaries are the compress side's offsets."""
    size = 1
    for s in shape:
        size *= int(s)
    if codec is not None:
        return codec[1](piece, shape, dtype, block_size)
    if size == 0:
        import torch
        if elem_size is None:
            return torch.empty(tuple(shape), dtype=dtype, device=piece.device)
        return torch.empty(0, dtype=torch.uint8, device=piece.device)
    from .api import decompress_lz4_dev
    return decompress_lz4_dev(piece, shape, dtype, block_size, elem_size=elem_size)


def gather_stream(piece, lengths, dst=0, group=None):
    """The whole stream on rank `dst` (a uint8 CPU tensor; None elsewhere):
    every piece padded to the longest, one gather to `dst` (only `dst` holds
    world x the longest piece), trimmed and joined in rank order."""
    import torch
    import torch.distributed as dist
    if not dist.is_available() or not dist.is_initialized():
        return piece.detach().to("cpu") if isinstance(piece, torch.Tensor) else torch.as_tensor(piece)
    world = dist.get_world_size(group)
    nccl = dist.get_backend(group) == "nccl"
    dev = piece.device if nccl and isinstance(piece, torch.Tensor) else torch.device("cpu")
    mx = max(max(lengths), 1)
    buf = torch.zeros(mx, dtype=torch.uint8, device=dev)
    mine = piece if isinstance(piece, torch.Tensor) else torch.as_tensor(piece)
    buf[: mine.numel()] = mine.to(dev).reshape(-1)
    if dist.get_rank(group) != dst:
        dist.gather(buf, None, dst=dst, group=group)
        return None
    parts = [torch.empty(mx, dtype=torch.uint8, device=dev) for _ in range(world)]
    dist.gather(buf, parts, dst=dst, group=group)
    return torch.cat([parts[r][: lengths[r]].cpu() for r in range(world)])


def piece_ranges(block_offsets, bounds, stream_len, elem_size, block_size=0):
    """[(start, end)] byte ranges of each rank's piece of one stream, from the
    stream's block index (every block's byte offset, e.g. `block_index_dev`)
    and the element `bounds` of `shard_bounds`."""
    bs = block_size or default_block_size(elem_size)
    offs = [int(v) for v in block_offsets]
    starts = []
    for s, e in bounds:
        k = s // bs
        if e <= s:
            starts.append(None)  # owns nothing: empty piece at the next start
        elif k < len(offs):
            starts.append(offs[k])
        else:
            # no record at all, only the raw `size % 8` tail (no partial block:
            # size % bs < 8); the reference writes it after the last record
            # (src/bitshuffle_core.c:1909-1926), so it is the stream's end.
            starts.append(stream_len - (e - s) * elem_size)
    out = []
    nxt = stream_len
    for r in range(len(bounds) - 1, -1, -1):
        st = starts[r] if starts[r] is not None else nxt
        out.append((st, nxt))
        nxt = st
    return out[::-1]


def split_stream(buf, size, elem_size, world, block_size=0):
    """Every rank's (element range, byte range) of the framed stream in device
    tensor `buf` of `size` elements, from its block index: what a rank decodes
    with `decompress_lz4_split(buf[b0:b1], ...)` when the compress side's piece
    lengths are not at hand."""
    from .api import block_index_dev
    bounds = shard_bounds(size, elem_size, world, block_size)
    offs = block_index_dev(buf, size, elem_size, block_size).cpu().tolist()
    return list(zip(bounds, piece_ranges(offs, bounds, buf.numel(), elem_size, block_size)))
