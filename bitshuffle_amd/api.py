"""numpy / torch front end over the C-ABI.

Host functions mirror bitshuffle/ext.pyx of the reference one for one
(argument names, C-contiguity check, `out=` reuse, RuntimeError("Failed.
Error code %d.", code) on negative returns, and decompress_lz4's check that
the whole input buffer was consumed, ext.pyx:501-504).  Unlike the Cython
wrapper, sizes are 64-bit, so arrays beyond 2**31 elements work.

Device functions take torch tensors that live on a HIP device and enqueue on
the current torch stream (or `stream=`); nothing is copied to the host except
the compressed length when `sync=True`.
"""
import ctypes

import numpy as np

from ._lib import BshufError, lib


def _fail(code, what="Failed. Error code %d."):
    raise BshufError(what % code, int(code))


def _check(code):
    if code < 0:
        _fail(code)
    return code


def _make_array(shape, dtype, out=None):
    # bitshuffle/ext.pyx:124-133
    if out is None:
        return np.empty(shape, dtype=dtype)
    size = int(np.prod(shape))
    base = out if out.base is None else out.base
    return base.ravel().view(dtype)[:size].reshape(shape)


def _setup_arr(arr, out=None):
    # bitshuffle/ext.pyx:136-145
    if not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("Input array must be C-contiguous.")
    return _make_array(tuple(arr.shape), arr.dtype, out), arr.size, arr.dtype.itemsize


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data)


def default_block_size(elem_size):
    return int(lib.bshuf_default_block_size(elem_size))


def compress_lz4_bound(size, elem_size, block_size=0):
    return int(lib.bshuf_compress_lz4_bound(size, elem_size, block_size))


# ---------------------------------------------------------------- host API
def bitshuffle(arr, block_size=0, out=None):
    """Bitshuffle an array (reference bitshuffle/ext.pyx:311-353)."""
    out, size, itemsize = _setup_arr(arr, out)
    _check(lib.bshuf_bitshuffle(_ptr(arr), _ptr(out), size, itemsize, block_size))
    return out


def bitunshuffle(arr, block_size=0, out=None):
    """Undo bitshuffle (reference bitshuffle/ext.pyx:356-398)."""
    out, size, itemsize = _setup_arr(arr, out)
    _check(lib.bshuf_bitunshuffle(_ptr(arr), _ptr(out), size, itemsize, block_size))
    return out


def compress_lz4(arr, block_size=0, out=None):
    """Bitshuffle then LZ4-compress; returns the framed uint8 stream
    (reference bitshuffle/ext.pyx:401-447)."""
    if not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("Input array must be C-contiguous.")
    size, itemsize = arr.size, arr.dtype.itemsize
    bound = compress_lz4_bound(size, itemsize, block_size)
    if bound > (1 << 62):  # the (size_t)-81 quirk of an invalid block size
        _fail(-81)
    out = _make_array((max(bound, 1),), np.uint8, out)
    count = _check(lib.bshuf_compress_lz4(_ptr(arr), _ptr(out), size, itemsize, block_size))
    return out[:count]


def decompress_lz4(arr, shape, dtype, block_size=0, out=None):
    """LZ4-decompress then bitunshuffle (reference bitshuffle/ext.pyx:452-505)."""
    if not arr.flags["C_CONTIGUOUS"]:
        raise ValueError("Input array must be C-contiguous.")
    dtype = np.dtype(dtype)
    size = int(np.prod(shape))
    out = _make_array(tuple(shape), dtype, out)
    count = _check(lib.bshuf_decompress_lz4(_ptr(arr), _ptr(out), size, dtype.itemsize,
                                            block_size))
    if count != arr.size:
        msg = "Decompressed different number of bytes than input buffer size."
        msg += "Input buffer %d, decompressed %d." % (arr.size, count)
        raise BshufError(msg, count)
    return out


# -------------------------------------------------------------- device API
def _torch():
    import torch
    return torch


def _stream(stream):
    torch = _torch()
    if stream is None:
        stream = torch.cuda.current_stream()
    return ctypes.c_void_p(stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream))


def _dptr(t):
    if not t.is_cuda:
        raise ValueError("device functions need a HIP (torch 'cuda') tensor")
    if not t.is_contiguous():
        raise ValueError("Input array must be C-contiguous.")
    return ctypes.c_void_p(t.data_ptr())


def bitshuffle_dev(t, block_size=0, out=None, stream=None):
    out = _torch().empty_like(t) if out is None else out
    _check(lib.bshuf_bitshuffle_dev(_dptr(t), _dptr(out), t.numel(), t.element_size(),
                                    block_size, _stream(stream)))
    return out


def bitunshuffle_dev(t, block_size=0, out=None, stream=None):
    out = _torch().empty_like(t) if out is None else out
    _check(lib.bshuf_bitunshuffle_dev(_dptr(t), _dptr(out), t.numel(), t.element_size(),
                                      block_size, _stream(stream)))
    return out


def compress_lz4_workspace(numel, elem_size, block_size=0, device=None):
    torch = _torch()
    n = int(lib.bshuf_compress_lz4_dev_workspace(numel, elem_size, block_size))
    return torch.empty(max(n, 256), dtype=torch.uint8, device=device or "cuda")


def decompress_lz4_workspace(in_nbytes, numel, elem_size, block_size=0, device=None):
    torch = _torch()
    n = int(lib.bshuf_decompress_lz4_dev_workspace(in_nbytes, numel, elem_size, block_size))
    return torch.empty(max(n, 256), dtype=torch.uint8, device=device or "cuda")


def _elems(t, elem_size):
    """(element count, element size) of tensor t; elem_size overrides the
    dtype's, for element sizes torch has no dtype for (t is then raw bytes)."""
    if elem_size is None:
        return t.numel(), t.element_size()
    nbytes = t.numel() * t.element_size()
    if elem_size <= 0 or nbytes % elem_size:
        raise ValueError("tensor of %d bytes is not a whole number of %d-byte elements"
                         % (nbytes, elem_size))
    return nbytes // elem_size, int(elem_size)


def compress_lz4_dev(t, block_size=0, out=None, workspace=None, result=None, offsets=None,
                     stream=None, sync=True, elem_size=None):
    """Device-resident bshuf_compress_lz4.  Returns the framed stream as a uint8
    tensor view (sync=True), or (out, result) where result is a 1-element int64
    device tensor holding the byte count / error (sync=False).  `elem_size`
    overrides the tensor's element size (any E, e.g. a uint8 tensor of
    7-byte records)."""
    torch = _torch()
    n, es = _elems(t, elem_size)
    bound = compress_lz4_bound(n, es, block_size)
    if bound > (1 << 62):
        _fail(-81)
    if out is None:
        out = torch.empty(max(bound, 1), dtype=torch.uint8, device=t.device)
    if result is None:
        result = torch.empty(1, dtype=torch.int64, device=t.device)
    ws = ctypes.c_void_p(workspace.data_ptr()) if workspace is not None else None
    wsb = workspace.numel() if workspace is not None else 0
    offp = _dptr(offsets) if offsets is not None else None
    _check(lib.bshuf_compress_lz4_dev(_dptr(t), _dptr(out), n, es, block_size, ws, wsb,
                                      _dptr(result), offp, _stream(stream)))
    if not sync:
        return out, result
    count = int(result.item())
    if count < 0:
        _fail(count)
    return out[:count]


def decompress_lz4_dev(buf, shape, dtype, block_size=0, out=None, workspace=None, result=None,
                       offsets=None, stream=None, sync=True, elem_size=None, length=None):
    """Device-resident bshuf_decompress_lz4 of the whole uint8 tensor `buf`
    (its length is the exact stream length).  With `elem_size`, `shape` counts
    elem_size-byte elements and the output is a uint8 tensor of their bytes.
    With `length` (a 1-element int64 DEVICE tensor, e.g. compress_lz4_dev's
    `result` with sync=False), the stream length is read on the device
    (bshuf_decompress_lz4_dev_dlen) and `buf` is only its capacity: nothing
    waits on the host between the two calls."""
    torch = _torch()
    size = 1
    for s in shape:
        size *= int(s)
    if out is None:
        if elem_size is None:
            out = torch.empty(tuple(shape), dtype=dtype, device=buf.device)
        else:
            out = torch.empty(size * int(elem_size), dtype=torch.uint8, device=buf.device)
    es = out.element_size() if elem_size is None else int(elem_size)
    if result is None:
        result = torch.empty(1, dtype=torch.int64, device=buf.device)
    ws = ctypes.c_void_p(workspace.data_ptr()) if workspace is not None else None
    wsb = workspace.numel() if workspace is not None else 0
    offp = _dptr(offsets) if offsets is not None else None
    if length is None:
        _check(lib.bshuf_decompress_lz4_dev(_dptr(buf), buf.numel(), _dptr(out), size,
                                            es, block_size, ws, wsb, _dptr(result),
                                            offp, _stream(stream)))
    else:
        if length.dtype != torch.int64 or length.numel() < 1 or length.device != buf.device:
            raise ValueError("length must be an int64 tensor on the stream's device")
        _check(lib.bshuf_decompress_lz4_dev_dlen(_dptr(buf), _dptr(length), buf.numel(), _dptr(out),
                                                 size, es, block_size, ws, wsb, _dptr(result),
                                                 offp, _stream(stream)))
    if not sync:
        return out, result
    count = int(result.item())
    if count < 0:
        _fail(count)
    want = buf.numel() if length is None else int(length.reshape(-1)[0].item())
    if count != want:
        raise BshufError("Decompressed different number of bytes than input buffer size."
                         "Input buffer %d, decompressed %d." % (want, count)
                         + ("" if length is None else " (buffer capacity %d)" % buf.numel()), count)
    return out


def block_index_dev(buf, size, elem_size, block_size=0, workspace=None, stream=None):
    """The block index of the framed stream in uint8 device tensor `buf` for
    `size` elements of `elem_size` bytes (bshuf_lz4_block_index_dev, the
    decoder's parallel header walk): an int64 tensor of every block's byte
    offset.  Raises BshufError(-91) when the records do not tile the stream,
    -1001 when a block cannot be placed."""
    torch = _torch()
    nb = int(lib.bshuf_lz4_dev_nblocks(size, elem_size, block_size))
    offs = torch.empty(max(nb, 1), dtype=torch.int64, device=buf.device)
    status = torch.empty(1, dtype=torch.int64, device=buf.device)
    ws = ctypes.c_void_p(workspace.data_ptr()) if workspace is not None else None
    wsb = workspace.numel() if workspace is not None else 0
    _check(lib.bshuf_lz4_block_index_dev(_dptr(buf), buf.numel(), size, elem_size, block_size, ws,
                                         wsb, _dptr(offs), _dptr(status), _stream(stream)))
    if int(status.item()) != 0:
        _fail(-91)
    if nb and bool((offs[:nb] == -1).any()):
        _fail(-1001)  # a block the walk could not place (the decoder's code for it)
    return offs[:nb]


def _ptr_array(vals):
    arr = (ctypes.c_void_p * len(vals))(*[ctypes.c_void_p(v) for v in vals])
    return ctypes.cast(arr, ctypes.c_void_p), arr


def _size_array(vals):
    arr = (ctypes.c_size_t * len(vals))(*vals)
    return ctypes.cast(arr, ctypes.c_void_p), arr


def compress_lz4_batch_dev(tensors, block_size=0, outs=None, workspace=None, offsets=None,
                           stream=None, sync=True, elem_size=None):
    """bshuf_compress_lz4_batch_dev over a list of device tensors (same dtype):
    one launch per kernel for all of them.  Returns the list of framed uint8
    streams (sync=True), or (outs, results) with results a device int64 tensor
    of per-stream byte counts / error codes.  `elem_size` overrides the
    tensors' element size (as in compress_lz4_dev)."""
    torch = _torch()
    if not tensors:
        return []
    es = _elems(tensors[0], elem_size)[1]
    sizes = [_elems(t, elem_size)[0] for t in tensors]
    if outs is None:
        outs = [torch.empty(max(compress_lz4_bound(n, es, block_size), 1), dtype=torch.uint8,
                            device=t.device) for n, t in zip(sizes, tensors)]
    for t in tensors:
        if _elems(t, elem_size)[1] != es:
            raise ValueError("all tensors of a batch need the same element size")
        _dptr(t)
    results = torch.empty(len(tensors), dtype=torch.int64, device=tensors[0].device)
    pin, keep1 = _ptr_array([t.data_ptr() for t in tensors])
    pout, keep2 = _ptr_array([o.data_ptr() for o in outs])
    psz, keep3 = _size_array(sizes)
    ws = ctypes.c_void_p(workspace.data_ptr()) if workspace is not None else None
    wsb = workspace.numel() if workspace is not None else 0
    offp = _dptr(offsets) if offsets is not None else None
    _check(lib.bshuf_compress_lz4_batch_dev(pin, pout, psz, len(tensors), es, block_size, ws, wsb,
                                            _dptr(results), offp, _stream(stream)))
    if not sync:
        return outs, results
    counts = results.cpu().tolist()
    for c in counts:
        if c < 0:
            _fail(c)
    return [o[:c] for o, c in zip(outs, counts)]


def decompress_lz4_batch_dev(bufs, shapes, dtype, block_size=0, outs=None, workspace=None,
                             stream=None, sync=True, elem_size=None, lengths=None):
    """bshuf_decompress_lz4_batch_dev: each uint8 device tensor of `bufs` is one
    whole framed stream; returns the decoded tensors (sync=True), or (outs,
    results) with per-stream consumed byte counts / error codes.  With
    `elem_size`, shapes count elem_size-byte elements and the outputs are
    uint8 tensors of their bytes.  With `lengths` (an int64 DEVICE tensor of
    len(bufs), e.g. compress_lz4_batch_dev's results with sync=False), the
    stream lengths are read on the device (bshuf_decompress_lz4_batch_dev_dlen)
    and each buffer is only its stream's capacity."""
    torch = _torch()
    if not bufs:
        return []

    def count(sh):
        c = 1
        for x in sh:
            c *= int(x)
        return c
    if outs is None:
        if elem_size is None:
            outs = [torch.empty(tuple(sh), dtype=dtype, device=b.device) for b, sh in zip(bufs, shapes)]
        else:
            outs = [torch.empty(count(sh) * int(elem_size), dtype=torch.uint8, device=b.device)
                    for b, sh in zip(bufs, shapes)]
    if elem_size is None:
        es = outs[0].element_size()
        sizes = [o.numel() for o in outs]
    else:
        es = int(elem_size)
        sizes = [count(sh) for sh in shapes]
    nbytes = [b.numel() for b in bufs]
    results = torch.empty(len(bufs), dtype=torch.int64, device=bufs[0].device)
    pin, keep1 = _ptr_array([_dptr(b).value or 0 for b in bufs])
    pout, keep2 = _ptr_array([_dptr(o).value or 0 for o in outs])
    psz, keep3 = _size_array(sizes)
    pnb, keep4 = _size_array(nbytes)
    ws = ctypes.c_void_p(workspace.data_ptr()) if workspace is not None else None
    wsb = workspace.numel() if workspace is not None else 0
    if lengths is None:
        _check(lib.bshuf_decompress_lz4_batch_dev(pin, pnb, pout, psz, len(bufs), es, block_size, ws,
                                                  wsb, _dptr(results), _stream(stream)))
    else:
        if lengths.dtype != torch.int64 or lengths.numel() < len(bufs):
            raise ValueError("lengths must be an int64 device tensor with one entry per stream")
        _check(lib.bshuf_decompress_lz4_batch_dev_dlen(pin, _dptr(lengths), pnb, pout, psz, len(bufs),
                                                       es, block_size, ws, wsb, _dptr(results),
                                                       _stream(stream)))
    if not sync:
        return outs, results
    counts = results.cpu().tolist()
    if lengths is not None:
        nbytes = lengths.reshape(-1)[: len(bufs)].cpu().tolist()
    for c, nb in zip(counts, nbytes):
        if c < 0:
            _fail(c)
        if c != nb:
            raise BshufError("Decompressed different number of bytes than input buffer size."
                             "Input buffer %d, decompressed %d." % (nb, c), c)
    return outs


def synth_fill_dev(t, gen, first=0, seed=12345, stream=None):
    """Fill tensor t with synthetic input G0 (int32 ramp), G1 (int16) or G2 (float32)."""
    _check(lib.bshuf_synth_fill_dev(_dptr(t), t.numel(), gen, first, seed, _stream(stream)))
    return t
