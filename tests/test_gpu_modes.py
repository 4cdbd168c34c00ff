"""Odd element sizes and large blocks at scale, pinned to the REFERENCE.

tests/golden/vectors.json "modes" holds the length + SHA-256 of the
reference's own bshuf_compress_lz4 output (oracle/_ref, compiled from
/root/reference; tests/golden/make_vectors.py --modes) for G1 int16 bytes
re-read as 3- and 12-byte elements and for 256 KiB blocks.  The 1 GiB cases
are exactly tools/ab.py's AB_ELEM workload.

Round 4's gpurun_out/r4o run got -1001 from decompress_lz4_dev on such a
stream.  Its (uncommitted) ab.py passed `x.shape` of the uint8 byte view
together with elem_size=E: `size` was the BYTE count, E times the element
count.  That moves the raw tail ((size % 8) * E bytes) and so the end of the
framed region, and asks for E times the blocks the stream holds; the index
rebuild leaves the missing blocks unresolved, which the header check reports
as -1001.  test_r4o_wrong_size_is_rejected replays that call and pins the
code; the same bytes with the right size decode exactly.
"""
import hashlib

import pytest

from tests.vectors import load_vectors

pytestmark = pytest.mark.gpu


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


def _digest(torch, t, nbytes=None):
    u8 = t.reshape(-1).view(torch.uint8)
    nbytes = u8.numel() if nbytes is None else nbytes
    h = hashlib.sha256()
    step = 1 << 28
    for i in range(0, nbytes, step):
        h.update(u8[i:min(i + step, nbytes)].cpu().numpy().tobytes())
    return h.hexdigest()


def _mode_input(bs, torch, spec):
    """G1 int16 generated on the device, its first nbytes as raw bytes."""
    x = torch.empty(spec["n"], dtype=torch.int16, device="cuda")
    bs.synth_fill_dev(x, 1, seed=spec.get("seed", 12345))
    return x.view(torch.uint8)[: spec["nbytes"]]


MODES_1G = ["mode_ab_g1_1GiB_E3", "mode_ab_g1_1GiB_E12", "mode_g1_1GiB_E2_bs131072"]


@pytest.mark.parametrize("name", MODES_1G)
def test_mode_streams_match_reference_digest(bs, torch, name):
    """compress_lz4_dev -> reference length + SHA-256; decompress_lz4_dev with
    the index rebuilt from the framing (no encoder offsets) -> exact bytes."""
    spec = {e["name"]: e for e in load_vectors()["modes"]}[name]
    x = _mode_input(bs, torch, spec)
    assert _digest(torch, x) == spec["input_sha256"]
    E, bsz = spec["elem_size"], spec["bs"]
    c = bs.compress_lz4_dev(x, block_size=bsz, elem_size=E)
    assert c.numel() == spec["compressed_len"], name
    assert _digest(torch, c) == spec["compressed_sha256"], name
    y = bs.decompress_lz4_dev(c, (spec["size"],), torch.uint8, block_size=bsz, elem_size=E)
    assert torch.equal(y.view(torch.uint8), x), name


@pytest.mark.parametrize("E", [3, 12])
def test_r4o_wrong_size_is_rejected(bs, torch, E):
    """The r4o call: `shape` of the byte view (size = bytes, not elements)."""
    spec = {e["name"]: e for e in load_vectors()["modes"]}["mode_ab_g1_1GiB_E%d" % E]
    x = _mode_input(bs, torch, spec)
    c = bs.compress_lz4_dev(x, elem_size=E)
    assert c.numel() == spec["compressed_len"]
    with pytest.raises(bs.BshufError) as ei:
        bs.decompress_lz4_dev(c, x.shape, x.dtype, elem_size=E)
    assert ei.value.args[1] == -1001
    y = bs.decompress_lz4_dev(c, (x.numel() // E,), x.dtype, elem_size=E)
    assert torch.equal(y, x)
    del y
    torch.cuda.empty_cache()
