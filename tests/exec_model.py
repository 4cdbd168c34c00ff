"""Lane-level numpy model of the decoder's phase 2 (lz4_exec_block in
bitshuffle_amd/csrc/lz4_decode.hip), used by the CPU tests to check the
batching rule against the oracle without a GPU.

One 64-lane chunk of sequences at a time: every lane decodes its sequence
from its token position, a prefix sum places the sequences, all literal runs
are copied (<= 16 bytes by the lane itself, longer ones by the whole wave),
then the matches run in batches of consecutive sequences whose sources end
before the batch's first output byte (only the batch head may overlap
itself).  Within one wave instruction every lane reads before any lane
writes, which the model reproduces by gathering a batch's sources first.
"""
import numpy as np

WAVE = 64
MINMATCH = 4


def _ext(C, q):
    add = 0
    while True:
        b = int(C[q])
        q += 1
        add += b
        if b != 255:
            return add, q


def decode_fields(C, tp, last):
    """(lit, lit_src, off, ml) of the sequence whose token is at C[tp]."""
    tok = int(C[tp])
    lit, q = tok >> 4, tp + 1
    if lit == 15:
        add, q = _ext(C, q)
        lit += add
    lsrc = q
    q += lit
    off = ml = 0
    if not last:
        off = int(C[q]) | (int(C[q + 1]) << 8)
        q += 2
        ml = tok & 15
        if ml == 15:
            add, q = _ext(C, q)
            ml += add
        ml += MINMATCH
    return lit, lsrc, off, ml


def wave_fill(D, op, off, ml):
    """Whole-wave self-overlapping match (off < ml) or offset 0 (zeros)."""
    if off == 0:
        D[op:op + ml] = 0
        return
    if off >= WAVE:
        for c in range(0, ml, WAVE):  # each 64-byte chunk reads earlier chunks
            k = min(WAVE, ml - c)
            D[op + c:op + c + k] = D[op - off + c:op - off + c + k].copy()
        return
    for i in range(ml):  # periodic: D[op+i] = D[op-off + i % off]
        D[op + i] = D[op - off + i % off]


def exec_block(C, positions, n):
    """Replays lz4_exec_block; C = record payload, positions = the scan's
    token positions.  Returns the decoded block (n bytes)."""
    D = np.zeros(n + 64, dtype=np.uint8)
    nseq = len(positions)
    opb = 0
    for c0 in range(0, nseq, WAVE):
        lanes = []
        for j in range(c0, min(c0 + WAVE, nseq)):
            lanes.append(decode_fields(C, int(positions[j]), j + 1 == nseq))
        lens = [lit + ml for lit, _, _, ml in lanes]
        ops = list(np.cumsum([0] + lens)[:-1] + opb)
        opb += sum(lens)
        # literals: independent of everything in this chunk
        for (lit, lsrc, _, _), op in zip(lanes, ops):
            D[op:op + lit] = C[lsrc:lsrc + lit]
        mop = [op + lit for (lit, _, _, _), op in zip(lanes, ops)]
        todo = [i for i, (_, _, _, ml) in enumerate(lanes) if ml > 0]
        while todo:
            f = todo[0]
            opf = mop[f]
            g = len(lanes)
            for i in range(f + 1, len(lanes)):
                _, _, off, ml = lanes[i]
                if ml > 0 and (off < ml or mop[i] - off + ml > opf):
                    g = i
                    break
            batch = [i for i in range(f, g) if lanes[i][3] > 0]
            # one instruction: all lanes read, then all write
            srcs = {}
            for i in batch:
                _, _, off, ml = lanes[i]
                if off >= ml:
                    srcs[i] = D[mop[i] - off:mop[i] - off + ml].copy()
            for i in batch:
                _, _, off, ml = lanes[i]
                if i in srcs:
                    D[mop[i]:mop[i] + ml] = srcs[i]
                else:
                    assert i == f, "only the batch head may overlap itself"
                    wave_fill(D, mop[i], off, ml)
            todo = [i for i in todo if i >= g]
    assert opb == n, (opb, n)
    return D[:n].copy()
