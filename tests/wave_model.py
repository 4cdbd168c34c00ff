"""Lane-vectorised model of the HIP encoder's wave-parallel LZ4 parse.

Test infrastructure: it mirrors, step by step, what k_lz4_encode in
bitshuffle_amd/csrc/lz4_encode.hip does with 64 lanes (probe windows, the
tentative-insert collision check, group resolution, table fix-up, ballot-based
catch-up / match count), so the algorithm can be checked against the oracle
on CPU in seconds.  Every "lane" array has 64 entries; ballot() packs a bool
array into a python int bitmask.
"""
import numpy as np

W = 64
LANES = np.arange(W)


def sched(k):
    """Offset of probe k from the search start (step = 1 for k<65, then
    (63+k)>>6), i.e. the skip-acceleration of lz4/lz4.c:1042-1053 in closed form."""
    k = np.asarray(k, dtype=np.int64)
    t = 62 + k
    q = t >> 6
    r = t & 63
    g = 32 * q * (q - 1) + q * (r + 1)
    return np.where(k == 0, 0, 1 + g)


def ballot(b):
    m = 0
    for i, v in enumerate(np.asarray(b)):
        if v:
            m |= 1 << i
    return m


def ffs(m):
    return (m & -m).bit_length() - 1


def rd32(D, p):
    p = np.asarray(p)
    return (D[p].astype(np.uint32) | (D[p + 1].astype(np.uint32) << 8) |
            (D[p + 2].astype(np.uint32) << 16) | (D[p + 3].astype(np.uint32) << 24))


def hash4(v):
    return ((v.astype(np.uint64) * 2654435761) & 0xFFFFFFFF) >> 19


def put_len(out, v):
    while v >= 255:
        out.append(255)
        v -= 255
    out.append(v)


def encode_block(src):
    n = len(src)
    D = np.zeros(n + 8 + 256, dtype=np.uint8)
    D[:n] = src
    T = np.zeros(8192, dtype=np.int64)
    out = []
    anchor = 0
    if n >= 13:
        limit = n - 11
        mlimit = n - 5
        ip = 1
        while True:
            # ---------------- search windows ----------------
            p0 = ip
            k0 = 0
            found = None
            while True:
                kk = k0 + LANES
                pos = p0 + sched(kk)
                nxt = p0 + sched(kk + 1)
                valid = nxt <= limit
                vmask = ballot(valid)
                if vmask == 0:
                    break
                posc = np.where(valid, pos, 0)
                seq = rd32(D, posc)
                h = hash4(seq).astype(np.int64)
                cold = T[h].copy()
                # tentative insert: the hardware keeps ONE of the same-address
                # writes; model an arbitrary winner (reverse order here)
                for l in range(W - 1, -1, -1):
                    if valid[l]:
                        T[h[l]] = pos[l]
                rb = T[h]
                loser = valid & (rb != pos)
                cand = cold.copy()
                grouped = np.zeros(W, bool)
                first = np.ones(W, bool)
                nextm = np.full(W, W)
                lmask = ballot(loser)
                while lmask:
                    l = int(ffs(lmask))
                    hl = h[l]
                    ing = valid & (h == hl)
                    g = ballot(ing)
                    for j in map(int, np.nonzero(ing)[0]):
                        grouped[j] = True
                        below = g & ((1 << j) - 1)
                        if below:
                            pl = below.bit_length() - 1
                            cand[j] = p0 + sched(k0 + pl)
                            first[j] = False
                        above = g & ~((2 << j) - 1) & ((1 << W) - 1)
                        nextm[j] = ffs(above) if above else W
                    lmask &= ~g
                ok = valid & (rd32(D, cand) == seq)
                mm = ballot(ok)
                if mm:
                    js = ffs(mm)
                    for j in range(W):
                        if not valid[j]:
                            continue
                        if not grouped[j]:
                            if j > js:
                                T[h[j]] = cold[j]
                        else:
                            if j <= js and nextm[j] > js:
                                T[h[j]] = pos[j]
                            elif first[j] and j > js:
                                T[h[j]] = cold[j]
                    found = (int(pos[js]), int(cand[js]))
                    break
                if vmask != (1 << W) - 1:
                    break
                for j in range(W):
                    if grouped[j] and nextm[j] == W:
                        T[h[j]] = pos[j]
                k0 += W
            if found is None:
                break  # last literals
            ip, mt = found
            # ---------------- catch-up ----------------
            while True:
                a = ip - 1 - LANES
                b = mt - 1 - LANES
                c = (a >= anchor) & (b >= 0)
                c &= D[np.maximum(a, 0)] == D[np.maximum(b, 0)]
                cm = ballot(c)
                inv = ~cm & ((1 << W) - 1)
                run = ffs(inv) if inv else W
                ip -= run
                mt -= run
                if run < W:
                    break
            lit = ip - anchor
            tokpos = len(out)
            out.append(0)
            tok = min(lit, 15) << 4
            if lit >= 15:
                put_len(out, lit - 15)
            out.extend(int(x) for x in D[anchor:ip])
            while True:
                off = ip - mt
                out.append(off & 255)
                out.append(off >> 8)
                total = 0
                while True:
                    pa = ip + 4 + total + 4 * LANES
                    pb = mt + 4 + total + 4 * LANES
                    pac = np.minimum(pa, n)
                    pbc = np.minimum(pb, n)
                    x = rd32(D, pac) ^ rd32(D, pbc)
                    eq = np.where(x == 0, 4, np.array([(int(v) & -int(v)).bit_length() - 1 if v else 0
                                                       for v in x]) >> 3)
                    avail = mlimit - pa
                    eq = np.minimum(eq, np.maximum(avail, 0))
                    fm = ballot(eq == 4)
                    if fm == (1 << W) - 1:
                        total += 4 * W
                        continue
                    f = ffs(~fm & ((1 << W) - 1))
                    total += 4 * f + int(eq[f])
                    break
                mc = total
                ip += mc + 4
                tok |= min(mc, 15)
                out[tokpos] = tok
                if mc >= 15:
                    put_len(out, mc - 15)
                anchor = ip
                if ip >= limit:
                    break
                hA = int(hash4(rd32(D, np.array([ip - 2])))[0])
                hB = int(hash4(rd32(D, np.array([ip])))[0])
                T[hA] = ip - 2
                c2 = int(T[hB])
                T[hB] = ip
                if int(rd32(D, np.array([c2]))[0]) == int(rd32(D, np.array([ip]))[0]):
                    tokpos = len(out)
                    out.append(0)
                    tok = 0
                    mt = c2
                    continue
                break
            if anchor >= limit:
                break
            ip = ip + 1
    run = n - anchor
    out.append(min(run, 15) << 4)
    if run >= 15:
        put_len(out, run - 15)
    out.extend(int(x) for x in D[anchor:n])
    return bytes(out)
