"""TEST/ANALYSIS (uses the oracle as the checker). Compact-hash-table feasibility for the byU16 LZ4 parse (round-6 DESIGN 6.0):
a pure-Python LZ4_compress_default (byU16, hash4, acceleration 1) logging every
table get / put, checked against the oracle's block compressor, then the log
replayed against compact tables to count the blocks an exact compact scheme
would have to send back to the dense 16 KiB table."""
import sys, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from oracle import Oracle
o = Oracle()
K = 2654435761

def h4(b, p):
    x = int.from_bytes(b[p:p+4], 'little')
    return ((x * K) & 0xFFFFFFFF) >> 19

def lz4_log(b):
    n = len(b); log = []; seqs = []
    tab = [0]*8192
    def get(h): log.append(('g', h)); return tab[h]
    def put(h, v): log.append(('p', h)); tab[h] = v
    anchor = 0
    if n < 13:
        pass
    else:
        limit = n - 12 + 1; mlimit = n - 5
        put(h4(b, 0), 0); ip = 1
        while True:
            fwd = ip; step = 1; nbm = 64
            while True:
                cur = fwd; h = h4(b, cur); cand = get(h)
                ip = fwd; fwd += step; step = nbm >> 6; nbm += 1
                if fwd > limit: ip = None; break
                put(h, cur)
                if b[cand:cand+4] == b[ip:ip+4]: match = cand; break
            if ip is None: break
            while ip > anchor and match > 0 and b[ip-1] == b[match-1]: ip -= 1; match -= 1
            while True:
                a = ip + 4; c = match + 4
                while a < mlimit and b[a] == b[c]: a += 1; c += 1
                seqs.append((ip - anchor, ip - match, a - ip))
                ip = a; anchor = ip
                if ip >= limit: break
                put(h4(b, ip-2), ip-2)
                h = h4(b, ip); cand = get(h); put(h, ip)
                if b[cand:cand+4] == b[ip:ip+4]: match = cand; continue
                break
            if ip >= limit: break
            ip += 1
    return log, seqs


def oracle_seqs(c):
    """(literals, offset, match length) of every sequence of an LZ4 block"""
    q, seqs = 0, []
    while q < len(c):
        t = c[q]; q += 1; lit = t >> 4
        if lit == 15:
            while True:
                x = c[q]; q += 1; lit += x
                if x != 255: break
        q += lit
        if q >= len(c): break
        off = c[q] | (c[q + 1] << 8); q += 2; ml = t & 15
        if ml == 15:
            while True:
                x = c[q]; q += 1; ml += x
                if x != 255: break
        seqs.append((lit, off, ml + 4))
    return seqs

def replay(log, S):
    """compact table of S slots (slot = h % S, tag = h // S) + an 'evicted'
    bitmap: a get is exact unless its key was evicted earlier (then: fallback)"""
    slot_key = [-1]*S; evicted = set(); keys = set()
    for op, h in log:
        s = h % S
        if op == 'p':
            keys.add(h)
            if slot_key[s] not in (-1, h): evicted.add(slot_key[s])
            slot_key[s] = h
        else:
            if slot_key[s] != h and h in evicted: return False, len(keys)
    return True, len(keys)

def blocks(arr, E, nblk):
    raw = np.ascontiguousarray(arr).view(np.uint8)
    bs = (8192 // E) // 8 * 8 * E
    for k in range(nblk):
        blk = raw[k*bs:(k+1)*bs]
        yield o.bitshuffle(blk.view(np.dtype('V%d' % E)) if E not in (1,2,4,8) else blk.view({2:np.int16,4:np.float32}[E]), 0).view(np.uint8).tobytes()

if __name__ == "__main__":
  for name, arr, E in [('G1', o.gen_g1(1 << 20), 2), ('G2', o.gen_g2(1 << 19), 4),
                       ('E3', o.gen_g1(1 << 20).view(np.uint8)[: (1 << 21)//3*3], 3)]:
      res = {4096: 0, 2048: 0}; nk = []; nb = 24
      for b in blocks(arr, E, nb):
          log, seqs = lz4_log(b)
          ref = o.lz4_compress_block(np.frombuffer(b, np.uint8)).tobytes()
          assert seqs == oracle_seqs(ref), name  # the logged parse IS the oracle's
          for S in res:
              ok, k = replay(log, S)
              res[S] += ok
          nk.append(k)
      print(name, 'distinct keys per block %.0f' % np.mean(nk),
            'blocks exact without fallback: S=4096 %d/%d, S=2048 %d/%d' % (res[4096], nb, res[2048], nb))
