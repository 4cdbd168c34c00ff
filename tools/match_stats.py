"""Match statistics of a bshuf LZ4 stream and the decoder's match batching.

Reads a raw bshuf_compress_lz4 stream (records [BE32 c][c bytes], no HDF5
header) from a file and prints, per block: the match classes the decoder's
phase 2 treats differently (self-overlapping or not, length <= 16 / <= 64 /
longer, offsets), and the number of match batches under three rules:
  current  -- lz4_decode.hip's stop rule: a later match joins the batch when
              the bytes it reads lie before the batch's first match output;
  literal  -- the same, or its source lies inside its own literal run;
  precise  -- its source overlaps no earlier batch member's match output.
The precise rule is the floor for any batch-at-a-time executor.

usage: python tools/match_stats.py STREAM_FILE
"""
import collections
import sys


def parse(c):
    p, n, blocks = 0, len(c), []
    while p + 4 <= n:
        L = int.from_bytes(c[p:p + 4], "big")
        p += 4
        end, q, seqs, op = p + L, p, [], 0
        if end > n:
            break
        while q < end:
            t = c[q]
            q += 1
            lit = t >> 4
            if lit == 15:
                while True:
                    b = c[q]
                    q += 1
                    lit += b
                    if b != 255:
                        break
            q += lit
            if q >= end:
                seqs.append((op, lit, 0, 0))
                break
            off = c[q] | (c[q + 1] << 8)
            q += 2
            ml = t & 15
            if ml == 15:
                while True:
                    b = c[q]
                    q += 1
                    ml += b
                    if b != 255:
                        break
            ml += 4
            seqs.append((op, lit, off, ml))
            op += lit + ml
        blocks.append(seqs)
        p = end
    return blocks


def batches(blocks, rule):
    nb = 0
    for seqs in blocks:
        for c0 in range(0, len(seqs), 64):
            ch = seqs[c0:c0 + 64]
            todo = [i for i, s in enumerate(ch) if s[3] > 0]
            while todo:
                f = todo[0]
                opf = ch[f][0] + ch[f][1]
                outs, g = [], len(ch)
                for l in todo:
                    op, lit, off, ml = ch[l]
                    mop = op + lit
                    ss, se = mop - off, mop - off + min(ml, off)
                    if rule == "precise":
                        ok = not any(ss < b and a < se for a, b in outs)
                    else:
                        ok = l == f or se <= opf or (rule == "literal" and off <= lit)
                    if not ok:
                        g = l
                        break
                    outs.append((mop, mop + ml))
                nb += 1
                todo = [l for l in todo if l >= g]
    return nb / max(len(blocks), 1)


def main(path):
    blocks = parse(open(path, "rb").read())
    cnt, tot = collections.Counter(), 0
    for seqs in blocks:
        for op, lit, off, ml in seqs:
            if ml == 0:
                continue
            tot += 1
            ov = "overlap" if off < ml else "plain"
            cnt[(ov, "<=16" if ml <= 16 else "<=64" if ml <= 64 else ">64")] += 1
            if off < ml:
                cnt[("overlap", "off=%s" % (off if off <= 4 else "5-8" if off <= 8 else "9+"))] += 1
    print("blocks %d, matches per block %.1f" % (len(blocks), tot / max(len(blocks), 1)))
    for k, v in sorted(cnt.items()):
        print("  %-8s %-6s %5.1f %%" % (k[0], k[1], 100.0 * v / max(tot, 1)))
    for rule in ("current", "literal", "precise"):
        print("batches per block, %-8s rule: %.1f" % (rule, batches(blocks, rule)))


if __name__ == "__main__":
    main(sys.argv[1])
