/*
 * bshuf_oracle.c -- TEST INFRASTRUCTURE ONLY (see bshuf_oracle.h).
 *
 * A plain, single-threaded restatement of the reference's hot path:
 *   - the blocked bit transpose, stated in closed form
 *       out[r*(m/8) + i/8] bit (i%8) = bit (r%8) of byte (r/8) of element i
 *     (equivalent to bshuf_trans_bit_elem_scal, src/bitshuffle_core.c:276-296,
 *      and its inverse bshuf_untrans_bit_elem_scal, :369-387);
 *   - the greedy LZ4 v1.10.0 block parse exactly as LZ4_compress_default runs
 *     it for a fresh, zeroed state (lz4/lz4.c:930-1338, 1382-1403, 1472);
 *   - a bounds-checked LZ4 block decoder (semantics of LZ4_decompress_safe,
 *     lz4/lz4.c:2451; error *values* on malformed input are not reproduced,
 *     only their sign);
 *   - bitshuffle's framing: per block u32 big-endian length + LZ4 payload,
 *     partial last block, n%8 raw tail (src/bitshuffle.c:36-119,
 *     src/bitshuffle_core.c:1877-1931).
 * Nothing here is shipped: the product path is bitshuffle_amd/ (HIP).
 */
#include "bshuf_oracle.h"

#include <stdlib.h>
#include <string.h>

#define BLOCKED_MULT 8          /* src/bitshuffle_internals.h:34 */
#define TARGET_BLOCK_BYTES 8192 /* src/bitshuffle_internals.h:35 */
#define MIN_RECOMMEND_BLOCK 128 /* src/bitshuffle_internals.h:33 */

/* ------------------------------------------------------------------ */
/* Block sizing                                                        */
/* ------------------------------------------------------------------ */

size_t orc_default_block_size(size_t elem_size) {
    size_t bs = TARGET_BLOCK_BYTES / elem_size;
    bs -= bs % BLOCKED_MULT;
    return bs > MIN_RECOMMEND_BLOCK ? bs : MIN_RECOMMEND_BLOCK;
}

/* ------------------------------------------------------------------ */
/* Bit transpose, closed form                                          */
/* ------------------------------------------------------------------ */

void orc_trans_bit_elem(const uint8_t* in, uint8_t* out, size_t m, size_t E) {
    const size_t plane = m / 8;
    for (size_t r = 0; r < 8 * E; r++) {
        const size_t byte = r / 8;
        const unsigned bit = (unsigned)(r % 8);
        uint8_t* dst = out + r * plane;
        for (size_t g = 0; g < plane; g++) {
            unsigned v = 0;
            for (unsigned k = 0; k < 8; k++)
                v |= ((unsigned)(in[(8 * g + k) * E + byte] >> bit) & 1u) << k;
            dst[g] = (uint8_t)v;
        }
    }
}

void orc_untrans_bit_elem(const uint8_t* in, uint8_t* out, size_t m, size_t E) {
    const size_t plane = m / 8;
    memset(out, 0, m * E);
    for (size_t r = 0; r < 8 * E; r++) {
        const size_t byte = r / 8;
        const unsigned bit = (unsigned)(r % 8);
        const uint8_t* src = in + r * plane;
        for (size_t g = 0; g < plane; g++) {
            const unsigned v = src[g];
            for (unsigned k = 0; k < 8; k++)
                out[(8 * g + k) * E + byte] |= (uint8_t)(((v >> k) & 1u) << bit);
        }
    }
}

/* ------------------------------------------------------------------ */
/* Blocked wrapper semantics                                           */
/* ------------------------------------------------------------------ */

typedef int64_t (*orc_block_fn)(const uint8_t* in, uint8_t* out, size_t m, size_t E,
                                size_t* consumed, size_t* produced);

static int64_t blocked(orc_block_fn fn, const void* vin, void* vout, size_t n, size_t E,
                       size_t bs) {
    const uint8_t* in = (const uint8_t*)vin;
    uint8_t* out = (uint8_t*)vout;
    if (bs == 0) bs = orc_default_block_size(E);
    if (bs % BLOCKED_MULT) return -81;
    int64_t total = 0;
    const size_t nfull = n / bs;
    size_t last = n % bs;
    last -= last % BLOCKED_MULT;
    for (size_t k = 0; k < nfull + (last ? 1 : 0); k++) {
        const size_t m = k < nfull ? bs : last;
        size_t c = 0, p = 0;
        const int64_t r = fn(in, out, m, E, &c, &p);
        if (r < 0) return r;
        total += r;
        in += c;
        out += p;
    }
    const size_t tail = (n % BLOCKED_MULT) * E;
    memcpy(out, in, tail);
    return total + (int64_t)tail;
}

static int64_t shuf_block(const uint8_t* in, uint8_t* out, size_t m, size_t E, size_t* c,
                          size_t* p) {
    orc_trans_bit_elem(in, out, m, E);
    *c = *p = m * E;
    return (int64_t)(m * E);
}

static int64_t unshuf_block(const uint8_t* in, uint8_t* out, size_t m, size_t E, size_t* c,
                            size_t* p) {
    orc_untrans_bit_elem(in, out, m, E);
    *c = *p = m * E;
    return (int64_t)(m * E);
}

int64_t orc_bitshuffle(const void* in, void* out, size_t n, size_t E, size_t bs) {
    return blocked(shuf_block, in, out, n, E, bs);
}

int64_t orc_bitunshuffle(const void* in, void* out, size_t n, size_t E, size_t bs) {
    return blocked(unshuf_block, in, out, n, E, bs);
}

/* ------------------------------------------------------------------ */
/* LZ4 block compressor, greedy parse of LZ4 v1.10.0                   */
/* ------------------------------------------------------------------ */

enum {
    MINMATCH = 4,
    MFLIMIT = 12,
    LASTLITERALS = 5,
    SMALL_INPUT = MFLIMIT + 1,          /* LZ4_minLength, lz4/lz4.c:249 */
    U16_TABLE_LIMIT = 65536 + MFLIMIT - 1, /* LZ4_64Klimit, lz4/lz4.c:710 */
    MAX_DISTANCE = 65535
};

static inline uint32_t ld32(const uint8_t* p) {
    return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
           ((uint32_t)p[3] << 24);
}

static inline uint64_t ld64(const uint8_t* p) {
    return (uint64_t)ld32(p) | ((uint64_t)ld32(p + 4) << 32);
}

/* byU16 table: 2^13 entries, hash of 4 bytes (lz4/lz4.c:777-783).
 * byU32 table: 2^12 entries, hash of 5 bytes (lz4/lz4.c:785-795). */
static inline uint32_t hpos(const uint8_t* p, int wide) {
    if (!wide) return (ld32(p) * 2654435761u) >> 19;
    return (uint32_t)(((ld64(p) << 24) * 889523592379ull) >> 52);
}

int orc_lz4_compress_bound(int n) { return n + n / 255 + 16; }

static uint8_t* put_len(uint8_t* op, size_t len) {
    /* the 255-run continuation used for literal and match lengths >= 15 */
    for (; len >= 255; len -= 255) *op++ = 255;
    *op++ = (uint8_t)len;
    return op;
}

int orc_lz4_compress_block(const uint8_t* src, int n, uint8_t* dst) {
    if (n == 0) {
        dst[0] = 0;
        return 1;
    }
    const int wide = n >= U16_TABLE_LIMIT;
    uint32_t* tab = (uint32_t*)calloc(8192, sizeof(uint32_t));
    uint8_t* op = dst;
    int anchor = 0;
    if (n >= SMALL_INPUT) {
        const int limit = n - MFLIMIT + 1;      /* mflimitPlusOne */
        const int matchlimit = n - LASTLITERALS;
        tab[hpos(src, wide)] = 0;
        int ip = 1;
        for (;;) {
            int match;
            /* Search with skip acceleration (lz4/lz4.c:1042-1101). */
            {
                int fwd = ip, step = 1, nb = 64;
                for (;;) {
                    const int cur = fwd;
                    const uint32_t h = hpos(src + cur, wide);
                    const uint32_t cand = tab[h];
                    ip = fwd;
                    fwd += step;
                    step = nb++ >> 6;
                    if (fwd > limit) goto last_literals;
                    tab[h] = (uint32_t)cur;
                    if (wide && cand + MAX_DISTANCE < (uint32_t)cur) continue;
                    if (ld32(src + cand) == ld32(src + ip)) {
                        match = (int)cand;
                        break;
                    }
                }
            }
            /* Catch up backwards (lz4/lz4.c:1105-1109). */
            while (ip > anchor && match > 0 && src[ip - 1] == src[match - 1]) {
                ip--;
                match--;
            }
            uint8_t* token = op++;
            {
                const int lit = ip - anchor;
                if (lit >= 15) {
                    *token = 15 << 4;
                    op = put_len(op, (size_t)(lit - 15));
                } else {
                    *token = (uint8_t)(lit << 4);
                }
                memcpy(op, src + anchor, (size_t)lit);
                op += lit;
            }
            for (;;) {
                /* offset + match length (lz4/lz4.c:1133-1226) */
                const int off = ip - match;
                *op++ = (uint8_t)off;
                *op++ = (uint8_t)(off >> 8);
                int mc = 0;
                {
                    int a = ip + MINMATCH, b = match + MINMATCH;
                    while (a < matchlimit && src[a] == src[b]) a++, b++;
                    mc = a - (ip + MINMATCH);
                }
                ip += mc + MINMATCH;
                if (mc >= 15) {
                    *token += 15;
                    op = put_len(op, (size_t)(mc - 15));
                } else {
                    *token += (uint8_t)mc;
                }
                anchor = ip;
                if (ip >= limit) goto last_literals;
                tab[hpos(src + ip - 2, wide)] = (uint32_t)(ip - 2);
                /* immediate re-test at ip, no catch-up (lz4/lz4.c:1255-1293) */
                const uint32_t h = hpos(src + ip, wide);
                const uint32_t cand = tab[h];
                tab[h] = (uint32_t)ip;
                if ((!wide || cand + MAX_DISTANCE >= (uint32_t)ip) &&
                    ld32(src + cand) == ld32(src + ip)) {
                    token = op++;
                    *token = 0;
                    match = (int)cand;
                    continue;
                }
                break;
            }
            ip++;
        }
    }
last_literals: {
    const size_t run = (size_t)(n - anchor);
    if (run >= 15) {
        *op++ = 15 << 4;
        op = put_len(op, run - 15);
    } else {
        *op++ = (uint8_t)(run << 4);
    }
    memcpy(op, src + anchor, run);
    op += run;
}
    free(tab);
    return (int)(op - dst);
}

/* ------------------------------------------------------------------ */
/* LZ4 block decoder                                                   */
/* ------------------------------------------------------------------ */

int orc_lz4_decompress_block(const uint8_t* src, int csize, uint8_t* dst, int cap) {
    const uint8_t* ip = src;
    const uint8_t* const iend = src + csize;
    uint8_t* op = dst;
    uint8_t* const oend = dst + cap;
    if (csize <= 0) return -1;
    for (;;) {
        if (ip >= iend) return -(int)(ip - src) - 1;
        const unsigned tok = *ip++;
        size_t lit = tok >> 4;
        if (lit == 15) {
            unsigned s;
            do {
                if (ip >= iend) return -(int)(ip - src) - 1;
                s = *ip++;
                lit += s;
            } while (s == 255);
        }
        if ((size_t)(iend - ip) < lit || (size_t)(oend - op) < lit)
            return -(int)(ip - src) - 1;
        memcpy(op, ip, lit);
        op += lit;
        ip += lit;
        if (ip == iend) break; /* last sequence: literals only */
        if (iend - ip < 2) return -(int)(ip - src) - 1;
        const size_t off = (size_t)ip[0] | ((size_t)ip[1] << 8);
        ip += 2;
        if (off == 0 || off > (size_t)(op - dst)) return -(int)(ip - src) - 1;
        size_t ml = tok & 15;
        if (ml == 15) {
            unsigned s;
            do {
                if (ip >= iend) return -(int)(ip - src) - 1;
                s = *ip++;
                ml += s;
            } while (s == 255);
        }
        ml += MINMATCH;
        if ((size_t)(oend - op) < ml) return -(int)(ip - src) - 1;
        const uint8_t* m = op - off;
        for (size_t i = 0; i < ml; i++) op[i] = m[i]; /* overlap-safe, byte order */
        op += ml;
    }
    return (int)(op - dst);
}

/* ------------------------------------------------------------------ */
/* Framing                                                             */
/* ------------------------------------------------------------------ */

static void put_be32(uint8_t* p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

static uint32_t get_be32(const uint8_t* p) {
    return ((uint32_t)p[0] << 24) | ((uint32_t)p[1] << 16) | ((uint32_t)p[2] << 8) | p[3];
}

size_t orc_compress_lz4_bound(size_t n, size_t E, size_t bs) {
    if (bs == 0) bs = orc_default_block_size(E);
    if (bs % BLOCKED_MULT) return (size_t)-81;
    size_t bound = (size_t)(orc_lz4_compress_bound((int)(bs * E)) + 4) * (n / bs);
    size_t last = n % bs;
    last -= last % BLOCKED_MULT;
    if (last) bound += (size_t)orc_lz4_compress_bound((int)(last * E)) + 4;
    return bound + (n % BLOCKED_MULT) * E;
}

static int64_t comp_block(const uint8_t* in, uint8_t* out, size_t m, size_t E, size_t* c,
                          size_t* p) {
    uint8_t* tmp = (uint8_t*)malloc(m * E);
    if (!tmp) return -1;
    orc_trans_bit_elem(in, tmp, m, E);
    const int nb = orc_lz4_compress_block(tmp, (int)(m * E), out + 4);
    free(tmp);
    if (nb < 0) return nb - 1000;
    put_be32(out, (uint32_t)nb);
    *c = m * E;
    *p = (size_t)nb + 4;
    return nb + 4;
}

static int64_t decomp_block(const uint8_t* in, uint8_t* out, size_t m, size_t E, size_t* c,
                            size_t* p) {
    const int32_t nb = (int32_t)get_be32(in);
    uint8_t* tmp = (uint8_t*)malloc(m * E);
    if (!tmp) return -1;
    const int r = orc_lz4_decompress_block(in + 4, nb, tmp, (int)(m * E));
    if (r < 0) {
        free(tmp);
        return (int64_t)r - 1000;
    }
    if ((size_t)r != m * E) {
        free(tmp);
        return -91;
    }
    orc_untrans_bit_elem(tmp, out, m, E);
    free(tmp);
    *c = (size_t)nb + 4;
    *p = m * E;
    return nb + 4;
}

int64_t orc_compress_lz4(const void* in, void* out, size_t n, size_t E, size_t bs) {
    return blocked(comp_block, in, out, n, E, bs);
}

int64_t orc_decompress_lz4(const void* in, void* out, size_t n, size_t E, size_t bs) {
    return blocked(decomp_block, in, out, n, E, bs);
}

/* ------------------------------------------------------------------ */
/* Synthetic generators                               */
/* ------------------------------------------------------------------ */

static inline uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static inline uint64_t ctr_hash(uint64_t seed, uint64_t i) {
    return mix64(seed + (i + 1) * 0x9E3779B97F4A7C15ull);
}

static inline uint32_t tri(uint64_t i) {
    const uint32_t p = (uint32_t)(i & 65535u);
    return p < 32768u ? p : 65536u - p;
}

void orc_gen_g0_ramp_i32(int32_t* out, size_t n, size_t first) {
    for (size_t k = 0; k < n; k++) out[k] = (int32_t)(first + k);
}

void orc_gen_g1_i16(int16_t* out, size_t n, size_t first, uint64_t seed) {
    for (size_t k = 0; k < n; k++) {
        const uint64_t i = first + k;
        const int v = (int)(tri(i) >> 3) - 2048 + (int)(ctr_hash(seed, i) & 31u) - 16;
        out[k] = (int16_t)v;
    }
}

void orc_gen_g2_f32(float* out, size_t n, size_t first, uint64_t seed) {
    for (size_t k = 0; k < n; k++) {
        const uint64_t i = first + k;
        out[k] = (float)(tri(i) * 64u + (uint32_t)(ctr_hash(seed, i) & 255u)) / 1024.0f;
    }
}
