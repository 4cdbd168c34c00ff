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
 *   - a bounds-checked LZ4 block decoder restating LZ4_decompress_safe's fast
 *     and safe loops (lz4/lz4.c:2022-2445, 2451), so malformed input gets the
 *     reference's accept/reject decision, error value -(pos)-1 and output
 *     (pinned against the compiled reference in tests/test_oracle.py);
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
    int64_t err = 0;
    for (size_t k = 0; k < nfull + (last ? 1 : 0); k++) {
        const size_t m = k < nfull ? bs : last;
        size_t c = 0, p = 0;
        const int64_t r = fn(in, out, m, E, &c, &p);
        /* bshuf_blocked_wrap_fun (src/bitshuffle_core.c:1903-1917) keeps going
         * and returns the error of the last failing block */
        if (r < 0) {
            err = r;
            if (c == 0 && p == 0) return err; /* the chain cannot continue */
        } else {
            total += r;
        }
        in += c;
        out += p;
    }
    if (err < 0) return err;
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

/* LZ4_decompress_safe of LZ4 1.10.0 (lz4/lz4.c:2022-2445 instantiated at
 * 2451-2455: noDict, full block).  Its fast loop (2083-2209) and safe loop
 * (2215-2435) check different margins, so both are restated to reproduce the
 * same accept/reject decisions and error positions -(ip)-1.  Copies use byte
 * semantics, which equal LZ4's wildcopies for every accepted stream (bytes a
 * wildcopy writes past the sequence are rewritten before anything reads
 * them); offset 0, which no compressor emits but the decoder accepts, copies
 * zeros (the LZ4_write32(op, 0) seed of lz4.c:501 / 2407). */
static int read_len(const uint8_t* src, int* ip, int ilimit, int initial_check, size_t* out) {
    /* read_variable_length, lz4/lz4.c:1978-2014 */
    if (initial_check && *ip >= ilimit) return -1;
    unsigned s = src[(*ip)++];
    size_t len = s;
    if (*ip > ilimit) return -1;
    while (s == 255) {
        s = src[(*ip)++];
        len += s;
        if (*ip > ilimit) return -1;
    }
    *out = len;
    return 0;
}

static void copy_match(uint8_t* dst, int64_t op, size_t off, size_t ml) {
    if (off == 0) {
        memset(dst + op, 0, ml);
        return;
    }
    for (size_t i = 0; i < ml; i++) dst[op + (int64_t)i] = dst[op - (int64_t)off + (int64_t)i];
}

int orc_lz4_decompress_block(const uint8_t* src, int csize, uint8_t* dst, int cap) {
    enum { E_NONE, E_LIT, E_COPY_MATCH, E_MATCH };
    if (cap < 0) return -1;
    if (cap == 0) return (csize == 1 && src[0] == 0) ? 0 : -1;
    if (csize == 0) return -1;
    const int64_t clen = csize, n = cap;
    int ip = 0;
    int64_t op = 0;
    int fast = n >= 64; /* FASTLOOP_SAFE_DISTANCE */
    for (;;) {
        const unsigned tok = src[ip++];
        size_t len = tok >> 4, ml = 0, off = 0, add = 0;
        int entry = E_NONE;
        if (fast) {
            if (len == 15) {
                if (read_len(src, &ip, (int)(clen - 15), 1, &add)) goto err;
                len += add;
                if (op + (int64_t)len > n - 32 || ip + (int64_t)len > clen - 32) entry = E_LIT;
            } else if (ip > clen - 17) {
                entry = E_LIT;
            }
            if (entry == E_NONE) {
                memcpy(dst + op, src + ip, len);
                ip += (int)len;
                op += (int64_t)len;
                off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
                ip += 2;
                ml = tok & 15;
                if (ml == 15) {
                    if (read_len(src, &ip, (int)(clen - 4), 0, &add)) goto err;
                    ml += add + MINMATCH;
                    if (op + (int64_t)ml >= n - 64) entry = E_MATCH;
                } else {
                    ml += MINMATCH;
                    if (op + (int64_t)ml >= n - 64) {
                        entry = E_MATCH;
                    } else if (off >= 8 && (int64_t)off <= op) {
                        copy_match(dst, op, off, ml);
                        op += (int64_t)ml;
                        continue;
                    }
                }
                if (entry == E_NONE) {
                    if ((int64_t)off > op) goto err;
                    copy_match(dst, op, off, ml);
                    op += (int64_t)ml;
                    continue;
                }
            }
            fast = 0; /* the rest of the block runs in the safe loop */
        } else {
            if (len != 15 && ip < clen - 16 && op <= n - 32) {
                memcpy(dst + op, src + ip, len);
                ip += (int)len;
                op += (int64_t)len;
                ml = tok & 15;
                off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
                ip += 2;
                if (ml != 15 && off >= 8 && (int64_t)off <= op) {
                    copy_match(dst, op, off, ml + MINMATCH);
                    op += (int64_t)ml + MINMATCH;
                    continue;
                }
                entry = E_COPY_MATCH;
            } else {
                if (len == 15) {
                    if (read_len(src, &ip, (int)(clen - 15), 1, &add)) goto err;
                    len += add;
                }
                entry = E_LIT;
            }
        }
        if (entry == E_LIT) {
            const int64_t cpy = op + (int64_t)len;
            if (cpy > n - MFLIMIT || ip + (int64_t)len > clen - 8) {
                /* must be the last sequence: consume the input exactly */
                if (ip + (int64_t)len != clen || cpy > n) goto err;
                memcpy(dst + op, src + ip, len);
                op = cpy;
                break;
            }
            memcpy(dst + op, src + ip, len);
            ip += (int)len;
            op = cpy;
            off = (size_t)src[ip] | ((size_t)src[ip + 1] << 8);
            ip += 2;
            ml = tok & 15;
            entry = E_COPY_MATCH;
        }
        if (entry == E_COPY_MATCH) {
            if (ml == 15) {
                if (read_len(src, &ip, (int)(clen - 4), 0, &add)) goto err;
                ml += add;
            }
            ml += MINMATCH;
        }
        /* safe_match_copy */
        if ((int64_t)off > op) goto err;
        if (op + (int64_t)ml > n - LASTLITERALS) goto err;
        copy_match(dst, op, off, ml);
        op += (int64_t)ml;
    }
    return (int)op;
err:
    return -ip - 1;
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

/* bshuf_decompress_lz4_block (src/bitshuffle.c:83-119): the next record and
 * output block are set from the header BEFORE decoding (lines 93-99), so a
 * failing block does not stop the chain; its output is left untouched. */
static int64_t decomp_block(const uint8_t* in, uint8_t* out, size_t m, size_t E, size_t* c,
                            size_t* p) {
    const int32_t nb = (int32_t)get_be32(in);
    if (nb < 0) return -1 - 1000; /* a negative size walks backwards: not followed */
    *c = (size_t)nb + 4;
    *p = m * E;
    uint8_t* tmp = (uint8_t*)malloc((m * E) != 0 ? (size_t)(m * E) : 1);
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
