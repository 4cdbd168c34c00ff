// TEST INFRASTRUCTURE ONLY -- AddressSanitizer / UBSan driver for the CPU-side
// C and C++ of this repo (race detection / sanitizers on the host
// paths).  Built by tests/asan/Makefile with -fsanitize=address,undefined and
// run by tests/test_asan.py on the CPU:
//   * oracle/bshuf_oracle.c: framed compress / decompress and bitshuffle round
//     trips over many element sizes, block sizes (incl. the byU32 table),
//     partial blocks and raw tails -- every buffer malloc'ed to its exact size,
//     so any over-read or over-write is reported;
//   * bitshuffle_amd/csrc/lz4_scan.h (the decoder's scan state machine, the
//     same source the GPU's k_seq_scan runs), on exact-size payloads, valid and
//     corrupted, against the oracle's LZ4_decompress_safe restatement:
//     identical accept / reject decision, error position and decoded length.
// Exit status 0 = all checks passed and no sanitizer report.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../../bitshuffle_amd/csrc/lz4_scan.h"
#include "../../oracle/bshuf_oracle.h"

namespace {

uint64_t g_rng = 0x9E3779B97F4A7C15ull;
uint64_t rnd() {
    g_rng ^= g_rng << 13;
    g_rng ^= g_rng >> 7;
    g_rng ^= g_rng << 17;
    return g_rng;
}

int g_fail = 0;
#define CHECK(c, ...)                                   \
    do {                                                \
        if (!(c)) {                                     \
            fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
            fprintf(stderr, __VA_ARGS__);               \
            fprintf(stderr, "\n");                      \
            g_fail++;                                   \
        }                                               \
    } while (0)

// exact-size heap copy, so ASan sees every byte past the end
struct Buf {
    uint8_t* p = nullptr;
    size_t n = 0;
    explicit Buf(size_t k) : p((uint8_t*)malloc(k ? k : 1)), n(k) {}
    Buf(const uint8_t* src, size_t k) : Buf(k) {
        if (k) memcpy(p, src, k);
    }
    ~Buf() { free(p); }
    Buf(const Buf&) = delete;
    Buf& operator=(const Buf&) = delete;
};

void fill(uint8_t* p, size_t n, int kind) {
    int16_t* q = (int16_t*)p;
    switch (kind) {
        case 0:  // G1 int16 over the whole-int16 part
            orc_gen_g1_i16(q, n / 2, rnd() & 0xFFFF, 12345);
            for (size_t i = n & ~(size_t)1; i < n; i++) p[i] = (uint8_t)rnd();
            break;
        case 1:  // random bytes
            for (size_t i = 0; i < n; i++) p[i] = (uint8_t)rnd();
            break;
        case 2: {  // runs
            size_t i = 0;
            while (i < n) {
                const size_t len = 1 + rnd() % 40;
                const uint8_t v = (uint8_t)rnd();
                for (size_t j = 0; j < len && i < n; j++) p[i++] = v;
            }
            break;
        }
        default:  // slow walk
            for (size_t i = 0; i < n; i++) p[i] = (uint8_t)((i / 7) * 3 + (rnd() & 1));
    }
}

struct HostReader {
    const uint8_t* P;
    uint32_t operator()(int p) const { return P[p]; }
};
struct HostOut {
    std::vector<uint32_t>* pos;
    void put(int i, uint32_t v, int op) {
        if ((int)pos->size() <= i) pos->resize(i + 1);
        (*pos)[i] = v;
        (void)op;
    }
};

// scan (lz4_scan.h) vs the oracle decoder on an exact-size payload
void scan_vs_oracle(const uint8_t* comp, int clen, int cap) {
    Buf c(comp, (size_t)clen);
    Buf out((size_t)cap);
    const int want = orc_lz4_decompress_block(c.p, clen, out.p, cap);
    std::vector<uint32_t> pos;
    HostReader rd{c.p};
    HostOut o{&pos};
    int cnt = 0;
    const int got = bshuf::scan_block(rd, clen, cap, o, cnt);
    CHECK(got == want, "scan %d oracle %d (clen %d cap %d)", got, want, clen, cap);
}

void codec_case(size_t E, size_t n, size_t bs, int kind) {
    const size_t bytes = n * E;
    Buf in(bytes);
    fill(in.p, bytes, kind);
    // bitshuffle round trip
    {
        Buf sh(bytes), back(bytes);
        const int64_t a = orc_bitshuffle(in.p, sh.p, n, E, bs);
        const int64_t b = orc_bitunshuffle(sh.p, back.p, n, E, bs);
        CHECK(a == (int64_t)bytes && b == (int64_t)bytes, "bitshuffle %ld %ld", (long)a, (long)b);
        CHECK(!bytes || memcmp(in.p, back.p, bytes) == 0, "bitshuffle round trip E %zu n %zu", E, n);
    }
    const size_t bound = orc_compress_lz4_bound(n, E, bs);
    Buf comp(bound);
    const int64_t c = orc_compress_lz4(in.p, comp.p, n, E, bs);
    CHECK(c >= 0 && (size_t)c <= bound, "compress %ld bound %zu", (long)c, bound);
    if (c < 0) return;
    Buf exact(comp.p, (size_t)c);
    Buf dec(bytes);
    const int64_t d = orc_decompress_lz4(exact.p, dec.p, n, E, bs);
    CHECK(d == c, "decompress consumed %ld of %ld (E %zu n %zu bs %zu)", (long)d, (long)c, E, n, bs);
    CHECK(!bytes || memcmp(in.p, dec.p, bytes) == 0, "lz4 round trip E %zu n %zu bs %zu", E, n, bs);
    // every record: the scan state machine, valid and corrupted
    const size_t blk = bs ? bs : orc_default_block_size(E);
    size_t off = 0, left = n - n % 8;
    while (left > 0 && off + 4 <= (size_t)c) {
        const size_t m = left >= blk ? blk : (left / 8) * 8;
        const uint32_t clen = ((uint32_t)exact.p[off] << 24) | ((uint32_t)exact.p[off + 1] << 16) |
                              ((uint32_t)exact.p[off + 2] << 8) | exact.p[off + 3];
        const uint8_t* pay = exact.p + off + 4;
        scan_vs_oracle(pay, (int)clen, (int)(m * E));
        for (int t = 0; t < 6 && clen > 0; t++) {
            std::vector<uint8_t> bad(pay, pay + clen);
            const int flips = 1 + (int)(rnd() % 3);
            for (int f = 0; f < flips; f++) bad[rnd() % clen] ^= (uint8_t)(1 + rnd() % 255);
            int cl = (int)clen;
            // truncated (never to 0 bytes: the device's header check rejects an
            // empty record before any scan, lz4_decode.hip header_status)
            if (t == 5) cl = 1 + (int)(rnd() % clen);
            scan_vs_oracle(bad.data(), cl, (int)(m * E));
        }
        off += 4 + clen;
        left -= m;
    }
}

}  // namespace

int main() {
    const size_t Es[] = {1, 2, 3, 4, 5, 8, 12, 24};
    const size_t bss[] = {0, 8, 64, 680};
    int cases = 0;
    for (size_t E : Es)
        for (size_t bs : bss)
            for (int kind = 0; kind < 4; kind++) {
                const size_t n = 1 + rnd() % (24000 / E);
                codec_case(E, n, bs, kind);
                cases++;
            }
    // byU32 table path (bs * E >= 65547) and a few multi-block streams
    codec_case(8, 16400 * 2 + 13, 8200, 0);
    codec_case(4, 16400 * 3 + 5, 16400, 3);
    codec_case(2, 4096 * 5 + 7, 0, 0);
    codec_case(1, 0, 0, 0);
    cases += 4;
    printf("asan_driver: %d codec cases, %d failures\n", cases, g_fail);
    return g_fail ? 1 : 0;
}
