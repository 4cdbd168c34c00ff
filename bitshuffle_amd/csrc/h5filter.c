/*
 * h5filter.c -- HDF5 filter 32008 over the MI355X codec (libbitshuffle_mi355x).
 *
 * Same protocol as the reference (src/bshuf_h5filter.c:29-260,
 * src/bshuf_h5plugin.c:17-18): set_local prepends {major, minor, elem_size}
 * to the user's cd_values; the filter callback frees HDF5's *buf and hands
 * back a malloc'ed result, returning 0 (after pushing an HDF5 error) on any
 * failure.  The chunk buffer lives in host memory: the codec stages it
 * through the GPU inside bshuf_compress_lz4 / bshuf_decompress_lz4.
 *
 * Built with -Wl,-z,nodelete so HDF5's dlclose() at H5close cannot unmap
 * code that HIP runtime threads may still reference (hazard 5).
 */
#define _GNU_SOURCE
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <sys/mman.h>
#include <time.h>

#include "bitshuffle.h"
#include "bshuf_h5filter.h"

#define H5ERR(fn, minor, msg) H5Epush1(__FILE__, fn, __LINE__, H5E_PLINE, minor, msg)

static void put_u64be(unsigned char* p, uint64_t v) {
    for (int i = 7; i >= 0; i--, v >>= 8) p[i] = (unsigned char)(v & 0xFF);
}

static void put_u32be(unsigned char* p, uint32_t v) {
    for (int i = 3; i >= 0; i--, v >>= 8) p[i] = (unsigned char)(v & 0xFF);
}

static uint64_t get_u64be(const unsigned char* p) {
    uint64_t v = 0;
    for (int i = 0; i < 8; i++) v = (v << 8) | p[i];
    return v;
}

static uint32_t get_u32be(const unsigned char* p) {
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) v = (v << 8) | p[i];
    return v;
}

/* Dataset creation: record version and element size in front of the user's
 * options (reference src/bshuf_h5filter.c:29-95). */
static herr_t bshuf_h5_set_local(hid_t dcpl, hid_t type, hid_t space) {
    (void)space;
    unsigned flags = 0, user[8] = {0}, cd[11] = {0};
    size_t nuser = 8;
    if (H5Pget_filter_by_id2(dcpl, BSHUF_H5FILTER, &flags, &nuser, user, 0, NULL, NULL) < 0)
        return -1;
    size_t n = 0;
    for (; n < nuser && n + 3 < 11; n++) cd[n + 3] = user[n];
    const size_t esz = H5Tget_size(type);
    if (esz == 0) {
        H5ERR("bshuf_h5_set_local", H5E_CALLBACK, "Invalid element size.");
        return -1;
    }
    cd[0] = BSHUF_VERSION_MAJOR;
    cd[1] = BSHUF_VERSION_MINOR;
    cd[2] = (unsigned)esz;
    n += 3;
    if (n > 3 && cd[3] % 8) {
        char msg[80];
        snprintf(msg, sizeof msg, "Error in bitshuffle. Invalid block size: %u.", cd[3]);
        H5ERR("bshuf_h5_set_local", H5E_CALLBACK, msg);
        return -1;
    }
    if (n > 4 && cd[4] != 0 && cd[4] != BSHUF_H5_COMPRESS_LZ4)
        /* the reference logs and carries on (src/bshuf_h5filter.c:85-88) */
        H5ERR("bshuf_h5_set_local", H5E_CALLBACK, "Invalid bitshuffle compression.");
    return H5Pmodify_filter(dcpl, BSHUF_H5FILTER, flags, n, cd) < 0 ? -1 : 1;
}

/* The result buffer HDF5 takes over (it frees it with free()).  Chunk buffers
 * are tens of MiB, so malloc hands out fresh mmap'ed pages every call and the
 * GPU -> host copy into them pays one page fault per 4 KiB; 2 MiB-aligned
 * memory advised for transparent huge pages faults once per 2 MiB instead.
 * BSHUF_H5_NO_HUGEPAGE=1 falls back to plain malloc. */
static void* out_alloc(size_t n) {
    static int plain = -1;
    if (plain < 0) plain = getenv("BSHUF_H5_NO_HUGEPAGE") != NULL;
    const size_t huge = (size_t)2 << 20;
    if (plain || n < huge) return malloc(n ? n : 1);
    const size_t rounded = (n + huge - 1) & ~(huge - 1);
    void* p = NULL;
    if (posix_memalign(&p, huge, rounded) != 0) return malloc(n);
    (void)madvise(p, rounded, MADV_HUGEPAGE);
    return p;
}

/* BSHUF_H5_TIMING=1: time spent inside the filter callback (per direction),
 * printed to stderr at process exit -- separates the codec's share of an
 * HDF5 read/write from HDF5's own chunk I/O. */
static double g_t[2];
static long g_n[2];
static int g_timing = -1;

static double wall(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static void timing_report(void) {
    fprintf(stderr, "bshuf_h5_filter: write %ld calls %.3f s, read %ld calls %.3f s\n", g_n[0], g_t[0],
            g_n[1], g_t[1]);
}

static size_t filter_impl(unsigned flags, size_t cd_nelmts, const unsigned cd_values[],
                          size_t nbytes, size_t* buf_size, void** buf);

static size_t bshuf_h5_filter(unsigned flags, size_t cd_nelmts, const unsigned cd_values[],
                              size_t nbytes, size_t* buf_size, void** buf) {
    if (g_timing < 0) {
        g_timing = getenv("BSHUF_H5_TIMING") != NULL;
        if (g_timing) atexit(timing_report);
    }
    if (!g_timing) return filter_impl(flags, cd_nelmts, cd_values, nbytes, buf_size, buf);
    const double t0 = wall();
    const size_t r = filter_impl(flags, cd_nelmts, cd_values, nbytes, buf_size, buf);
    const int dir = (flags & H5Z_FLAG_REVERSE) != 0;
    g_t[dir] += wall() - t0;
    g_n[dir]++;
    return r;
}

static size_t filter_impl(unsigned flags, size_t cd_nelmts, const unsigned cd_values[],
                              size_t nbytes, size_t* buf_size, void** buf) {
    if (cd_nelmts < 3) {
        H5ERR("bshuf_h5_filter", H5E_CALLBACK, "Not enough parameters.");
        return 0;
    }
    const size_t esz = cd_values[2];
    size_t block = cd_nelmts > 3 ? cd_values[3] : 0;
    if (block == 0) block = bshuf_default_block_size(esz);
    const int mode = cd_nelmts > 4 ? (int)cd_values[4] : 0;
    if (mode == BSHUF_H5_COMPRESS_ZSTD) {
        H5ERR("bshuf_h5_filter", H5E_CALLBACK,
              "ZSTD compression filter chosen but ZSTD support not installed.");
        return 0;
    }
    const int lz4 = mode == BSHUF_H5_COMPRESS_LZ4;
    const int reverse = (flags & H5Z_FLAG_REVERSE) != 0;
    const unsigned char* in = (const unsigned char*)*buf;
    size_t raw_bytes, out_cap;
    if (lz4 && reverse) {
        raw_bytes = (size_t)get_u64be(in);
        block = get_u32be(in + 8) / esz;  /* the chunk header wins over cd_values */
        in += 12;
        out_cap = raw_bytes;
    } else if (lz4) {
        raw_bytes = nbytes;
        out_cap = bshuf_compress_lz4_bound(raw_bytes / esz, esz, block) + 12;
    } else {
        raw_bytes = nbytes;
        out_cap = nbytes;
    }
    if (raw_bytes % esz) {
        H5ERR("bshuf_h5_filter", H5E_CALLBACK, "Non integer number of elements.");
        return 0;
    }
    const size_t nelem = raw_bytes / esz;
    unsigned char* out = (unsigned char*)out_alloc(out_cap);
    if (!out) {
        H5ERR("bshuf_h5_filter", H5E_CALLBACK, "Could not allocate output buffer.");
        return 0;
    }
    int64_t r;
    size_t produced;
    if (lz4 && reverse) {
        r = bshuf_decompress_lz4(in, out, nelem, esz, block);
        produced = raw_bytes;
    } else if (lz4) {
        put_u64be(out, (uint64_t)raw_bytes);
        put_u32be(out + 8, (uint32_t)(block * esz));
        r = bshuf_compress_lz4(in, out + 12, nelem, esz, block);
        produced = (size_t)r + 12;
    } else {
        r = reverse ? bshuf_bitunshuffle(in, out, nelem, esz, block)
                    : bshuf_bitshuffle(in, out, nelem, esz, block);
        produced = nbytes;
    }
    if (r < 0) {
        char msg[80];
        snprintf(msg, sizeof msg, "Error in bitshuffle with error code %lld.", (long long)r);
        H5ERR("bshuf_h5_filter", H5E_CALLBACK, msg);
        free(out);
        return 0;
    }
    free(*buf);
    *buf = out;
    *buf_size = out_cap;
    return produced;
}

H5Z_class_t bshuf_H5Filter[1] = {{
    H5Z_CLASS_T_VERS,
    (H5Z_filter_t)(BSHUF_H5FILTER),
    1,
    1,
    "bitshuffle; see https://github.com/kiyo-masui/bitshuffle",
    NULL,
    (H5Z_set_local_func_t)(bshuf_h5_set_local),
    (H5Z_func_t)(bshuf_h5_filter),
}};

int bshuf_register_h5filter(void) {
    const int r = H5Zregister(bshuf_H5Filter);
    if (r < 0) H5ERR("bshuf_register_h5filter", H5E_CANTREGISTER, "Can't register bitshuffle filter");
    return r;
}

H5PL_type_t H5PLget_plugin_type(void) { return H5PL_TYPE_FILTER; }
const void* H5PLget_plugin_info(void) { return bshuf_H5Filter; }
