/*
 * h5_harness.c -- drives the filter-32008 plugin through the real HDF5 C
 * library, loaded dynamically via HDF5_PLUGIN_PATH (as h5py / h5dump would).
 *
 *   h5_harness regress <fixture_dir> <scratch.h5>
 *     For each of the 42 LZ4 datasets of the reference's regression files
 *     (extracted to tests/golden/regression by extract_regression.c):
 *       encode: H5Dwrite(original) through the filter, then H5Dread_chunk of
 *               the stored chunk must equal the reference's stored chunk;
 *       decode: H5Dwrite_chunk(the reference's chunk) raw, then H5Dread
 *               through the filter must equal `original`.
 *   h5_harness roundtrip <scratch.h5> <n_elem> <chunk_elem>
 *     BASELINE config 5: uint16 (G1 + 32768) dataset written and read back
 *     through the filter (block 0, LZ4), verified, host-memory end to end;
 *     prints one JSON line with write/read GB/s.
 *   h5_harness chunks <file.h5> <dataset>
 *     Writes every stored (filtered) chunk of a 1-D dataset to stdout, raw, in
 *     chunk order (H5Dread_chunk), for byte-for-byte / digest comparison with
 *     the reference's u64BE || u32BE || bshuf_compress_lz4 chunk format.
 */
#include <hdf5.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#define FILTER 32008

static unsigned char* slurp(const char* path, size_t* n) {
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    *n = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* b = malloc(*n + 1);
    if (fread(b, 1, *n, f) != *n) {
        fclose(f);
        free(b);
        return NULL;
    }
    fclose(f);
    return b;
}

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

static hid_t make_dset_f(hid_t file, const char* name, hid_t type, hsize_t n, hsize_t chunk,
                         unsigned block, int filtered) {
    hid_t space = H5Screate_simple(1, &n, NULL);
    hid_t dcpl = H5Pcreate(H5P_DATASET_CREATE);
    H5Pset_chunk(dcpl, 1, &chunk);
    const unsigned opts[2] = {block, 2 /* LZ4 */};
    if (filtered && H5Pset_filter(dcpl, FILTER, H5Z_FLAG_MANDATORY, 2, opts) < 0) return -1;
    hid_t d = H5Dcreate2(file, name, type, space, H5P_DEFAULT, dcpl, H5P_DEFAULT);
    H5Pclose(dcpl);
    H5Sclose(space);
    return d;
}

static hid_t make_dset(hid_t file, const char* name, hid_t type, hsize_t n, hsize_t chunk,
                       unsigned block) {
    return make_dset_f(file, name, type, n, chunk, block, 1);
}

/* The same chunked write + read with NO filter: HDF5's own I/O floor on this
 * machine (chunk copies, file writes/reads), for reading the filtered rates. */
static void io_floor(const char* out, const uint16_t* a, uint16_t* b, long long n, long long chunk,
                     double* w, double* r) {
    char path[1100];
    snprintf(path, sizeof path, "%s.raw", out);
    hid_t file = H5Fcreate(path, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    hid_t d = make_dset_f(file, "data", H5T_NATIVE_UINT16, (hsize_t)n, (hsize_t)chunk, 0, 0);
    double t0 = now();
    H5Dwrite(d, H5T_NATIVE_UINT16, H5S_ALL, H5S_ALL, H5P_DEFAULT, a);
    H5Dclose(d);
    H5Fclose(file);
    double t1 = now();
    file = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
    d = H5Dopen2(file, "data", H5P_DEFAULT);
    double t2 = now();
    H5Dread(d, H5T_NATIVE_UINT16, H5S_ALL, H5S_ALL, H5P_DEFAULT, b);
    double t3 = now();
    H5Dclose(d);
    H5Fclose(file);
    remove(path);
    *w = n * 2 / (t1 - t0) / 1e9;
    *r = n * 2 / (t3 - t2) / 1e9;
}

static int regress(const char* dir, const char* out) {
    char path[1024], line[512];
    snprintf(path, sizeof path, "%s/MANIFEST", dir);
    FILE* m = fopen(path, "r");
    if (!m) return 2;
    hid_t file = H5Fcreate(out, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    int ok = 0, total = 0;
    /* H5H_PASSES=k: run the whole list k times in this process (pass p's
     * failures are reported with its number) */
    const int passes = getenv("H5H_PASSES") ? atoi(getenv("H5H_PASSES")) : 1;
    for (int pass = 0; pass < passes; pass++) {
    rewind(m);
    if (pass) fprintf(stderr, "pass %d\n", pass);
    while (fgets(line, sizeof line, m)) {
        char ver[32], name[128];
        size_t esz;
        long long n, csz;
        if (sscanf(line, "%31s %127s %zu %lld %lld", ver, name, &esz, &n, &csz) != 5) continue;
        total++;
        size_t no, nc;
        snprintf(path, sizeof path, "%s/%s__%s.orig", dir, ver, name);
        unsigned char* orig = slurp(path, &no);
        snprintf(path, sizeof path, "%s/%s__%s.chunk", dir, ver, name);
        unsigned char* chunk = slurp(path, &nc);
        if (!orig || !chunk || no != (size_t)n * esz || nc != (size_t)csz) {
            fprintf(stderr, "fixture %s/%s unreadable\n", ver, name);
            continue;
        }
        const unsigned block = (unsigned)((chunk[8] << 24 | chunk[9] << 16 | chunk[10] << 8 |
                                           chunk[11]) / esz);
        hid_t type = H5Tcreate(H5T_OPAQUE, esz);
        H5Tset_tag(type, "raw");
        char dname[300];
        /* encode through the plugin */
        snprintf(dname, sizeof dname, "enc%d_%s_%s", pass, ver, name);
        hid_t d = make_dset(file, dname, type, (hsize_t)n, (hsize_t)n, block);
        int good = d >= 0 && H5Dwrite(d, type, H5S_ALL, H5S_ALL, H5P_DEFAULT, orig) >= 0;
        H5Dflush(d);
        hsize_t off[1] = {0}, sz = 0;
        uint32_t fm = 0;
        good = good && H5Dget_chunk_storage_size(d, off, &sz) >= 0 && sz == (hsize_t)nc;
        unsigned char* got = malloc(nc + 16);
        good = good && H5Dread_chunk(d, H5P_DEFAULT, off, &fm, got) >= 0 &&
               memcmp(got, chunk, nc) == 0;
        if (!good) fprintf(stderr, "ENCODE mismatch %s/%s (%llu vs %zu bytes)\n", ver, name,
                           (unsigned long long)sz, nc);
        H5Dclose(d);
        /* decode through the plugin */
        snprintf(dname, sizeof dname, "dec%d_%s_%s", pass, ver, name);
        d = make_dset(file, dname, type, (hsize_t)n, (hsize_t)n, block);
        int good2 = d >= 0 && H5Dwrite_chunk(d, H5P_DEFAULT, 0, off, nc, chunk) >= 0;
        unsigned char* back = malloc(no + 16);
        memset(back, 0xA5, no + 16);
        const herr_t rd = good2 ? H5Dread(d, type, H5S_ALL, H5S_ALL, H5P_DEFAULT, back) : -1;
        if (good2 && rd < 0) fprintf(stderr, "DECODE read failed %s/%s\n", ver, name);
        good2 = good2 && rd >= 0 && memcmp(back, orig, no) == 0;
        if (!good2) {
            size_t first = no, diff = 0;
            for (size_t i = 0; i < no; i++)
                if (back[i] != orig[i]) {
                    if (first == no) first = i;
                    diff++;
                }
            fprintf(stderr, "DECODE mismatch %s/%s (%zu of %zu bytes differ, first at %zu)\n", ver,
                    name, diff, no, first);
            if (getenv("H5H_DUMP") && first < no) {
                fprintf(stderr, " got   ");
                for (size_t i = first; i < no && i < first + 32; i++) fprintf(stderr, "%02x", back[i]);
                fprintf(stderr, "\n orig  ");
                for (size_t i = first; i < no && i < first + 32; i++) fprintf(stderr, "%02x", orig[i]);
                fprintf(stderr, "\n chunk ");
                for (size_t i = first; i + 12 < nc && i < first + 32; i++) fprintf(stderr, "%02x", chunk[12 + i]);
                fprintf(stderr, "\n");
            }
        }
        H5Dclose(d);
        H5Tclose(type);
        ok += good && good2;
        free(orig), free(chunk), free(got), free(back);
    }
    }
    fclose(m);
    H5Fclose(file);
    printf("regress %d/%d\n", ok, total);
    return ok == total && total == 42 * passes ? 0 : 1;
}

static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

static int roundtrip(const char* out, long long n, long long chunk) {
    uint16_t* a = malloc((size_t)n * 2);
    uint16_t* b = malloc((size_t)n * 2);
    if (!a || !b) return 2;
    for (long long i = 0; i < n; i++) {
        const uint32_t p = (uint32_t)(i & 65535), tri = p < 32768 ? p : 65536 - p;
        const uint64_t h = mix64(12345 + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull);
        a[i] = (uint16_t)((int)(tri >> 3) - 2048 + (int)(h & 31) - 16 + 32768);
    }
    hid_t file = H5Fcreate(out, H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT);
    hid_t d = make_dset(file, "data", H5T_NATIVE_UINT16, (hsize_t)n, (hsize_t)chunk, 0);
    if (d < 0) return 3;
    double t0 = now();
    if (H5Dwrite(d, H5T_NATIVE_UINT16, H5S_ALL, H5S_ALL, H5P_DEFAULT, a) < 0) return 4;
    H5Dclose(d);
    H5Fclose(file);
    double t1 = now();
    file = H5Fopen(out, H5F_ACC_RDONLY, H5P_DEFAULT);
    d = H5Dopen2(file, "data", H5P_DEFAULT);
    hsize_t stored = H5Dget_storage_size(d);
    double t2 = now();
    if (H5Dread(d, H5T_NATIVE_UINT16, H5S_ALL, H5S_ALL, H5P_DEFAULT, b) < 0) return 5;
    double t3 = now();
    H5Dclose(d);
    H5Fclose(file);
    const int same = memcmp(a, b, (size_t)n * 2) == 0;
    double fw = 0, fr = 0;
    if (getenv("BSHUF_H5_IO_FLOOR")) io_floor(out, a, b, n, chunk, &fw, &fr);
    printf("{\"config\": \"hdf5 filter 32008 uint16 G1+32768\", \"bytes\": %lld, \"chunk_bytes\": %lld, "
           "\"stored_bytes\": %llu, \"write_GBps\": %.3f, \"read_GBps\": %.3f, "
           "\"nofilter_write_GBps\": %.3f, \"nofilter_read_GBps\": %.3f, \"match\": %s}\n",
           n * 2, chunk * 2, (unsigned long long)stored, n * 2 / (t1 - t0) / 1e9,
           n * 2 / (t3 - t2) / 1e9, fw, fr, same ? "true" : "false");
    free(a), free(b);
    return same ? 0 : 1;
}

static int chunks(const char* path, const char* name) {
    hid_t file = H5Fopen(path, H5F_ACC_RDONLY, H5P_DEFAULT);
    if (file < 0) return 2;
    hid_t d = H5Dopen2(file, name, H5P_DEFAULT);
    if (d < 0) return 3;
    hid_t space = H5Dget_space(d);
    hsize_t n = 0, chunk = 0;
    H5Sget_simple_extent_dims(space, &n, NULL);
    hid_t dcpl = H5Dget_create_plist(d);
    if (H5Pget_chunk(dcpl, 1, &chunk) != 1 || chunk == 0) return 4;
    size_t cap = 0;
    unsigned char* buf = NULL;
    for (hsize_t o = 0; o < n; o += chunk) {
        hsize_t off[1] = {o}, sz = 0;
        uint32_t fm = 0;
        if (H5Dget_chunk_storage_size(d, off, &sz) < 0) return 5;
        if (sz > cap) {
            free(buf);
            cap = (size_t)sz;
            buf = malloc(cap);
            if (!buf) return 6;
        }
        if (H5Dread_chunk(d, H5P_DEFAULT, off, &fm, buf) < 0) return 7;
        if (fwrite(buf, 1, (size_t)sz, stdout) != (size_t)sz) return 8;
        fprintf(stderr, "chunk %llu %llu\n", (unsigned long long)o, (unsigned long long)sz);
    }
    fflush(stdout);
    free(buf);
    H5Pclose(dcpl);
    H5Sclose(space);
    H5Dclose(d);
    H5Fclose(file);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 4 && !strcmp(argv[1], "chunks")) return chunks(argv[2], argv[3]);
    if (argc == 4 && !strcmp(argv[1], "regress")) return regress(argv[2], argv[3]);
    if (argc == 5 && !strcmp(argv[1], "roundtrip"))
        return roundtrip(argv[2], atoll(argv[3]), atoll(argv[4]));
    fprintf(stderr, "usage: h5_harness regress DIR OUT.h5 | roundtrip OUT.h5 N CHUNK\n");
    return 2;
}
