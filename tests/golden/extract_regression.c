/*
 * extract_regression.c -- fixture generator (runs in the build container only).
 *
 * Reads the reference's regression files (tests/data/regression_{0.1.3,0.4.0}.h5,
 * written by tests/make_regression_tdata.py:14-67) with the HDF5 C API and
 * dumps, for every LZ4 dataset under /compressed:
 *   <out>/<ver>__<name>.orig   raw bytes of /original/<name>
 *   <out>/<ver>__<name>.chunk  raw stored chunk of /compressed/<name>
 *                              (12-byte filter header + bitshuffle LZ4 stream,
 *                               src/bshuf_h5filter.c:198-202)
 * and one manifest line per dataset: ver name elem_size n_elem chunk_bytes cd_values...
 * These are data (inputs and expected outputs), not reference source.
 */
#include <hdf5.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static const char* g_out;
static const char* g_ver;
static FILE* g_manifest;
static hid_t g_file;

static void sanitize(const char* in, char* out) {
    for (; *in; in++) *out++ = (*in == '|') ? 'S' : *in;
    *out = 0;
}

static void dump(const char* path, const void* buf, size_t n) {
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(buf, 1, n, f) != n) {
        perror(path);
        exit(1);
    }
    fclose(f);
}

static herr_t visit(hid_t group, const char* name, const H5L_info_t* info, void* op) {
    (void)info;
    (void)op;
    char cpath[512], opath[512], clean[256], fpath[1024];
    snprintf(cpath, sizeof cpath, "/compressed/%s", name);
    snprintf(opath, sizeof opath, "/original/%s", name);
    sanitize(name, clean);

    hid_t dc = H5Dopen2(g_file, cpath, H5P_DEFAULT);
    hid_t dorig = H5Dopen2(g_file, opath, H5P_DEFAULT);
    if (dc < 0 || dorig < 0) return -1;
    hid_t type = H5Dget_type(dorig);
    size_t esize = H5Tget_size(type);
    hid_t space = H5Dget_space(dorig);
    hssize_t n = H5Sget_simple_extent_npoints(space);

    unsigned char* orig = malloc((size_t)n * esize + 1);
    if (H5Dread(dorig, type, H5S_ALL, H5S_ALL, H5P_DEFAULT, orig) < 0) return -1;
    snprintf(fpath, sizeof fpath, "%s/%s__%s.orig", g_out, g_ver, clean);
    dump(fpath, orig, (size_t)n * esize);

    hsize_t off[1] = {0}, csz = 0;
    if (H5Dget_chunk_storage_size(dc, off, &csz) < 0) return -1;
    unsigned char* chunk = malloc(csz + 1);
    uint32_t fmask = 0;
    if (H5Dread_chunk(dc, H5P_DEFAULT, off, &fmask, chunk) < 0) return -1;
    snprintf(fpath, sizeof fpath, "%s/%s__%s.chunk", g_out, g_ver, clean);
    dump(fpath, chunk, (size_t)csz);

    hid_t dcpl = H5Dget_create_plist(dc);
    unsigned flags, cd[16];
    size_t ncd = 16;
    char fname[128];
    H5Pget_filter_by_id2(dcpl, 32008, &flags, &ncd, cd, sizeof fname, fname, NULL);
    fprintf(g_manifest, "%s %s %zu %lld %llu", g_ver, clean, esize, (long long)n,
            (unsigned long long)csz);
    for (size_t i = 0; i < ncd; i++) fprintf(g_manifest, " %u", cd[i]);
    fprintf(g_manifest, "\n");

    free(orig);
    free(chunk);
    H5Pclose(dcpl);
    H5Sclose(space);
    H5Tclose(type);
    H5Dclose(dc);
    H5Dclose(dorig);
    (void)group;
    return 0;
}

int main(int argc, char** argv) {
    if (argc != 5) {
        fprintf(stderr, "usage: %s file.h5 version outdir manifest\n", argv[0]);
        return 2;
    }
    g_ver = argv[2];
    g_out = argv[3];
    g_manifest = fopen(argv[4], "a");
    g_file = H5Fopen(argv[1], H5F_ACC_RDONLY, H5P_DEFAULT);
    if (g_file < 0) return 1;
    hid_t g = H5Gopen2(g_file, "/compressed", H5P_DEFAULT);
    hsize_t idx = 0;
    if (H5Literate(g, H5_INDEX_NAME, H5_ITER_INC, &idx, visit, NULL) < 0) return 1;
    H5Gclose(g);
    H5Fclose(g_file);
    fclose(g_manifest);
    return 0;
}
