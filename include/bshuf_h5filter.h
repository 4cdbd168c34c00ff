/*
 * bshuf_h5filter.h -- HDF5 filter 32008 ("bitshuffle") backed by the MI355X
 * codec.  Drop-in for the reference's src/bshuf_h5filter.h:14-67 and the
 * dynamic-plugin entry points of src/bshuf_h5plugin.c:17-18.
 *
 * Filter options (cd_values), unchanged from the reference
 * (src/bshuf_h5filter.c:47-64):
 *   [0] BSHUF_VERSION_MAJOR  [1] BSHUF_VERSION_MINOR  [2] element size
 *   [3] block size in elements (0 = auto)  [4] 0 or BSHUF_H5_COMPRESS_LZ4
 * With LZ4 each chunk is stored as
 *   u64 BE uncompressed bytes || u32 BE block_size*elem_size || bitshuffle LZ4 stream
 * (src/bshuf_h5filter.c:135-143, 198-202); on read the block size comes from
 * that header.  BSHUF_H5_COMPRESS_ZSTD is recognised but rejected (no zstd).
 */
#ifndef BSHUF_H5FILTER_H
#define BSHUF_H5FILTER_H

#ifdef __cplusplus
extern "C" {
#endif

#define H5Z_class_t_vers 2
#include "hdf5.h"
#include "H5PLextern.h"

#define BSHUF_H5FILTER 32008
#define BSHUF_H5_COMPRESS_LZ4 2
#define BSHUF_H5_COMPRESS_ZSTD 3

extern H5Z_class_t bshuf_H5Filter[1];

/* Register the filter in-process (for C programs not using HDF5_PLUGIN_PATH). */
int bshuf_register_h5filter(void);

/* Dynamic plugin protocol (HDF5 >= 1.8.11). */
H5PL_type_t H5PLget_plugin_type(void);
const void* H5PLget_plugin_info(void);

#ifdef __cplusplus
}
#endif

#endif /* BSHUF_H5FILTER_H */
