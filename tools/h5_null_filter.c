/* h5_null_filter.c -- measurement aid for config 5: an HDF5
 * dynamic plugin that registers filter id 32008 with a pass-through callback
 * (the chunk buffer goes back unchanged).  Timing the same h5_harness
 * roundtrip through it gives HDF5's own filtered-I/O floor: chunk buffers,
 * the filter pipeline and file I/O with zero codec work.  Never a product. */
#include <H5PLextern.h>
#include <H5Zpublic.h>

static size_t null_filter(unsigned flags, size_t cd_nelmts, const unsigned cd_values[], size_t nbytes,
                          size_t* buf_size, void** buf) {
    (void)flags, (void)cd_nelmts, (void)cd_values, (void)buf_size, (void)buf;
    return nbytes;
}

static const H5Z_class2_t null_class = {H5Z_CLASS_T_VERS, (H5Z_filter_t)32008, 1, 1,
                                        "pass-through (timing floor)", NULL, NULL, null_filter};

H5PL_type_t H5PLget_plugin_type(void) { return H5PL_TYPE_FILTER; }
const void* H5PLget_plugin_info(void) { return &null_class; }
