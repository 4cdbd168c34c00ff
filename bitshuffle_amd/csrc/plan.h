// plan.h -- blocking plan and error codes shared by the C-ABI translation
// units (api.hip: device entry points, host.hip: host-pointer entry points).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "launch.h"

namespace bshuf {

constexpr int64_t kErrHip = -70;          // no usable HIP device, or a HIP/transport error
constexpr int64_t kErrUnsupported = -71;  // an argument the device path does not take

struct Plan {
    Layout L;
    int64_t tail;  // raw tail bytes
    int64_t nb;    // nblocks
};

// Blocking of src/bitshuffle_core.c:1877-1931.
inline int64_t make_plan(size_t size, size_t elem_size, size_t block_size, Plan& p) {
    if (elem_size == 0) return kErrUnsupported;
    if (block_size == 0) {
        // bshuf_default_block_size (src/bitshuffle_core.c:2038-2046)
        block_size = 8192 / elem_size;
        block_size = (block_size / kBlockedMult) * kBlockedMult;
        if (block_size < 128) block_size = 128;
    }
    if (block_size % kBlockedMult) return -81;
    if (block_size * elem_size > (size_t)INT32_MAX / 2 || elem_size > 65536) return kErrUnsupported;
    p.L.bs = (int32_t)block_size;
    p.L.E = (int32_t)elem_size;
    p.L.nfull = (int64_t)(size / block_size);
    size_t last = size % block_size;
    last -= last % kBlockedMult;
    p.L.last = (int32_t)last;
    p.tail = (int64_t)((size % kBlockedMult) * elem_size);
    p.nb = p.L.nblocks();
    return 0;
}

inline bool have_device() {
    static int n = -1;
    if (n < 0) {
        int c = 0;
        n = (hipGetDeviceCount(&c) == hipSuccess) ? c : 0;
    }
    return n > 0;
}

}  // namespace bshuf
