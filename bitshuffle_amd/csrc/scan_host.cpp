// Host build of the decoder's scan state machine (lz4_scan.h) for the CPU
// test suite (tests/test_scan_host.py).  Not part of the product library.
#include <stdint.h>

#include "lz4_scan.h"

namespace {
struct HostReader {
    const uint8_t* P;
    uint32_t operator()(int p) const { return P[p]; }
};
struct HostOut {
    uint32_t* pos;
    void put(int i, uint32_t v, int op) {
        pos[i] = v;
        (void)op;
    }
};
}  // namespace

extern "C" int bshuf_hostcheck_scan(const uint8_t* payload, int clen, int n, uint32_t* pos,
                                    int* nseq) {
    HostReader rd{payload};
    HostOut out{pos};
    int cnt = 0;
    const int r = bshuf::scan_block(rd, clen, n, out, cnt);
    *nseq = cnt;
    return r;
}
