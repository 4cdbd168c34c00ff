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

// The two-level form the device token scans run (k_seq_scan, k_seq_scan_big):
// common sequences by scan_common, every other one by scan_step.
extern "C" int bshuf_hostcheck_scan2(const uint8_t* payload, int clen, int n, uint32_t* pos,
                                     int* nseq) {
    HostReader rd{payload};
    HostOut out{pos};
    int ip = 0, op = 0, cnt = 0;
    bool fast = n >= 64;
    for (;;) {
        while (fast && ip + 1 <= clen - 17) {
            const int tok = payload[ip], lit = tok >> 4;
            const int off = payload[ip + 1 + lit] | (payload[ip + 2 + lit] << 8);
            if (!bshuf::scan_common(tok, off, ip, op, clen, n)) break;
            out.put(cnt++, (uint32_t)ip, op);
            ip += 3 + lit;
            op += lit + (tok & 15) + bshuf::kScanMinMatch;
        }
        const int r = bshuf::scan_step(rd, clen, n, out, ip, op, cnt, fast);
        if (r != bshuf::kScanCont) {
            *nseq = cnt;
            return r;
        }
    }
}
