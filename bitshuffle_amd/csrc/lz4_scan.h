// lz4_scan.h -- the control flow of LZ4_decompress_safe without the copies:
// accept/reject, error position, and the token position of every sequence.
// Shared by the device scan (k_seq_scan, lz4_decode.hip) and a host build
// (scan_host.cpp, loaded only by the CPU tests), so the exact state machine
// the GPU runs is also checked against the oracle without a GPU.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define BSHUF_HD __host__ __device__
#else
#define BSHUF_HD
#endif

namespace bshuf {

constexpr int kScanMinMatch = 4;

// read_variable_length (lz4/lz4.c:1978-2014) over the lane's window.
template <class Rd>
BSHUF_HD inline bool scan_len(Rd& rd, int& ip, int ilimit, bool initial_check, int& len) {
    if (initial_check && ip >= ilimit) return false;
    int s = (int)rd(ip++);
    len = s;
    if (ip > ilimit) return false;
    while (s == 255) {
        s = (int)rd(ip++);
        len += s;
        if (ip > ilimit) return false;
    }
    return true;
}

// The control flow of LZ4_decompress_safe (LZ4 1.10.0, lz4/lz4.c:2022-2445;
// restated and pinned against the compiled reference in oracle/bshuf_oracle.c)
// without the copies: the fast loop (2083-2209) and the safe loop (2215-2435)
// check different margins, so both are followed to reach the same accept /
// reject decision and error position.  Records each sequence's token position.
// Returns op (bytes the block decodes to) or -(ip)-1.  Token positions go to
// out.put(i, pos, op) in increasing i, with op the output position where that
// sequence starts (a rejected block may have put one more).
template <class Rd, class Out>
BSHUF_HD inline int scan_block(Rd& rd, const int clen, const int n, Out& out, int& cnt) {
    enum { kNone, kLit, kCopyMatch, kMatch };
    int ip = 0, op = 0;
    cnt = 0;
    bool fast = n >= 64;  // FASTLOOP_SAFE_DISTANCE
    for (;;) {
        const int tp = ip;
        const int tok = (int)rd(ip++);
        int len = tok >> 4, ml = 0, off = 0, add = 0;
        int entry = kNone;
        if (fast) {
            if (len == 15) {
                if (!scan_len(rd, ip, clen - 15, true, add)) return -ip - 1;
                len += add;
                if (op + len > n - 32 || ip + len > clen - 32) entry = kLit;
            } else if (ip > clen - 17) {
                entry = kLit;
            }
            if (entry == kNone) {
                out.put(cnt++, (uint32_t)tp, op);
                ip += len;
                op += len;
                off = (int)(rd(ip) | (rd(ip + 1) << 8));
                ip += 2;
                ml = tok & 15;
                if (ml == 15) {
                    if (!scan_len(rd, ip, clen - 4, false, add)) return -ip - 1;
                    ml += add + kScanMinMatch;
                    if (op + ml >= n - 64) entry = kMatch;
                } else {
                    ml += kScanMinMatch;
                    if (op + ml >= n - 64) {
                        entry = kMatch;
                    } else if (off >= 8 && off <= op) {
                        op += ml;
                        continue;
                    }
                }
                if (entry == kNone) {
                    if (off > op) return -ip - 1;
                    op += ml;
                    continue;
                }
            }
            fast = false;  // the rest of the block runs in the safe loop
        } else {
            if (len != 15 && ip < clen - 16 && op <= n - 32) {
                out.put(cnt++, (uint32_t)tp, op);
                ip += len;
                op += len;
                ml = tok & 15;
                off = (int)(rd(ip) | (rd(ip + 1) << 8));
                ip += 2;
                if (ml != 15 && off >= 8 && off <= op) {
                    op += ml + kScanMinMatch;
                    continue;
                }
                entry = kCopyMatch;
            } else {
                if (len == 15) {
                    if (!scan_len(rd, ip, clen - 15, true, add)) return -ip - 1;
                    len += add;
                }
                entry = kLit;
            }
        }
        if (entry == kLit) {
            out.put(cnt++, (uint32_t)tp, op);
            const int cpy = op + len;
            if (cpy > n - 12 || ip + len > clen - 8) {
                // must be the last sequence: consume the input exactly
                if (ip + len != clen || cpy > n) {
                    cnt--;
                    return -ip - 1;
                }
                return cpy;
            }
            ip += len;
            op = cpy;
            off = (int)(rd(ip) | (rd(ip + 1) << 8));
            ip += 2;
            ml = tok & 15;
            entry = kCopyMatch;
        }
        if (entry == kCopyMatch) {
            if (ml == 15) {
                if (!scan_len(rd, ip, clen - 4, false, add)) return -ip - 1;
                ml += add;
            }
            ml += kScanMinMatch;
        }
        // safe_match_copy
        if (off > op) return -ip - 1;
        if (op + ml > n - 5) return -ip - 1;  // the last LASTLITERALS bytes are literals
        op += ml;
    }
}

}  // namespace bshuf
