// stage_pack.h -- the add's per-range work (TxnStage::add, stage.hip): check
// begin < end and copy a transaction's ranges into its stream record.  Host
// code only, header-only so that tests/native/stage_pack_fuzz.cpp checks it
// against a plain restatement without a GPU.
#pragma once

#include <emmintrin.h>

#include <algorithm>
#include <cstdint>
#include <cstring>

#include "../../include/fdbcs.h"

// Keys up to this long are copied whole, both of them, whatever the range
// (no shared end for a point range); longer point ranges store k\x00 once.
#ifndef FDBCS_PACK_SHARE_ABOVE
#define FDBCS_PACK_SHARE_ABOVE 32  // (A/B: 0 shares every point range, as round 4's add did)
#endif

namespace fdbcs_pack {

// ~70,000 short keys per config-2 batch: inline word compares and copies
// instead of a libc call per key (measured: 185 -> ~110 us per batch).
inline uint64_t ld64(const uint8_t* p) {
    uint64_t x;
    memcpy(&x, p, 8);
    return x;
}

// the first 16 bytes as one big-endian number
inline unsigned __int128 be128(const uint8_t* p) {
    return (unsigned __int128)__builtin_bswap64(ld64(p)) << 64 | __builtin_bswap64(ld64(p + 8));
}

// Keys longer than 16 bytes, equal in their first 16 (config 4: a 64-byte
// tenant prefix): 16 bytes a step, the last step overlapping the one before
// it, where a word and a byte loop ran up to 15 data-dependent iterations.
// (Out of line: the 16-byte keys' path stays as compact as before.)
__attribute__((noinline)) inline int key_cmp_long(const uint8_t* a, const uint8_t* b, uint32_t n, int lc) {
    for (uint32_t i = 16;; i += 16) {
        const uint32_t j = std::min(i, n - 16);
        const __m128i u = _mm_loadu_si128(reinterpret_cast<const __m128i*>(a + j));
        const __m128i v = _mm_loadu_si128(reinterpret_cast<const __m128i*>(b + j));
        const uint32_t m = (uint32_t)_mm_movemask_epi8(_mm_cmpeq_epi8(u, v)) ^ 0xFFFFu;
        if (m) {
            const uint32_t k = j + (uint32_t)__builtin_ctz(m);
            return a[k] < b[k] ? -1 : 1;
        }
        if (j + 16 >= n) return lc;
    }
}

// the reference's key order (SkipList.cpp:113-120); -2: a is a proper prefix
// of b (so a < b).  Keys of 16 bytes or more compare their first 16 bytes with
// carry-flag arithmetic and no jump on the bytes: in config 2 one read in five
// is a short range [k, k + d) among point ranges [k, k\x00), in random order,
// and a jump on where the keys first differ mispredicted once per short range.
__attribute__((always_inline)) inline int key_cmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t n = std::min(al, bl);
    const int lc = al < bl ? -2 : (al > bl ? 1 : 0);
    uint32_t i = 0;
    if (n >= 16) {
        const unsigned __int128 x = be128(a), y = be128(b);
        const int gt = (int)(x > y), lt = (int)(x < y);
        const int eq = 1 - gt - lt;
        // (the one jump depends on the lengths alone: past 16 equal bytes of longer keys)
        if (__builtin_expect((eq & (int)(n > 16)) == 0, 1)) return gt - lt + eq * lc;
        return key_cmp_long(a, b, n, lc);
    }
    for (; i + 8 <= n; i += 8) {
        const uint64_t x = ld64(a + i), y = ld64(b + i);
        if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y) ? -1 : 1;
    }
    for (; i < n; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return lc;
}

// n > 32 bytes: up to 128 (config 4's 68-100-byte keys) in 16-byte pieces,
// the last one overlapping, instead of a libc call per key (out of line, as
// key_cmp_long)
__attribute__((noinline)) inline void copy_long(uint8_t* d, const uint8_t* s, uint32_t n) {
    if (n > 128) {
        memcpy(d, s, n);
        return;
    }
    for (uint32_t i = 0; i < n; i += 16) {
        const uint32_t j = std::min(i, n - 16);
        uint8_t t[16];
        memcpy(t, s + j, 16);
        memcpy(d + j, t, 16);
    }
}

// copy n bytes; reads and writes stay inside the n bytes
__attribute__((always_inline)) inline void copy_small(uint8_t* d, const uint8_t* s, uint32_t n) {
    if (n >= 16 && n <= 32) {
        uint8_t t0[16], t1[16];
        memcpy(t0, s, 16);
        memcpy(t1, s + n - 16, 16);
        memcpy(d, t0, 16);
        memcpy(d + n - 16, t1, 16);
    } else if (n >= 8 && n < 16) {
        const uint64_t x = ld64(s), y = ld64(s + n - 8);
        memcpy(d, &x, 8);
        memcpy(d + n - 8, &y, 8);
    } else if (n > 32) {
        copy_long(d, s, n);
    } else {
        for (uint32_t i = 0; i < n; i++) d[i] = s[i];
    }
}

// Check and copy ranges into the record at rec: entries (where the keys are,
// their lengths) and the key bytes at kp (advanced); true if some range has
// begin >= end.
//   keys up to FDBCS_PACK_SHARE_ABOVE bytes: both keys, begin then end, so
//     that nothing the add does depends on the keys' bytes but the compare's
//     result -- no jump, and the cursor advances by the lengths alone.  When a
//     point range wrote k\x00 once and a short range both keys, the jump on
//     which one it was mispredicted once per short range (config 2, adds
//     only, same batch: 164-176 us shared against 150-159 us copied; the
//     stream grows by 16 bytes per point range);
//   longer keys: a point range [k, k\x00) is written as k\x00 once (flag
//     SHARED in the entry's end length; kernels.h STAGE_SHARED), which saves
//     a long key's copy and its PCIe bytes.
template <class Ent, uint16_t SHARED, uint32_t SHARE_ABOVE = FDBCS_PACK_SHARE_ABOVE>
__attribute__((always_inline)) inline bool put_ranges(const fdbcs_range* rg, int n, Ent* ent, const uint8_t* rec,
                                                      uint8_t*& kp_io) {
    // (a local cursor: kp_io itself may alias the bytes stored through it, so
    // the compiler would store and reload it around every key copy)
    uint8_t* kp = kp_io;
    bool bad = false;
    for (int i = 0; i < n; i++) {
        const uint8_t *b = rg[i].begin, *e = rg[i].end;
        const uint32_t bl = rg[i].begin_len, el = rg[i].end_len;
        const int c = key_cmp(b, bl, e, el);
        bad |= c >= 0;
        if (bl <= SHARE_ABOVE) {
            if (bl == 16) memcpy(kp, b, 16);  // (the configs' 16-byte keys: one store)
            else copy_small(kp, b, bl);
            copy_small(kp + bl, e, el);
            ent[i] = Ent{(uint32_t)(kp - rec), (uint16_t)bl, (uint16_t)el};
            kp += bl + el;
            continue;
        }
        copy_small(kp, b, bl);
        if (c == -2 && el == bl + 1 && e[bl] == 0) {  // point range: k then one 0 byte
            ent[i] = Ent{(uint32_t)(kp - rec), (uint16_t)bl, (uint16_t)(el | SHARED)};
            kp[bl] = 0;
            kp += bl + 1;
        } else {
            ent[i] = Ent{(uint32_t)(kp - rec), (uint16_t)bl, (uint16_t)el};
            copy_small(kp + bl, e, el);
            kp += bl + el;
        }
    }
    kp_io = kp;
    return bad;
}

// The key bytes put_ranges<_, _, SHARE_ABOVE> writes for a transaction's
// ranges (reads, then writes: n of them in all) and its status as the add
// would refuse it -- FDBCS_E_KEY (a key over FDBCS_MAX_KEY, any range) before
// FDBCS_E_RANGE (begin >= end) -- for the borrowed batches' first pass at
// detect (stage.hip TxnStage::pack_borrowed).
template <uint32_t SHARE_ABOVE>
inline uint64_t ranges_bytes(const fdbcs_range* rd, int nr, const fdbcs_range* wr, int nw, int& status) {
    uint64_t k = 0;
    bool range_bad = false;
    status = FDBCS_OK;
    for (int i = 0; i < nr + nw; i++) {
        const fdbcs_range& g = i < nr ? rd[i] : wr[i - nr];
        const uint8_t *b = g.begin, *e = g.end;
        const uint32_t bl = g.begin_len, el = g.end_len;
        if (bl > FDBCS_MAX_KEY || el > FDBCS_MAX_KEY) {
            status = FDBCS_E_KEY;
            return 0;
        }
        const int c = key_cmp(b, bl, e, el);
        range_bad |= c >= 0;
        k += bl <= SHARE_ABOVE || !(c == -2 && el == bl + 1 && e[bl] == 0) ? bl + el : bl + 1;
    }
    if (range_bad) status = FDBCS_E_RANGE;
    return k;
}

}  // namespace fdbcs_pack
