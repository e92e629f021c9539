// hist_search.h -- searches over the paged HBM history.
//
// The reference walks a skip list with 16 interleaved fingers
// (SkipList.cpp:403-475, 524-553).  Here a search is two binary searches:
// first over the directory's copy of each page's first key, then inside one
// 256-slot page.  Page 0 is the default target for keys below every first key,
// so the first key of directory entry 0 is never consulted (it may be empty).
#pragma once
#include "common.h"

namespace fdbcs_dev {

__device__ inline Key dir_first(const Dir& d, int j) { return Key{d.fhi[j], d.flo[j], d.fmeta[j], d.ftail[j]}; }

__device__ inline Key pool_key(const Pool& p, int64_t slot) {
    return Key{p.hi[slot], p.lo[slot], p.meta[slot], p.tail[slot]};
}

// (Global-memory searches use the early-exit kcmp: with random keys the
// first word decides, so one 8-byte load per step.)
// Last directory entry j in [lo0-1, D) such that j == lo0-1 or first(j) <= k.
// With lo0 = 1 this is "the page a key k belongs to".
__device__ inline int dir_search(const Dir& d, int D, const Key& k, int lo0 = 1) {
    int lo = lo0, hi = D;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (kcmp(dir_first(d, mid), k) <= 0) lo = mid + 1;
        else hi = mid;
    }
    return lo - 1;
}

// First slot i in [lo, cnt) of page `page` with key(i) >= k (cnt if none).
__device__ inline int page_lb(const Pool& p, int page, int lo, int cnt, const Key& k) {
    const int64_t base = (int64_t)page * PAGE;
    int hi = cnt;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (kcmp(pool_key(p, base + mid), k) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// (pa, ia) <= (pb, ib) lexicographically
__device__ inline bool pos_le(int pa, int ia, int pb, int ib) { return pa < pb || (pa == pb && ia <= ib); }
__device__ inline bool pos_lt(int pa, int ia, int pb, int ib) { return pa < pb || (pa == pb && ia < ib); }

}  // namespace fdbcs_dev
