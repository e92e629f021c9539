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

// ------------------------------------------------- cooperative searches ----
// A group of G lanes (G divides 64, groups aligned within the wavefront)
// answers one query: each step probes G evenly spaced candidates at once, so
// a directory of ~10^5 entries takes 5 dependent loads (G = 16) instead of
// 17, a page 2 instead of 8.  Two keys are searched in lockstep so their
// loads overlap.  Every lane of a group must reach these calls together and
// with the same arguments; groups of one wavefront may diverge.
template <int G>
struct Group {
    static_assert(G >= 2 && G < 64 && (G & (G - 1)) == 0, "group size");
    int lane, shift;
    __device__ Group() {
        const int l = threadIdx.x & 63;
        lane = l & (G - 1);
        shift = l & ~(G - 1);
    }
    __device__ uint32_t ballot(bool p) const { return (uint32_t)((__ballot(p) >> shift) & ((1ull << G) - 1)); }
};

// first(j) <= k, one 8-byte load unless the high words tie
__device__ inline bool dir_le(const Dir& d, int j, const Key& k) {
    const uint64_t h = d.fhi[j];
    if (h != k.hi) return h < k.hi;
    return kcmp(dir_first(d, j), k) <= 0;
}

// narrow [lo, hi) -- the first j with pred(j) false lies in [lo, hi] -- by
// the count of true probes at lo + l*st
__device__ inline void narrow(int& lo, int& hi, int st, int cnt) {
    if (cnt == 0) {
        hi = lo;
    } else {
        const int nhi = min(hi, lo + cnt * st);
        lo = lo + (cnt - 1) * st + 1;
        hi = nhi;
    }
}

// dir_search(d, D, k1, 1) and dir_search(d, D, k2, 1) by a group of G lanes
template <int G>
__device__ inline void grp_dir_search2(const Group<G>& g, const Dir& d, int D, const Key& k1, const Key& k2, int& r1,
                                       int& r2) {
    int lo1 = 1, hi1 = D, lo2 = 1, hi2 = D;
    while (hi1 - lo1 > G || hi2 - lo2 > G) {
        const bool a1 = hi1 - lo1 > G, a2 = hi2 - lo2 > G;
        const int st1 = (hi1 - lo1 + G - 1) / G, st2 = (hi2 - lo2 + G - 1) / G;
        const int j1 = lo1 + g.lane * st1, j2 = lo2 + g.lane * st2;
        const bool le1 = a1 && j1 < hi1 && dir_le(d, j1, k1);
        const bool le2 = a2 && j2 < hi2 && dir_le(d, j2, k2);
        const int c1 = __popc(g.ballot(le1)), c2 = __popc(g.ballot(le2));
        if (a1) narrow(lo1, hi1, st1, c1);
        if (a2) narrow(lo2, hi2, st2, c2);
    }
    const int j1 = lo1 + g.lane, j2 = lo2 + g.lane;
    const bool le1 = j1 < hi1 && dir_le(d, j1, k1);
    const bool le2 = j2 < hi2 && dir_le(d, j2, k2);
    r1 = lo1 - 1 + __popc(g.ballot(le1));
    r2 = lo2 - 1 + __popc(g.ballot(le2));
}

// The same two searches over the directory's search index (Dir::sidx): one
// 16-wide window -- one 128-byte line -- per level, top level first; level 0
// (the directory itself) also fetches each candidate's page and count.
// (Staging the upper levels in LDS per workgroup was measured: the fill cost
// more than the L2-resident upper levels it replaced.)  The index holds the first 8 bytes of the keys only; a tie
// falls back to the directory entry's full key.  Windows shared by both keys
// are loaded once.
__device__ inline int sidx_n(int D, int l) {
    return (int)(((int64_t)D + (1ll << (SIDX_LOG * l)) - 1) >> (SIDX_LOG * l));
}
__device__ inline int sidx_top(int D) {
    int l = 0;
    while (sidx_n(D, l) > SIDX_B) l++;
    return l;
}

__device__ inline bool sidx_le(const Dir& d, int64_t i, int l, uint64_t v, const Key& k) {
    if (i == 0) return true;  // directory entry 0 is the default target
    if (v != k.hi) return v < k.hi;
    return kcmp(dir_first(d, (int)(i << (SIDX_LOG * l))), k) <= 0;
}

struct DirHit {
    int x, page, cnt;  // directory entry, its pool page and boundary count
};

// A query's tail words across its group: lane j holds word j (0 past the end).
template <int G>
__device__ inline uint64_t q_tail_word(const Group<G>& g, const Key& k) {
    const int len = (int)key_len(k.meta);
    const int words = len > 17 ? (len - 17 + 7) >> 3 : 0;
    return g.lane < words ? reinterpret_cast<const uint64_t*>(k.tail)[g.lane] : 0;
}

// key_bytes_at(k, s) from the group's tail words (PX_MIN_SKIP <= s <= PX_MAX_SKIP)
template <int G>
__device__ inline uint64_t q_bytes_at(const Group<G>& g, uint64_t qtw, const Key& k, int s) {
    const int t = s - 17, w = t >> 3, sh = t & 7;
    const uint64_t x0 = __builtin_bswap64((uint64_t)__shfl((long long)qtw, g.shift + w));
    const uint64_t x1 = __builtin_bswap64((uint64_t)__shfl((long long)qtw, g.shift + w + 1));
    if (s >= (int)key_len(k.meta)) return 0;
    return sh ? (x0 << (8 * sh)) | (x1 >> (64 - 8 * sh)) : x0;
}

// Probes of level l's window w (entry values v) not above k: the count.  A
// tie of the first 8 bytes is decided by the window's skip and 8 bytes of
// each key from there (common.h Dir::wsk) when it has one, else by the keys.
// spec: the level above tied, so this level's skip and 8-byte words (s0, x0)
// were loaded with v (one round trip instead of two); returns whether any
// probe tied here.
#ifndef FDBCS_PX_SPEC
#define FDBCS_PX_SPEC 1
#endif
__device__ inline const uint64_t* dir_px(const Dir& d, int l) { return l == 0 ? d.fpx : d.spx + sidx_off(d.cap, l); }
template <bool PX>
__device__ inline int dir_count(const Group<SIDX_B>& g, const Dir& d, int l, int n, int w, uint64_t v, const Key& k,
                                uint64_t qtw, bool& spec, int s0, uint64_t x0) {
    const int i = w + g.lane;
    const bool in = i < n;
    const bool tie = in && i != 0 && v == k.hi;
    bool le = in && (i == 0 || v < k.hi);
    const bool any = g.ballot(tie) != 0;
    if (any) {
        const int s = !PX ? 0 : spec ? s0 : d.wsk[wsk_off(d.cap, l) + (w >> SIDX_LOG)];
        if (s) {
            const uint64_t x = !tie ? 0 : spec ? x0 : dir_px(d, l)[i];
            const uint64_t qx = q_bytes_at(g, qtw, k, s);
            if (tie) le = x != qx ? x < qx : kcmp(dir_first(d, (int)((int64_t)i << (SIDX_LOG * l))), k) <= 0;
        } else if (tie) {
            le = kcmp(dir_first(d, (int)((int64_t)i << (SIDX_LOG * l))), k) <= 0;
        }
    }
    spec = PX && FDBCS_PX_SPEC && any;
    return __popc(g.ballot(le));
}
// (the speculative loads of a level: its window skip and the lane's word)
__device__ inline void dir_spec(const Group<SIDX_B>& g, const Dir& d, int l, int n, int w, bool spec, int& s0,
                                uint64_t& x0) {
    s0 = 0;
    x0 = 0;
    if (spec) {
        s0 = d.wsk[wsk_off(d.cap, l) + (w >> SIDX_LOG)];
        if (w + g.lane < n) x0 = dir_px(d, l)[w + g.lane];
    }
}

// dir_search(d, D, k, 1) for two keys by a group of 16 lanes
// PX: the history holds long keys (Scalars::px_on) -- the prefix skips;
// without, the plain searches (no tie bookkeeping on the hot path)
template <bool PX = false>
__device__ inline void grp_dir_find2(const Group<SIDX_B>& g, const Dir& d, int D, const Key& k1, const Key& k2,
                                     DirHit& h1, DirHit& h2) {
    int w1 = 0, w2 = 0;  // window starts (entry index at the current level)
    const uint64_t q1 = PX ? q_tail_word(g, k1) : 0, q2 = PX ? q_tail_word(g, k2) : 0;  // (long keys only)
    bool sp1 = false, sp2 = false;
    int s1, s2;
    uint64_t x1, x2;
    for (int l = sidx_top(D); l >= 1; l--) {
        const int n = sidx_n(D, l);
        const uint64_t* arr = d.sidx + sidx_off(d.cap, l);
        const int i1 = w1 + g.lane, i2 = w2 + g.lane;
        const uint64_t v1 = i1 < n ? arr[i1] : 0;
        const uint64_t v2 = w2 == w1 ? v1 : (i2 < n ? arr[i2] : 0);
        dir_spec(g, d, l, n, w1, sp1, s1, x1);
        dir_spec(g, d, l, n, w2, sp2, s2, x2);
        const int c1 = dir_count<PX>(g, d, l, n, w1, v1, k1, q1, sp1, s1, x1);  // >= 1: slot w is <= k
        const int c2 = dir_count<PX>(g, d, l, n, w2, v2, k2, q2, sp2, s2, x2);
        w1 = (w1 + c1 - 1) << SIDX_LOG;
        w2 = (w2 + c2 - 1) << SIDX_LOG;
    }
    // level 0: the directory itself, with each candidate's page and count
    const int i1 = w1 + g.lane, i2 = w2 + g.lane;
    uint64_t v1 = 0, v2 = 0;
    int pg1 = 0, cn1 = 0, pg2 = 0, cn2 = 0;
    if (i1 < D) {
        v1 = d.fhi[i1];
        pg1 = d.page[i1];
        cn1 = d.cnt[i1];
    }
    if (w2 == w1) {
        v2 = v1; pg2 = pg1; cn2 = cn1;
    } else if (i2 < D) {
        v2 = d.fhi[i2];
        pg2 = d.page[i2];
        cn2 = d.cnt[i2];
    }
    dir_spec(g, d, 0, D, w1, sp1, s1, x1);
    dir_spec(g, d, 0, D, w2, sp2, s2, x2);
    const int c1 = dir_count<PX>(g, d, 0, D, w1, v1, k1, q1, sp1, s1, x1);
    const int c2 = dir_count<PX>(g, d, 0, D, w2, v2, k2, q2, sp2, s2, x2);
    h1.x = w1 + c1 - 1;
    h2.x = w2 + c2 - 1;
    h1.page = __shfl(pg1, g.shift + c1 - 1);
    h1.cnt = __shfl(cn1, g.shift + c1 - 1);
    h2.page = __shfl(pg2, g.shift + c2 - 1);
    h2.cnt = __shfl(cn2, g.shift + c2 - 1);
}

// three-way compare of pool slot against k, one 8-byte load unless tied
__device__ inline int pool_cmp(const Pool& p, int64_t slot, const Key& k) {
    const uint64_t h = p.hi[slot];
    if (h != k.hi) return h < k.hi ? -1 : 1;
    return kcmp(pool_key(p, slot), k);
}

// Group lower bound of k in slots [0, cnt) of `page`: first i with key(i) >= k
// (cnt if none) and whether key(i) == k.
struct LbState {
    int lo, hi;
    bool hi_eq;  // key(hi) == k, when hi < cnt was probed
};

template <int G>
__device__ inline void grp_page_lb2(const Group<G>& g, const Pool& p, int page1, int cnt1, const Key& k1, int page2,
                                    int cnt2, const Key& k2, int& i1, bool& eq1, int& i2, bool& eq2) {
    const int64_t b1 = (int64_t)page1 * PAGE, b2 = (int64_t)page2 * PAGE;
    LbState s1{0, cnt1, false}, s2{0, cnt2, false};
    while (s1.hi - s1.lo > G || s2.hi - s2.lo > G) {
        const bool a1 = s1.hi - s1.lo > G, a2 = s2.hi - s2.lo > G;
        const int st1 = (s1.hi - s1.lo + G - 1) / G, st2 = (s2.hi - s2.lo + G - 1) / G;
        const int j1 = s1.lo + g.lane * st1, j2 = s2.lo + g.lane * st2;
        const int c1 = a1 && j1 < s1.hi ? pool_cmp(p, b1 + j1, k1) : 1;
        const int c2 = a2 && j2 < s2.hi ? pool_cmp(p, b2 + j2, k2) : 1;
        const uint32_t lt1 = g.ballot(c1 < 0), lt2 = g.ballot(c2 < 0);
        const uint32_t q1 = g.ballot(c1 == 0), q2 = g.ballot(c2 == 0);
        if (a1) {
            const int n = __popc(lt1), nhi = n == 0 ? s1.lo : min(s1.hi, s1.lo + n * st1);
            if (nhi < s1.hi) s1.hi_eq = (q1 >> n) & 1;  // lane n probed slot nhi
            narrow(s1.lo, s1.hi, st1, n);
        }
        if (a2) {
            const int n = __popc(lt2), nhi = n == 0 ? s2.lo : min(s2.hi, s2.lo + n * st2);
            if (nhi < s2.hi) s2.hi_eq = (q2 >> n) & 1;
            narrow(s2.lo, s2.hi, st2, n);
        }
    }
    const int j1 = s1.lo + g.lane, j2 = s2.lo + g.lane;
    const int c1 = j1 < s1.hi ? pool_cmp(p, b1 + j1, k1) : 1;
    const int c2 = j2 < s2.hi ? pool_cmp(p, b2 + j2, k2) : 1;
    const uint32_t lt1 = g.ballot(c1 < 0), lt2 = g.ballot(c2 < 0);
    const uint32_t q1 = g.ballot(c1 == 0), q2 = g.ballot(c2 == 0);
    const int n1 = __popc(lt1), n2 = __popc(lt2);
    i1 = s1.lo + n1;
    i2 = s2.lo + n2;
    eq1 = i1 < s1.hi ? ((q1 >> n1) & 1) : s1.hi_eq;
    eq2 = i2 < s2.hi ? ((q2 >> n2) & 1) : s2.hi_eq;
}

// Lower bounds of k1 in page1 [0, cnt1) and k2 in page2 [0, cnt2) by a group
// of 16 lanes with the page index: step 1 compares the 16 indexed slots
// (0, 16, ..., 240 -- one line), step 2 the 16 slots of the chosen window
// (one line).  Returns the slot and whether it holds k exactly.
struct PageWin {
    int w, e;     // window [w, e): slot w < k known, slot e >= k (or e == cnt)
    bool e_eq;    // key(e) == k (when e < cnt)
    bool done;
    int i;
    bool eq;
};

// Step 1: the 16 indexed slots.  A tie of their first 8 bytes with k (all
// of them, in a page whose keys share a long prefix) is decided by the
// page's skip and 8 bytes of each key from there (common.h Pool::pskip) when
// the page's directory window vouches for the skip (Dir::wsk of entry x):
// *ps and *qx return the skip (0: none) and k's 8 bytes for step 2.
template <bool PX>
__device__ inline void pwin_step1(const Group<PIDX_STRIDE>& g, const Pool& p, const Dir& d, int x, int page,
                                  int64_t base, int cnt, const Key& k, uint64_t v, uint64_t qtw, PageWin& W, int& ps,
                                  uint64_t& qx) {
    const int slot = g.lane * PIDX_STRIDE;
    const bool tie = slot < cnt && v == k.hi;
    int c = slot < cnt ? (v < k.hi ? -1 : 1) : 1;
    ps = 0;
    qx = 0;
    if (g.ballot(tie)) {
        if (PX) {
            const int s = p.pskip[page];
            if (s > 0 && s <= d.wsk[x >> SIDX_LOG]) ps = s;
        }
        if (ps) {
            const uint64_t u = tie ? p.pxidx[(int64_t)page * (PAGE / PIDX_STRIDE) + g.lane] : 0;
            qx = q_bytes_at(g, qtw, k, ps);
            if (tie) c = u != qx ? (u < qx ? -1 : 1) : kcmp(pool_key(p, base + slot), k);
        } else if (tie) {
            c = kcmp(pool_key(p, base + slot), k);
        }
    }
    const uint32_t lt = g.ballot(c < 0), eq = g.ballot(c == 0);
    const int n = __popc(lt);
    if (n == 0) {  // k <= key(0) (or empty page)
        W.done = true;
        W.i = 0;
        W.eq = eq & 1;
    } else {
        W.done = false;
        W.w = (n - 1) * PIDX_STRIDE;
        W.e = min(cnt, n * PIDX_STRIDE);
        W.e_eq = W.e < cnt && ((eq >> n) & 1);
    }
}

// Step 2: the 16 slots of the window; v: their first words, or with a skip
// (ps > 0) their 8 bytes from it, against qx
__device__ inline void pwin_step2(const Group<PIDX_STRIDE>& g, const Pool& p, int64_t base, const Key& k, uint64_t v,
                                  int ps, uint64_t qx, PageWin& W) {
    const int slot = W.w + g.lane;
    int c = 1;
    if (slot < W.e) {
        const uint64_t kv = ps ? qx : k.hi;
        c = v != kv ? (v < kv ? -1 : 1) : kcmp(pool_key(p, base + slot), k);
    }
    const uint32_t lt = g.ballot(c < 0), eq = g.ballot(c == 0);
    const int n = __popc(lt);  // >= 1: slot w < k
    W.i = W.w + n;
    W.eq = W.i < W.e ? ((eq >> n) & 1) : W.e_eq;
}

// x1, x2: the pages' directory entries (their window's skip, Dir::wsk)
template <bool PX = false>
__device__ inline void grp_page_find2(const Group<PIDX_STRIDE>& g, const Pool& p, const Dir& d, int x1, int page1,
                                      int cnt1, const Key& k1, int x2, int page2, int cnt2, const Key& k2, int& i1,
                                      bool& eq1, int& i2, bool& eq2) {
    const int64_t b1 = (int64_t)page1 * PAGE, b2 = (int64_t)page2 * PAGE;
    const uint64_t u1 = p.pidx[(int64_t)page1 * (PAGE / PIDX_STRIDE) + g.lane];
    const uint64_t u2 = page2 == page1 ? u1 : p.pidx[(int64_t)page2 * (PAGE / PIDX_STRIDE) + g.lane];
    const uint64_t q1 = PX ? q_tail_word(g, k1) : 0, q2 = PX ? q_tail_word(g, k2) : 0;  // (long keys only)
    PageWin W1, W2;
    int ps1, ps2;
    uint64_t qx1, qx2;
    pwin_step1<PX>(g, p, d, x1, page1, b1, cnt1, k1, u1, q1, W1, ps1, qx1);
    pwin_step1<PX>(g, p, d, x2, page2, b2, cnt2, k2, u2, q2, W2, ps2, qx2);
    const bool s1 = !W1.done, s2 = !W2.done;
    const uint64_t* a1 = ps1 ? p.px : p.hi;
    const uint64_t* a2 = ps2 ? p.px : p.hi;
    uint64_t v1 = 0, v2 = 0;
    if (s1 && W1.w + g.lane < W1.e) v1 = a1[b1 + W1.w + g.lane];
    if (s2 && W2.w + g.lane < W2.e)
        v2 = (s1 && page2 == page1 && W2.w == W1.w && ps2 == ps1) ? v1 : a2[b2 + W2.w + g.lane];
    if (s1) pwin_step2(g, p, b1, k1, v1, ps1, qx1, W1);
    if (s2) pwin_step2(g, p, b2, k2, v2, ps2, qx2, W2);
    i1 = W1.i; eq1 = W1.eq;
    i2 = W2.i; eq2 = W2.eq;
}

// ---------------------------------------------------------------- holes ----
// Real boundaries before slot i (0 <= i <= PAGE) of a page with hole mask hm.
__device__ inline int real_before(const uint64_t* hm, int i) {
    int h = 0;
#pragma unroll
    for (int w = 0; w < HM_WORDS; w++) {
        const int lo = 64 * w;
        if (i >= lo + 64) h += __popcll(hm[w]);
        else if (i > lo) h += __popcll(hm[w] & ((1ull << (i - lo)) - 1));
    }
    return i - h;
}

__device__ inline void load_hmask(const Pool& p, int page, uint64_t hm[HM_WORDS]) {
    const ulonglong2* q = reinterpret_cast<const ulonglong2*>(p.hmask + (int64_t)page * HM_WORDS);
    const ulonglong2 a = q[0], b = q[1];
    hm[0] = a.x; hm[1] = a.y; hm[2] = b.x; hm[3] = b.y;
}

// the same for a page the whole wavefront works on: the mask in scalar registers
__device__ inline uint64_t sgpr64(uint64_t x) {
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
    return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ inline void load_hmask_uniform(const Pool& p, int page, uint64_t hm[HM_WORDS]) {
    load_hmask(p, page, hm);
#pragma unroll
    for (int w = 0; w < HM_WORDS; w++) hm[w] = sgpr64(hm[w]);
}

// The slot of real boundary r (0 <= r < real count) of a page with `used`
// slots, by one wavefront (every lane gets the answer).
__device__ inline int wave_select_real(const uint64_t* hm, int used, int r) {
    const int lane = threadIdx.x & 63;
    int flags = 0, c = 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int s = 4 * lane + q;
        const int w = s >> 6;  // (selects, not a dynamic index: see hm_word)
        const uint64_t hw = w < 2 ? (w == 0 ? hm[0] : hm[1]) : (w == 2 ? hm[2] : hm[3]);
        const bool real = s < used && !((hw >> (s & 63)) & 1);
        flags |= (int)real << q;
        c += real;
    }
    int incl = c;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const int o = __shfl_up(incl, d);
        if (lane >= d) incl += o;
    }
    int res = -1;
    if (r >= incl - c && r < incl) {
        int k = r - (incl - c);
        for (int q = 0; q < 4; q++)
            if ((flags >> q) & 1) {
                if (k == 0) {
                    res = 4 * lane + q;
                    break;
                }
                k--;
            }
    }
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) res = max(res, __shfl_xor(res, d));
    return res;
}

// (pa, ia) <= (pb, ib) lexicographically
__device__ inline bool pos_le(int pa, int ia, int pb, int ib) { return pa < pb || (pa == pb && ia <= ib); }
__device__ inline bool pos_lt(int pa, int ia, int pb, int ib) { return pa < pb || (pa == pb && ia < ib); }

}  // namespace fdbcs_dev
