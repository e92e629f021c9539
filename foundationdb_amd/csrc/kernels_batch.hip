// kernels_batch.hip -- batch-side stages of ConflictBatch::detectConflicts.
//
//   prep        addTransaction's tooOld rule            SkipList.cpp:979-1008
//   encode      key -> (hi, lo, meta, tail) records      (replaces KeyInfo/getCharacter, :134-177)
//   read check  checkReadConflictRanges / CheckMax       :1210-1233, :755-837
//   sort        begin keys of reads and of writes        (replaces sortPoints, :227-279)
//   edges       read x write overlaps, u < t             (replaces MiniConflictSet ranks, :1028-1130)
//   decide      ordered commit decision                  checkIntraBatchConflicts :1133-1153
//   combine     union of committed writes                combineWriteConflictRanges :1320-1337
#include <algorithm>
#include "kernels.h"
#include "devutil.h"
#include "hist_search.h"

namespace fdbcs_dev {


// ---------------------------------------------------------------- prep ----
__global__ __launch_bounds__(256) void k_prep(int T, const int64_t* __restrict__ snap, const int32_t* __restrict__ ro,
                                              const int32_t* __restrict__ wo, int64_t oldest,
                                              uint8_t* __restrict__ too_old, uint8_t* __restrict__ hist,
                                              int32_t* __restrict__ read_txn, int32_t* __restrict__ write_txn,
                                              int32_t* __restrict__ deg, int32_t* __restrict__ cur) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= T) return;
    const int r0 = ro[t], r1 = ro[t + 1];
    // tooOld uses the previous batch's oldestVersion and needs >= 1 read (SkipList.cpp:985)
    too_old[t] = (snap[t] < oldest && r1 > r0) ? 1 : 0;
    hist[t] = 0;
    deg[t] = 0;
    cur[t] = 0;
    for (int r = r0; r < r1; r++) read_txn[r] = t;
    for (int w = wo[t], w1 = wo[t + 1]; w < w1; w++) write_txn[w] = t;
}

void launch_prep(const fdbcs_batch_view& v, int64_t oldest, BatchBufs& b, Scalars* sc, hipStream_t s) {
    (void)sc;
    if (v.txn_count == 0) return;
    hipLaunchKernelGGL(k_prep, dim3(cdiv(v.txn_count, 256)), dim3(256), 0, s, v.txn_count, v.snapshot, v.read_off,
                       v.write_off, oldest, b.too_old, b.hist, b.read_txn, b.write_txn, b.deg, b.cur);
}

// -------------------------------------------------------------- encode ----
__global__ __launch_bounds__(256) void k_encode(int64_t nslots, const uint64_t* __restrict__ koff,
                                                const uint32_t* __restrict__ klen, const uint8_t* __restrict__ bytes,
                                                KeyArrays out, uint8_t* __restrict__ btail, uint64_t btail_cap,
                                                Scalars* sc) {
    const int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (s >= nslots) return;
    const uint8_t* p = bytes + koff[s];
    uint32_t L = klen[s];
    if (L > FDBCS_MAX_KEY) {
        atomicCAS(&sc->err, 0, FDBCS_E_KEY);
        L = FDBCS_MAX_KEY;
    }
    uint64_t hi = 0, lo = 0;
    uint32_t b16 = 0;
    const uint32_t n = L < 17 ? L : 17;
    for (uint32_t i = 0; i < n; i++) {
        uint64_t c = p[i];
        if (i < 8) hi |= c << (56 - 8 * i);
        else if (i < 16) lo |= c << (56 - 8 * (i - 8));
        else b16 = (uint32_t)c;
    }
    const uint8_t* tail = nullptr;
    if (L > 17) {
        const uint64_t m = L - 17, padded = (m + 7) & ~7ull;
        const uint64_t o = atomicAdd((unsigned long long*)&sc->btail_used, (unsigned long long)padded);
        if (o + padded > btail_cap) {
            atomicCAS(&sc->err, 0, FDBCS_E_CAPACITY);
        } else {
            uint8_t* d = btail + o;
            for (uint64_t i = 0; i < padded; i++) d[i] = i < m ? p[17 + i] : 0;
            tail = d;
        }
    }
    out.hi[s] = hi;
    out.lo[s] = lo;
    out.meta[s] = (b16 << 24) | L;
    out.tail[s] = tail;
}

// every range must be non-empty: reference precondition
__global__ __launch_bounds__(256) void k_validate(int64_t nranges, KeyArrays k, Scalars* sc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= nranges) return;
    if (kcmp(k.get(2 * i), k.get(2 * i + 1)) >= 0) atomicCAS(&sc->err, 0, FDBCS_E_RANGE);
}

void launch_encode(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, hipStream_t s) {
    const int64_t nr = (int64_t)v.read_count + v.write_count;
    if (nr == 0) return;
    hipLaunchKernelGGL(k_encode, dim3(cdiv(2 * nr, 256)), dim3(256), 0, s, 2 * nr, v.key_off, v.key_len, v.key_bytes,
                       b.keys, b.btail, b.btail_cap, sc);
    hipLaunchKernelGGL(k_validate, dim3(cdiv(nr, 256)), dim3(256), 0, s, nr, b.keys, sc);
}

// ---------------------------------------------------------- read check ----
// One lane per read range.  conflict iff max(version over boundaries in
// [b, e), plus valueBefore(b) if b is not a boundary) > snapshot -- the
// predicate CheckMax evaluates on the skip list (SkipList.cpp:755-837;
// SURVEY.md Appendix A step 1).  Pages fully inside the range are skipped
// through the directory's per-page maxima (the skip list's upper-level
// maxVersion plays this role in the reference).
__global__ __launch_bounds__(256) void k_read_check(int R, KeyArrays keys, const int32_t* __restrict__ read_txn,
                                                    const int64_t* __restrict__ snap,
                                                    const uint8_t* __restrict__ too_old, uint8_t* __restrict__ hist,
                                                    Pool pool, Dir dir, const Scalars* __restrict__ sc, int64_t v0) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const int t = read_txn[r];
    if (too_old[t]) return;
    const int64_t s = snap[t];
    const Key b = keys.get(2 * (int64_t)r), e = keys.get(2 * (int64_t)r + 1);
    const int D = sc->D;
    const int pb = dir_search(dir, D, b, 1);
    const int cb = dir.cnt[pb], pgb = dir.page[pb];
    const int64_t baseb = (int64_t)pgb * PAGE;
    const int ib = page_lb(pool, pgb, 0, cb, b);
    bool conflict = false;
    const bool exact = ib < cb && kcmp(pool_key(pool, baseb + ib), b) == 0;
    if (!exact) {
        const int64_t vb = ib > 0 ? pool.ver[baseb + ib - 1] : v0;
        conflict = vb > s;
    }
    if (!conflict) {
        int pe = pb;
        if (pb + 1 < D && kcmp(dir_first(dir, pb + 1), e) <= 0) pe = dir_search(dir, D, e, pb + 1);
        if (pe == pb) {
            const int ie = page_lb(pool, pgb, ib, cb, e);
            for (int i = ib; i < ie && !conflict; i++) conflict = pool.ver[baseb + i] > s;
        } else {
            for (int i = ib; i < cb && !conflict; i++) conflict = pool.ver[baseb + i] > s;
            int q = pb + 1;
            while (q < pe && !conflict) {
                if ((q & 63) == 0 && q + 64 <= pe) {
                    conflict = dir.bmax[q >> 6] > s;
                    q += 64;
                } else {
                    conflict = dir.maxv[q] > s;
                    q++;
                }
            }
            if (!conflict) {
                const int pge = dir.page[pe], ce = dir.cnt[pe];
                const int64_t basee = (int64_t)pge * PAGE;
                const int ie = page_lb(pool, pge, 0, ce, e);
                for (int i = 0; i < ie && !conflict; i++) conflict = pool.ver[basee + i] > s;
            }
        }
    }
    if (conflict) hist[t] = 1;
}

void launch_read_check(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t v0,
                       hipStream_t s) {
    if (v.read_count == 0) return;
    hipLaunchKernelGGL(k_read_check, dim3(cdiv(v.read_count, 256)), dim3(256), 0, s, v.read_count, b.keys,
                       b.read_txn, v.snapshot, b.too_old, b.hist, h.pool, h.dir[cur], sc, v0);
}

// ---------------------------------------------------------------- sort ----
// Merge sort of range begin keys: bitonic sort of 1024-record tiles in LDS,
// then merge passes where every record finds its rank in the partner run by
// binary search.  Ties between equal keys are irrelevant downstream (SURVEY.md
// Appendix A, note on ties), so stability is not needed.
static constexpr uint32_t INVALID = 0xFFFFFFFFu;
static constexpr int SORT_TILE = 1024;

__device__ inline Key rec_key(const SRec& r, const uint8_t* const* tails, int64_t slot_base) {
    return Key{r.hi, r.lo, r.meta, key_len(r.meta) > 17 ? tails[slot_base + 2 * (int64_t)r.idx] : nullptr};
}

__device__ inline bool rec_less(const SRec& a, const SRec& b, const uint8_t* const* tails, int64_t slot_base) {
    if (a.idx == INVALID) return false;
    if (b.idx == INVALID) return true;
    return kcmp(rec_key(a, tails, slot_base), rec_key(b, tails, slot_base)) < 0;
}

__global__ __launch_bounds__(256) void k_block_sort(int n, KeyArrays keys, int64_t slot_base, SRec* __restrict__ out) {
    __shared__ SRec sm[SORT_TILE];
    const int base = blockIdx.x * SORT_TILE;
    for (int i = threadIdx.x; i < SORT_TILE; i += blockDim.x) {
        const int g = base + i;
        if (g < n) {
            const int64_t slot = slot_base + 2 * (int64_t)g;
            sm[i] = SRec{keys.hi[slot], keys.lo[slot], keys.meta[slot], (uint32_t)g};
        } else {
            sm[i] = SRec{~0ull, ~0ull, ~0u, INVALID};
        }
    }
    __syncthreads();
    for (int k = 2; k <= SORT_TILE; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < SORT_TILE; i += blockDim.x) {
                const int ixj = i ^ j;
                if (ixj > i) {
                    const SRec a = sm[i], c = sm[ixj];
                    const bool up = (i & k) == 0;
                    const bool sw = up ? rec_less(c, a, keys.tail, slot_base) : rec_less(a, c, keys.tail, slot_base);
                    if (sw) {
                        sm[i] = c;
                        sm[ixj] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (int i = threadIdx.x; i < SORT_TILE; i += blockDim.x) {
        const int g = base + i;
        if (g < n) out[g] = sm[i];
    }
}

__global__ __launch_bounds__(256) void k_merge_pass(int n, int width, const SRec* __restrict__ in,
                                                    SRec* __restrict__ out, const uint8_t* const* tails,
                                                    int64_t slot_base) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const int run = i / width;
    const int base = (run & ~1) * width;
    const int a0 = base, a1 = min(n, base + width);
    const int b0 = a1, b1 = min(n, base + 2 * width);
    const SRec x = in[i];
    if (run & 1) {  // x in run B: count A records <= x
        int lo = a0, hi = a1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (!rec_less(x, in[mid], tails, slot_base)) lo = mid + 1;
            else hi = mid;
        }
        out[base + (i - b0) + (lo - a0)] = x;
    } else {        // x in run A: count B records < x
        int lo = b0, hi = b1;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (rec_less(in[mid], x, tails, slot_base)) lo = mid + 1;
            else hi = mid;
        }
        out[base + (i - a0) + (lo - b0)] = x;
    }
}

static SRec* sort_one(int n, KeyArrays keys, int64_t slot_base, SRec* buf0, SRec* buf1, hipStream_t s) {
    if (n == 0) return buf0;
    hipLaunchKernelGGL(k_block_sort, dim3(cdiv(n, SORT_TILE)), dim3(256), 0, s, n, keys, slot_base, buf0);
    SRec* src = buf0;
    SRec* dst = buf1;
    for (int width = SORT_TILE; width < n; width <<= 1) {
        hipLaunchKernelGGL(k_merge_pass, dim3(cdiv(n, 256)), dim3(256), 0, s, n, width, (const SRec*)src, dst,
                           (const uint8_t* const*)keys.tail, slot_base);
        std::swap(src, dst);
    }
    return src;
}

void launch_sort_ranges(const fdbcs_batch_view& v, BatchBufs& b, hipStream_t s) {
    b.sr = sort_one(v.read_count, b.keys, 0, b.rec_r0, b.rec_r1, s);
    b.sw = sort_one(v.write_count, b.keys, 2 * (int64_t)v.read_count, b.rec_w0, b.rec_w1, s);
}

// --------------------------------------------------------------- edges ----
// A read r of t and a write w of u overlap iff r.b < w.e && w.b < r.e.
// Split on which begin comes first (keys only, no ranks):
//   w.b >= r.b : w in  [lower_bound(W, r.b), lower_bound(W, r.e))  (by reader)
//   w.b <  r.b : r in  [upper_bound(R, w.b), lower_bound(R, w.e))  (by writer)
// Only pairs u < t where both are still undecided (not tooOld, no history
// conflict) matter.  A T x T bit matrix dedups pairs: pass 0 sets bits and
// counts unique sources per reader; pass 1 clears them and emits each pair
// exactly once, leaving the matrix zero for the next batch.
__device__ inline int lb_rec(const SRec* a, int n, const Key& k, const uint8_t* const* tails, int64_t slot_base) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (kcmp(rec_key(a[mid], tails, slot_base), k) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ inline int ub_rec(const SRec* a, int n, const Key& k, const uint8_t* const* tails, int64_t slot_base) {
    int lo = 0, hi = n;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (kcmp(rec_key(a[mid], tails, slot_base), k) <= 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

template <int PASS>
__device__ inline void edge_pair(int t, int u, uint32_t* bits, int row_words, int32_t* deg, const int32_t* off,
                                 int32_t* cur, int32_t* edges) {
    uint32_t* word = bits + (int64_t)t * row_words + (u >> 5);
    const uint32_t bit = 1u << (u & 31);
    if (PASS == 0) {
        const uint32_t old = atomicOr(word, bit);
        if (!(old & bit)) atomicAdd(&deg[t], 1);
    } else {
        const uint32_t old = atomicAnd(word, ~bit);
        if (old & bit) edges[off[t] + atomicAdd(&cur[t], 1)] = u;
    }
}

template <int PASS>
__global__ __launch_bounds__(256) void k_edges(int R, int W, KeyArrays keys, const SRec* __restrict__ sr,
                                               const SRec* __restrict__ sw, const int32_t* __restrict__ read_txn,
                                               const int32_t* __restrict__ write_txn,
                                               const uint8_t* __restrict__ too_old, const uint8_t* __restrict__ hist,
                                               uint32_t* bits, int row_words, int32_t* deg, const int32_t* off,
                                               int32_t* cur, int32_t* edges) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t wbase = 2 * (int64_t)R;
    if (i < R) {
        const int t = read_txn[i];
        if (too_old[t] || hist[t]) return;
        const Key b = keys.get(2 * (int64_t)i), e = keys.get(2 * (int64_t)i + 1);
        const int lo = lb_rec(sw, W, b, keys.tail, wbase);
        const int hi = lb_rec(sw, W, e, keys.tail, wbase);
        for (int k = lo; k < hi; k++) {
            const int u = write_txn[sw[k].idx];
            if (u < t && !too_old[u] && !hist[u]) edge_pair<PASS>(t, u, bits, row_words, deg, off, cur, edges);
        }
    } else if (i < R + W) {
        const int w = i - R;
        const int u = write_txn[w];
        if (too_old[u] || hist[u]) return;
        const Key b = keys.get(wbase + 2 * (int64_t)w), e = keys.get(wbase + 2 * (int64_t)w + 1);
        const int lo = ub_rec(sr, R, b, keys.tail, 0);
        const int hi = lb_rec(sr, R, e, keys.tail, 0);
        for (int k = lo; k < hi; k++) {
            const int t = read_txn[sr[k].idx];
            if (t > u && !too_old[t] && !hist[t]) edge_pair<PASS>(t, u, bits, row_words, deg, off, cur, edges);
        }
    }
}

void launch_edges(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, hipStream_t s) {
    const int R = v.read_count, W = v.write_count, T = v.txn_count;
    const int n = R + W;
    if (n > 0 && R > 0 && W > 0) {
        hipLaunchKernelGGL(k_edges<0>, dim3(cdiv(n, 256)), dim3(256), 0, s, R, W, b.keys, (const SRec*)b.sr,
                           (const SRec*)b.sw, b.read_txn, b.write_txn, b.too_old, b.hist, b.pair_bits, b.row_words,
                           b.deg, b.off, b.cur, b.edges);
    }
    scan_i32(b.deg, b.off, nullptr, T, &sc->edges_total, b.scan_tmp, s);
    if (n > 0 && R > 0 && W > 0) {
        hipLaunchKernelGGL(k_edges<1>, dim3(cdiv(n, 256)), dim3(256), 0, s, R, W, b.keys, (const SRec*)b.sr,
                           (const SRec*)b.sw, b.read_txn, b.write_txn, b.too_old, b.hist, b.pair_bits, b.row_words,
                           b.deg, b.off, b.cur, b.edges);
    }
}

// -------------------------------------------------------------- decide ----
// The order-dependent decision of checkIntraBatchConflicts (SkipList.cpp:
// 1133-1153): conflict[t] = tooOld[t] || hist[t] || some source u < t (an
// earlier txn with a write overlapping a read of t) committed.  Txns without
// sources are decided in parallel.  Dependents are walked in index order in
// chunks of 64 by one wavefront: each lane folds in its sources from earlier
// chunks (final), then the chunk's 64x64 lower-triangular dependency masks are
// resolved by a Jacobi iteration on ballots, which reaches the unique
// solution of the recurrence in at most depth+1 rounds.
__global__ __launch_bounds__(1024) void k_decide(int T, const uint8_t* __restrict__ too_old,
                                                 const uint8_t* __restrict__ hist, const int32_t* __restrict__ deg,
                                                 const int32_t* __restrict__ off, const int32_t* __restrict__ edges,
                                                 int32_t* __restrict__ dep_list, int32_t* __restrict__ dep_idx,
                                                 uint8_t* __restrict__ committed, uint8_t* __restrict__ verdict,
                                                 Scalars* sc) {
    extern __shared__ uint32_t cbits[];
    __shared__ int32_t tmp[1024 / 64 + 1];
    const int nwords = (T + 31) >> 5;
    for (int i = threadIdx.x; i < nwords; i += blockDim.x) cbits[i] = 0;
    __syncthreads();
    int ndep = 0;
    for (int base = 0; base < T; base += blockDim.x) {
        const int t = base + threadIdx.x;
        const bool valid = t < T;
        const bool und = valid && !too_old[t] && !hist[t];
        const int d = valid ? deg[t] : 0;
        const bool dep = und && d > 0;
        if (und && d == 0) atomicOr(&cbits[t >> 5], 1u << (t & 31));
        int tot;
        const int ex = block_excl_scan((int)dep, tmp, tot);
        if (dep) {
            dep_list[ndep + ex] = t;
            dep_idx[t] = ndep + ex;
        } else if (valid) {
            dep_idx[t] = -1;
        }
        ndep += tot;
    }
    __threadfence_block();
    __syncthreads();
    int iters = 0;
    if (threadIdx.x < 64) {
        const int lane = threadIdx.x;
        for (int c0 = 0; c0 < ndep; c0 += 64) {
            const int k = c0 + lane;
            const bool valid = k < ndep;
            const int t = valid ? dep_list[k] : 0;
            bool ext = false;
            uint64_t L = 0;
            if (valid) {
                const int e0 = off[t], e1 = e0 + deg[t];
                for (int e = e0; e < e1 && !ext; e++) {
                    const int u = edges[e];
                    const int di = dep_idx[u];
                    if (di >= c0) L |= 1ull << (di - c0);
                    else ext = (cbits[u >> 5] >> (u & 31)) & 1;
                }
            }
            const uint64_t vm = __ballot(valid);
            const uint64_t em = __ballot(valid && ext);
            uint64_t cm = vm & ~em;
            while (true) {
                const bool ci = valid && !ext && (L & cm) == 0;
                const uint64_t nm = __ballot(ci);
                iters++;
                if (nm == cm) break;
                cm = nm;
            }
            if (valid && ((cm >> lane) & 1)) atomicOr(&cbits[t >> 5], 1u << (t & 31));
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < T; t += blockDim.x) {
        const bool c = (cbits[t >> 5] >> (t & 31)) & 1;
        committed[t] = c;
        verdict[t] = c ? FDBCS_COMMITTED : (too_old[t] ? FDBCS_TOO_OLD : FDBCS_CONFLICT);
    }
    if (threadIdx.x == 0) {
        sc->n_dep = ndep;
        sc->jac_iters = iters;
    }
}

void launch_decide(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, hipStream_t s) {
    const int T = v.txn_count;
    if (T == 0) return;
    const size_t lds = (size_t)((T + 31) / 32) * 4;
    hipLaunchKernelGGL(k_decide, dim3(1), dim3(1024), lds, s, T, b.too_old, b.hist, b.deg, b.off, b.edges,
                       b.dep_list, b.dep_idx, b.committed, b.verdict, sc);
}

// ------------------------------------------------------------- combine ----
// Union of the committed writes (combineWriteConflictRanges, SkipList.cpp:
// 1320-1337).  Over writes sorted by begin key, a group starts where the begin
// is >= the running max of earlier committed ends (END sorts before BEGIN at
// equal keys, so touching ranges stay separate); the group's range is
// [first begin, max end).  Single workgroup: a 1024-wide Hillis-Steele
// running max per chunk plus a carried max.
static constexpr int COMBINE_THREADS = 512;

struct MaxKey {
    uint64_t hi, lo;
    uint32_t meta;
    uint32_t valid;
    const uint8_t* tail;
};

__device__ inline MaxKey mk_max(const MaxKey& a, const MaxKey& b) {
    if (!a.valid) return b;
    if (!b.valid) return a;
    return kcmp(a.hi, a.lo, a.meta, a.tail, b.hi, b.lo, b.meta, b.tail) >= 0 ? a : b;
}

__global__ __launch_bounds__(COMBINE_THREADS) void k_combine(int R, int W, KeyArrays keys, const SRec* __restrict__ sw,
                                                  const int32_t* __restrict__ write_txn,
                                                  const uint8_t* __restrict__ committed, KeyArrays cb, KeyArrays ce,
                                                  Scalars* sc) {
    __shared__ MaxKey buf[2][COMBINE_THREADS];
    __shared__ int32_t tmp[COMBINE_THREADS / 64 + 1];
    const int64_t wbase = 2 * (int64_t)R;
    MaxKey carry{0, 0, 0, 0, nullptr};
    int ngroups = 0;
    for (int base = 0; base < W; base += COMBINE_THREADS) {
        const int i = base + threadIdx.x;
        const bool valid = i < W;
        int w = 0;
        bool c = false;
        SRec rb{};
        if (valid) {
            rb = sw[i];
            w = (int)rb.idx;
            c = committed[write_txn[w]] != 0;
        }
        MaxKey e{0, 0, 0, 0, nullptr};
        if (c) {
            const int64_t slot = wbase + 2 * (int64_t)w + 1;
            e = MaxKey{keys.hi[slot], keys.lo[slot], keys.meta[slot], 1u, keys.tail[slot]};
        }
        int cur = 0;
        buf[cur][threadIdx.x] = e;
        __syncthreads();
        for (int d = 1; d < COMBINE_THREADS; d <<= 1) {
            MaxKey x = buf[cur][threadIdx.x];
            if (threadIdx.x >= (unsigned)d) x = mk_max(buf[cur][threadIdx.x - d], x);
            buf[cur ^ 1][threadIdx.x] = x;
            cur ^= 1;
            __syncthreads();
        }
        MaxKey excl = threadIdx.x > 0 ? buf[cur][threadIdx.x - 1] : MaxKey{0, 0, 0, 0, nullptr};
        excl = mk_max(carry, excl);
        bool gs = false;
        Key bk{};
        if (c) {
            bk = Key{rb.hi, rb.lo, rb.meta, key_len(rb.meta) > 17 ? keys.tail[wbase + 2 * (int64_t)w] : nullptr};
            gs = !excl.valid || kcmp(bk.hi, bk.lo, bk.meta, bk.tail, excl.hi, excl.lo, excl.meta, excl.tail) >= 0;
        }
        int tot;
        const int gex = block_excl_scan((int)gs, tmp, tot);
        if (gs) {
            const int g = ngroups + gex;
            cb.put(g, bk);
            if (g > 0) ce.put(g - 1, Key{excl.hi, excl.lo, excl.meta, excl.tail});
        }
        carry = mk_max(carry, buf[cur][COMBINE_THREADS - 1]);
        ngroups += tot;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        if (ngroups > 0) ce.put(ngroups - 1, Key{carry.hi, carry.lo, carry.meta, carry.tail});
        sc->n_comb = ngroups;
    }
}

void launch_combine(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, hipStream_t s) {
    hipLaunchKernelGGL(k_combine, dim3(1), dim3(COMBINE_THREADS), 0, s, v.read_count, v.write_count, b.keys, (const SRec*)b.sw,
                       b.write_txn, b.committed, b.cb, b.ce, sc);
}

}  // namespace fdbcs_dev
