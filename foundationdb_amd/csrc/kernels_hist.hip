// kernels_hist.hip -- history-side stages: write insertion and compaction.
//
// The reference mutates a skip list node by node (mergeWriteConflictRanges ->
// SkipList::addConflictRanges, SkipList.cpp:1235-1318, 511-522; removeBefore
// :665-702).  Here the history is a pool of 256-slot pages listed in key
// order by a directory.  A batch rewrites only the pages its combined writes
// touch (one workgroup per page, in LDS) and the pages of the compaction
// window, then rebuilds the (small) directory.  Net effect per combined range
// [b, e): e keeps its pre-batch value
// valueBefore(e) unless e is already a boundary or the next range's begin;
// every boundary in [b, e) is erased; b gets version `now`.
//
// Launches per batch: merge = plan_ranges, plan_aggr, plan_scan, page_merge,
// bmax_commit (+ the compaction window setup); compaction = win_keep,
// win_repack, win_dir (+ page-group maxima, search index, commit).  Directory
// `start[]` (global index of a page's first boundary) is carried forward
// incrementally, never rescanned.
#include <algorithm>
#include <cstdlib>
#include "kernels.h"
#include "devutil.h"
#include "hist_search.h"

namespace fdbcs_dev {

static constexpr int GRID_PAGES = 4096;  // workgroups for per-page kernels (grid-stride)
static constexpr int MAXP = 64;          // output parts per page tracked in LDS

// ------------------------------------------------ small single-block scan ----
template <int NA>
struct ScanArgs {
    const int32_t* in[NA];
    int32_t* out[NA];
};

// Exclusive scans of NA int32 arrays of the same device-resident length n;
// out[k][n] receives the total.  One workgroup; each 4096-element tile of all
// NA arrays is staged in LDS with coalesced loads (all in flight together),
// scanned there (4 consecutive elements per lane), and written back coalesced.
template <int NA>
__global__ __launch_bounds__(1024) void k_scan_small(ScanArgs<NA> a, const int32_t* n_ptr) {
    __shared__ int32_t tile[NA][4096];
    __shared__ int32_t tmp[1024 / 64 + 1];
    const int n = *n_ptr;
    const int tid = threadIdx.x;
    int carry[NA];
#pragma unroll
    for (int k = 0; k < NA; k++) carry[k] = 0;
    for (int base = 0; base < n; base += 4096) {
#pragma unroll
        for (int k = 0; k < NA; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int i = base + j * 1024 + tid;
                tile[k][j * 1024 + tid] = i < n ? a.in[k][i] : 0;
            }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NA; k++) {
            int v[4];
            int s = 0;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                v[j] = tile[k][tid * 4 + j];
                s += v[j];
            }
            int tot;
            int run = carry[k] + block_excl_scan(s, tmp, tot);
#pragma unroll
            for (int j = 0; j < 4; j++) {
                tile[k][tid * 4 + j] = run;
                run += v[j];
            }
            carry[k] += tot;
        }
        __syncthreads();
#pragma unroll
        for (int k = 0; k < NA; k++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const int i = base + j * 1024 + tid;
                if (i < n) a.out[k][i] = tile[k][j * 1024 + tid];
            }
        __syncthreads();
    }
    if (tid == 0)
#pragma unroll
        for (int k = 0; k < NA; k++) a.out[k][n] = carry[k];
}

// ------------------------------------------------------- insertion plan ----
// K1 k_plan_ranges, one lane per combined range j.  A combined range opens
// with the begin of one write and closes with the end of another, so where
// its b and e fall in the pre-batch history was already found by the
// speculative per-write searches (k_edges_read_check, WriteHits).  The lane
// records the range's plan -- where b and e fall, whether e needs a node and
// the value it keeps -- and its contribution to the pages it touches,
// accumulated per directory entry: erased old entries, new entries, first /
// last range touching the page, first old slot changed.  Pages strictly
// inside [pb, pe] are wholly erased; they are marked in a difference array
// (+1 at pb+1, -1 at pe) and resolved by the scan.
__device__ inline Key srec_key(const SRec& x, const uint8_t* const* tails) {
    return Key{x.hi, x.lo, x.meta, key_len(x.meta) > 17 ? tails[x.idx] : nullptr};  // (short keys: null, as encoded)
}

__global__ __launch_bounds__(256) void k_plan_ranges(const int32_t* __restrict__ cb_pos,
                                                     const int32_t* __restrict__ ce_pos, const SRec* __restrict__ sw,
                                                     const uint8_t* const* tails, WriteHits wh, int64_t wbase,
                                                     int64_t v0, ShardBounds shard, Scalars* sc, int32_t* __restrict__ pb_o,
                                                     int32_t* __restrict__ ib_o, int32_t* __restrict__ pe_o,
                                                     int32_t* __restrict__ ie_o, uint8_t* __restrict__ need_o,
                                                     int64_t* __restrict__ vb_o, PageAcc acc, KeyArrays rb,
                                                     KeyArrays re) {
    if (sc->err) return;
    const int nC = sc->n_comb;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nC) return;
    // (combined ranges are in key order: their sorted records are read nearly
    // in sequence, the keys' slots only for long keys' tails)
    const SRec xb = sw[cb_pos[j]], xe = sw[ce_pos[j]];
    const int wb = (int)(((int64_t)xb.idx - wbase) >> 1), we = (int)(((int64_t)xe.idx - wbase) >> 1);
    const Key b = srec_key(xb, tails), e = srec_key(xe, tails);
    const bool touch = j + 1 < nC && kcmp(srec_key(sw[cb_pos[j + 1]], tails), e) == 0;
    // erased boundaries are counted as real ones (r_b, r_e: real boundaries
    // before the slots i_b, i_e; c_b: real boundaries in b's page)
    const WHitB hb = wh.b[wb];
    const WHitE he = wh.e[we];
    const int p_b = hb.pb, i_b = hb.ib, c_b = hb.cb, r_b = hb.rb;
    const int p_e = he.pe, i_e = he.ie, r_e = he.re;
    const bool found = he.feq & 1;
    // valueBefore(e) fell back to the header version: the merge's v0 (sharded
    // mode: the exact carry-in, which may differ from the one the search saw)
    const int64_t vb = (he.feq & 2) ? (sc->carry_dev ? sc->carry_apply : v0) : he.vb;
    // sharded mode (protocol A step 5): a range acts on this shard iff b < hi
    // and e >= lo; its begin node only if b >= lo, its end node only if e < hi
    // (the positions of keys outside the shard clamp to the shard's ends)
    if (shard.at_or_above(b) || shard.below(e)) return;
    const int has_b = shard.below(b) ? 0 : 1;
    const bool e_in = !shard.at_or_above(e);
    if (shard.has_lo | shard.has_hi) {  // (the global compaction budget sums these over shards)
        const uint64_t m = __ballot(has_b);  // one atomic per wavefront
        if (has_b && (int)__lane_id() == __ffsll((unsigned long long)m) - 1) atomicAdd(&sc->n_comb_own, __popcll(m));
    }
    rb.put(j, b);  // compact copies for the page merge
    re.put(j, e);
    const int need = (e_in && !found && !touch) ? 1 : 0;
    pb_o[j] = p_b;
    ib_o[j] = i_b;
    pe_o[j] = p_e;
    ie_o[j] = i_e;
    need_o[j] = (uint8_t)(need | has_b << 1);
    vb_o[j] = vb;
    if (p_b == p_e) {
        if (r_e > r_b) atomicAdd(&acc.er[p_b], r_e - r_b);
        atomicAdd(&acc.nn[p_b], has_b + need);
        atomicMin(&acc.jlo[p_b], j);
        atomicMax(&acc.jhi[p_b], j);
    } else {
        if (c_b > r_b) atomicAdd(&acc.er[p_b], c_b - r_b);
        atomicAdd(&acc.nn[p_b], has_b);
        atomicMin(&acc.jlo[p_b], j);
        atomicMax(&acc.jhi[p_b], j);
        if (r_e) atomicAdd(&acc.er[p_e], r_e);
        if (need) atomicAdd(&acc.nn[p_e], 1);
        atomicMin(&acc.jlo[p_e], j);
        atomicMax(&acc.jhi[p_e], j);
        if (p_e > p_b + 1) {
            atomicAdd(&acc.diff[p_b + 1], 1);
            atomicAdd(&acc.diff[p_e], -1);
        }
    }
}

// K2: the directory after the merge.  Per directory entry x: affected?
// (touched by a range, or wholly inside one), boundaries out, output pages
// (parts), pages taken from / returned to the free stack, boundary delta, new
// entries.  Exclusive scans over x give every entry its new directory
// position, start[] shift and free-stack slots.  Two launches: K2a reduces
// each 1024-entry block for both possible "inside a wide range" states at the
// block start (the state is the prefix of the difference array, 0 or 1, as
// combined ranges are disjoint); K2b resolves every block's prefix from its
// predecessors' aggregates, scans, writes the unaffected directory entries
// at their new positions and the affected pages' merge plan, and resets the
// accumulators for the next batch.
static constexpr int PS_THREADS = 256;
#ifndef FDBCS_PS_ITEMS
#define FDBCS_PS_ITEMS 2
#endif
static constexpr int PS_ITEMS = FDBCS_PS_ITEMS;
static constexpr int PS_BLOCK = PS_THREADS * PS_ITEMS;

struct PlanItem {
    bool affected;
    int32_t nout, parts, nn, jlo, jhi;
};

// An entry's accumulators and real boundary count (Dir::nr), loaded
// together before the plan kernels' scans (not behind their barriers).
struct PlanIn {
    int cnt, jlo, jhi, nn, er;
};
__device__ inline PlanIn plan_load(const PageAcc& acc, const int32_t* nr, int x) {
    return PlanIn{nr[x], acc.jlo[x], acc.jhi[x], acc.nn[x], acc.er[x]};
}

__device__ inline PlanItem plan_item(const PlanIn& in, int x, bool covered) {
    PlanItem it;
    const int cnt = in.cnt;
    it.jlo = in.jlo;
    it.jhi = in.jhi;
    it.nn = 0;
    if (covered) {
        it.affected = true;
        it.nout = 0;
    } else if (it.jhi >= 0) {
        it.affected = true;
        it.nn = in.nn;
        it.nout = cnt - in.er + it.nn;
    } else {
        it.affected = false;
        it.nout = cnt;
    }
    // an emptied entry 0 stays (as an empty page): the directory never has
    // zero entries (a shard's whole history can be erased in sharded mode).
    // Pages split early (SPLIT < PAGE) so that they keep holes.
    it.parts = !it.affected ? 1 : (it.nout == 0 ? (x == 0 ? 1 : 0) : (it.nout <= SPLIT ? 1 : cdiv(it.nout, FILL)));
    return it;
}

// packed scan words: (parts << 32 | affected), (freed << 32 | extra), (delta << 32 | nn)
// An affected page keeps its pool page for its first part; further parts come
// from the free stack ("extra"); a page that disappears goes back ("freed").
__device__ inline void pack_item(const PlanItem& it, int cnt, int64_t w[3]) {
    const int64_t extra = it.affected && it.parts > 1 ? it.parts - 1 : 0;
    const int64_t freed = it.affected && it.parts == 0;
    w[0] = ((int64_t)it.parts << 32) | (int64_t)it.affected;
    w[1] = (freed << 32) | extra;
    w[2] = (int64_t)((uint64_t)(uint32_t)(it.nout - cnt) << 32) | (int64_t)it.nn;
}

template <int N>
__device__ inline void block_reduce_n(int64_t (&v)[N], int64_t (*red)[N]) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
    for (int k = 0; k < N; k++) v[k] = wave_reduce_sum(v[k]);
    if (lane == 0)
#pragma unroll
        for (int k = 0; k < N; k++) red[wid][k] = v[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < N; k++) {
        int64_t t = 0;
        for (int w = 0; w < nw; w++) t += red[w][k];
        v[k] = t;
    }
    __syncthreads();
}

__global__ __launch_bounds__(PS_THREADS) void k_plan_aggr(Dir dir, const Scalars* sc, PageAcc acc,
                                                          int64_t* __restrict__ blk_agg,
                                                          int32_t* __restrict__ blk_diff) {
    __shared__ int32_t red32[PS_THREADS / 64 + 1];
    __shared__ int64_t red[PS_THREADS / 64][7];
    const int D = sc->D;
    const int base = blockIdx.x * PS_BLOCK;
    if (base >= D) return;
    const int x0 = base + threadIdx.x * PS_ITEMS;
    int dl[PS_ITEMS], dsum = 0;
    PlanIn in[PS_ITEMS];
#pragma unroll
    for (int k = 0; k < PS_ITEMS; k++) {
        dl[k] = x0 + k < D ? acc.diff[x0 + k] : 0;
        in[k] = x0 + k < D ? plan_load(acc, dir.nr, x0 + k) : PlanIn{0, 0, -1, 0, 0};
        dsum += dl[k];
    }
    int dtot;
    int cov = block_excl_scan(dsum, red32, dtot);  // local prefix, excluding this thread's items
    int64_t v[7] = {0, 0, 0, 0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < PS_ITEMS; k++) {
        cov += dl[k];
        const int x = x0 + k;
        if (x < D) {
            const int cnt = in[k].cnt;
#pragma unroll
            for (int s = 0; s < 2; s++) {  // s = state at the block start
                const PlanItem it = plan_item(in[k], x, s + cov > 0);
                int64_t w[3];
                pack_item(it, cnt, w);
                v[3 * s + 0] += w[0];
                v[3 * s + 1] += w[1];
                v[3 * s + 2] += w[2];
            }
        }
    }
    block_reduce_n<7>(v, red);
    if (threadIdx.x == 0) {
#pragma unroll
        for (int k = 0; k < 6; k++) blk_agg[(int64_t)blockIdx.x * 6 + k] = v[k];
        blk_diff[blockIdx.x] = dtot;
    }
}

struct PlanArgs {
    Dir src, dst;
    Scalars* sc;
    PageAcc acc;
    const int64_t* blk_agg;
    const int32_t* blk_diff;
    int32_t *aff_list, *aff_jlo, *aff_jhi, *aff_nn, *aff_parts, *aff_nn_off, *aff_parts_off, *aff_extra_off,
        *aff_free_off, *aff_page, *aff_cnt;
    int64_t* aff_start;
};

__global__ __launch_bounds__(PS_THREADS) void k_plan_scan(PlanArgs A) {
    __shared__ int32_t red32[PS_THREADS / 64 + 1];
    __shared__ int64_t red64[PS_THREADS / 64 + 1];
    __shared__ int64_t s_pre[4];  // block prefix: 3 packed words + start state
    Scalars* sc = A.sc;
    const int D = sc->D;
    const int base = blockIdx.x * PS_BLOCK;
    if (base >= D) return;
    const int lane = threadIdx.x & 63;
    // this thread's entries: accumulators and directory fields, loaded before
    // the prefix and the scans (their barriers would hold these loads back)
    const int x0 = base + threadIdx.x * PS_ITEMS;
    int dl[PS_ITEMS];
    PlanIn in[PS_ITEMS];
    int64_t e_start[PS_ITEMS], e_maxv[PS_ITEMS];
    int e_page[PS_ITEMS], e_cnt[PS_ITEMS];
    uint64_t e_fhi[PS_ITEMS], e_flo[PS_ITEMS];
    uint32_t e_fmeta[PS_ITEMS];
    const uint8_t* e_ftail[PS_ITEMS];
#pragma unroll
    for (int k = 0; k < PS_ITEMS; k++) {
        const int x = x0 + k;
        const bool ok = x < D;
        dl[k] = ok ? A.acc.diff[x] : 0;
        in[k] = ok ? plan_load(A.acc, A.src.nr, x) : PlanIn{0, 0, -1, 0, 0};
        e_start[k] = ok ? A.src.start[x] : 0;
        e_page[k] = ok ? A.src.page[x] : 0;
        e_cnt[k] = ok ? A.src.cnt[x] : 0;
        e_maxv[k] = ok ? A.src.maxv[x] : 0;
        e_fhi[k] = ok ? A.src.fhi[x] : 0;
        e_flo[k] = ok ? A.src.flo[x] : 0;
        e_fmeta[k] = ok ? A.src.fmeta[x] : 0;
        e_ftail[k] = ok ? A.src.ftail[x] : nullptr;
    }
    // ---- this block's prefix from its predecessors (wave 0) ----
    if (threadIdx.x < 64) {
        int64_t p0 = 0, p1 = 0, p2 = 0;
        int carry = 0;
        // 256 predecessors a round: their differences and both halves of
        // their aggregates (either start state) loaded together, the state
        // chosen after the scan -- one round trip where loading each
        // aggregate behind its state took two per 64 predecessors
        const int nb = (int)blockIdx.x;
        for (int k0 = 0; k0 < nb; k0 += 256) {
            int d[4];
            int64_t a[4][6];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int k = k0 + 64 * u + lane;
                const bool ok = k < nb;
                d[u] = ok ? A.blk_diff[k] : 0;
#pragma unroll
                for (int j = 0; j < 6; j++) a[u][j] = ok ? A.blk_agg[(int64_t)k * 6 + j] : 0;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int st = carry + wave_incl_scan(d[u]) - d[u];  // state at block k's start
                p0 += st > 0 ? a[u][3] : a[u][0];
                p1 += st > 0 ? a[u][4] : a[u][1];
                p2 += st > 0 ? a[u][5] : a[u][2];
                carry += wave_reduce_sum(d[u]);
            }
        }
        p0 = wave_reduce_sum(p0);
        p1 = wave_reduce_sum(p1);
        p2 = wave_reduce_sum(p2);
        if (lane == 0) {
            s_pre[0] = p0;
            s_pre[1] = p1;
            s_pre[2] = p2;
            s_pre[3] = carry;
        }
    }
    __syncthreads();
    int dsum = 0;
#pragma unroll
    for (int k = 0; k < PS_ITEMS; k++) dsum += dl[k];
    int dtot;
    int cov = (int)s_pre[3] + block_excl_scan(dsum, red32, dtot);
    PlanItem it[PS_ITEMS];
    int cnt[PS_ITEMS];
    int64_t w[PS_ITEMS][3], tsum[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < PS_ITEMS; k++) {
        cov += dl[k];
        const int x = x0 + k;
        cnt[k] = 0;
        it[k] = PlanItem{false, 0, 0, 0, 0, -1};
        w[k][0] = w[k][1] = w[k][2] = 0;
        if (x < D) {
            cnt[k] = in[k].cnt;
            it[k] = plan_item(in[k], x, cov > 0);
            pack_item(it[k], cnt[k], w[k]);
        }
        tsum[0] += w[k][0];
        tsum[1] += w[k][1];
        tsum[2] += w[k][2];
    }
    int64_t tot[3], ex[3];
#pragma unroll
    for (int f = 0; f < 3; f++) ex[f] = s_pre[f] + block_excl_scan(tsum[f], red64, tot[f]);
    const int64_t top0 = sc->free_top;
#pragma unroll
    for (int k = 0; k < PS_ITEMS; k++) {
        const int x = x0 + k;
        if (x < D) {
            const int pos = (int)(ex[0] >> 32);
            const int64_t st = e_start[k] + (int64_t)(int32_t)(uint32_t)((uint64_t)ex[2] >> 32);
            if (it[k].affected) {
                const int a = (int)(uint32_t)ex[0];
                A.aff_list[a] = x;
                A.aff_page[a] = e_page[k];
                A.aff_cnt[a] = e_cnt[k];  // slots in use
                A.aff_jlo[a] = it[k].jlo;
                A.aff_jhi[a] = it[k].jhi;
                A.aff_nn[a] = it[k].nn;
                A.aff_parts[a] = it[k].parts;
                A.aff_nn_off[a] = (int)(uint32_t)ex[2];
                A.aff_parts_off[a] = pos;
                A.aff_extra_off[a] = (int)(uint32_t)ex[1];
                A.aff_free_off[a] = (int)(ex[1] >> 32);
                A.aff_start[a] = st;
            } else {
                A.dst.page[pos] = e_page[k];
                A.dst.cnt[pos] = e_cnt[k];
                A.dst.nr[pos] = cnt[k];
                A.dst.maxv[pos] = e_maxv[k];
                A.dst.fhi[pos] = e_fhi[k];
                A.dst.flo[pos] = e_flo[k];
                A.dst.fmeta[pos] = e_fmeta[k];
                A.dst.ftail[pos] = e_ftail[k];
                A.dst.start[pos] = st;
            }
            // reset the accumulators for the next batch
            A.acc.er[x] = 0;
            A.acc.nn[x] = 0;
            A.acc.jlo[x] = INT32_MAX;
            A.acc.jhi[x] = -1;
            A.acc.diff[x] = 0;
#pragma unroll
            for (int f = 0; f < 3; f++) ex[f] += w[k][f];
        }
    }
    if (blockIdx.x == (D - 1) / PS_BLOCK && threadIdx.x == 0) {
        // totals: the last block's inclusive sums
        const int64_t t0 = s_pre[0] + tot[0], t1 = s_pre[1] + tot[1], t2 = s_pre[2] + tot[2];
        const int Dn = (int)(t0 >> 32);
        const int extra = (int)(uint32_t)t1, freed = (int)(t1 >> 32);
        sc->n_aff = (int)(uint32_t)t0;
        sc->n_full = 0;
        sc->D_next = Dn;
        sc->extra_total = extra;
        sc->free_next = (int)(top0 - extra + freed);
        sc->free_base = (int)(top0 - extra);
        A.dst.start[Dn] = A.src.start[D] + (int64_t)(int32_t)(uint32_t)((uint64_t)t2 >> 32);
    }
}

__device__ inline void copy_tail(const Key& k, uint8_t* arena, uint64_t cap, Scalars* sc, const uint8_t** out) {
    const uint32_t L = key_len(k.meta);
    if (L <= 17) {
        *out = nullptr;
        return;
    }
    const uint64_t half = tail_half_bytes(cap);
    const uint64_t padded = ((uint64_t)(L - 17) + 7) & ~7ull;
    const uint64_t o = atomicAdd((unsigned long long*)&sc->tail_used, (unsigned long long)padded);
    if (o + padded > half) {
        atomicCAS(&sc->err, 0, FDBCS_E_CAPACITY);
        *out = nullptr;
        return;
    }
    const uint64_t* src = reinterpret_cast<const uint64_t*>(k.tail);
    uint64_t* dst = reinterpret_cast<uint64_t*>(arena + (sc->tail_half ? half : 0) + o);
    for (uint64_t w = 0; w < padded / 8; w++) dst[w] = src[w];
    *out = reinterpret_cast<const uint8_t*>(dst);
}

// The compaction window's survivors move their tails out of the half being
// freed (tail arena GC).  The moves fill the new half to at most its middle
// (the merges' room is kept by ensure_history); past that, or with nothing to
// move, the old pointer stays and this sweep frees nothing (TF_NOGC).
__device__ inline const uint8_t* move_tail(const uint8_t* tail, uint32_t meta, uint8_t* arena, uint64_t cap,
                                           Scalars* sc) {
    const uint32_t L = key_len(meta);
    if (L <= 17 || !tail) return tail;
    const uint64_t half = tail_half_bytes(cap);
    const uint8_t* from = arena + (sc->tail_half ? 0 : half);
    if (tail < from || tail >= from + half) return tail;
    const uint64_t padded = ((uint64_t)(L - 17) + 7) & ~7ull;
    const uint64_t o = atomicAdd((unsigned long long*)&sc->tail_used, (unsigned long long)padded);
    if (o + padded > half / 2) {
        atomicAdd((unsigned long long*)&sc->tail_used, (unsigned long long)(0ull - padded));
        atomicOr(&sc->tail_flags, TF_NOGC);
        return tail;
    }
    uint64_t* dst = reinterpret_cast<uint64_t*>(arena + (sc->tail_half ? half : 0) + o);
    const uint64_t* src = reinterpret_cast<const uint64_t*>(tail);
    for (uint64_t w = 0; w < padded / 8; w++) dst[w] = src[w];
    return reinterpret_cast<const uint8_t*>(dst);
}

struct DescArrays {
    int32_t* page;
    int32_t* cnt;  // slots in use
    int32_t* nr;   // boundaries
    int64_t* maxv;
    uint64_t* fhi;
    uint64_t* flo;
    uint32_t* fmeta;
    const uint8_t** ftail;
};

struct MergeArgs {
    Pool pool;
    Dir dir;   // pre-batch directory
    Dir dst;   // directory being built (affected pages' parts are written here)
    Scalars* sc;
    const int32_t* free_stack;
    int32_t* freed_list;
    int32_t* full_list;  // pages the in-place pass left to the rewrite
    const int32_t* aff_list;
    const int32_t *aff_page, *aff_cnt;
    const int32_t *jlo, *jhi, *nn, *nn_off, *parts, *parts_off, *extra_off, *free_off;
    const int64_t* aff_start;
    const int32_t *pb, *ib, *pe, *ie;
    const uint8_t* need_e;
    const int64_t* vb;
    KeyArrays rb, re;  // keys of each combined range's begin / end (compact, from K1)
    Pool ne;
    int32_t* ne_ins;
    uint8_t* arena;
    uint64_t arena_cap;
    int64_t now;
    int px;  // HistBufs::px_host: pages may hold prefix skips (else none was ever set)
};

__device__ inline void put_entry(const Pool& pool, int64_t d, uint64_t hi, uint64_t lo, uint32_t meta, int64_t ver,
                                 const uint8_t* tail) {
    pool.hi[d] = hi; pool.lo[d] = lo; pool.meta[d] = meta; pool.ver[d] = ver; pool.tail[d] = tail;
    if ((d & (PIDX_STRIDE - 1)) == 0) pool.pidx[d / PIDX_STRIDE] = hi;
}
// a slot's 8 bytes past its page's prefix skip (common.h Pool::px)
__device__ inline void put_px(const Pool& pool, int64_t d, uint64_t px) {
    pool.px[d] = px;
    if ((d & (PIDX_STRIDE - 1)) == 0) pool.pxidx[d / PIDX_STRIDE] = px;
}

__device__ inline void put_desc(const DescArrays& D, int x, int page, int n, uint64_t hi, uint64_t lo,
                                uint32_t meta, const uint8_t* tail) {
    D.page[x] = page; D.cnt[x] = spread_used(n); D.nr[x] = n;
    D.fhi[x] = hi; D.flo[x] = lo; D.fmeta[x] = meta; D.ftail[x] = tail;
}

// K3: one wavefront per affected page (four pages per workgroup, no
// workgroup barriers), four consecutive old slots per lane.
//   1. plan lanes (one per combined range touching the page) mark the slots
//      their range erases (+1 / -1 in a difference array) and count the new
//      boundaries inserted before each old slot (b_j at ib_j, e_j at ie_j).
//   2a. In place (the usual case: the page stays one page and nothing in it
//      is erased): new boundaries are pushed right into the next hole
//      (common.h "holes").  A carry of pending entries runs over the slots:
//      it grows by the insertions at a slot and a hole with carry > 0 absorbs
//      one, so the carry arriving at slot i is a saturating prefix
//      c(i) = max(c(i-1) + a(i-1) - h(i-1), 0), scanned across the wavefront
//      as a composition of x -> max(x + d, L).  Old boundary i moves to
//      i + c(i) + a(i) (most do not move); the new entries at slot i land at
//      i + c(i) + t.  Free slots past the used ones count as holes.  Only
//      moved slots are read and written.
//   2b. Otherwise (erasures, a split, no room to the right): the page is
//      rewritten.  An old slot survives if no range covers it and it is not a
//      hole; survivors and new entries are numbered in key order and spread
//      over the output parts with fresh holes (spread_slot).
// Output pages: the first in place (every old slot is loaded before any
// write), the others from the free stack; a page that disappears goes back on
// it (k_bmax_commit pushes it after every pop).  Directory entries go to the
// positions K2 assigned.
static constexpr int MW_WAVES = 4;  // pages in flight per workgroup

struct WaveMerge {
    int32_t er[PAGE + 1];   // erase marks (difference array), then kept-before per slot; in place: carry
    int32_t ins[PAGE + 1];  // new boundaries inserted before each old slot; in place: their exclusive prefix
    long long pmax[MAXP];
    // first key of each output part (its directory entry), written by whichever lane lands it
    uint64_t f_hi[MAXP], f_lo[MAXP];
    const uint8_t* f_tail[MAXP];
    uint32_t f_meta[MAXP];
    int32_t f_dp[MAXP];
    unsigned long long hm[HM_WORDS];  // in place: the page's hole mask as holes are consumed
};

// Lanes of one wavefront exchanging data through LDS: LDS operations of a
// wavefront complete in order, so waiting for this wavefront's LDS traffic
// suffices (no wait on its outstanding global loads, unlike a fence).
__device__ inline void wave_lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// every global load of this wavefront has returned (the page is read before
// it is written in place: all lanes' loads precede all lanes' stores)
__device__ inline void wave_loads_done() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

__device__ inline int lane_read(int v, int k) { return __builtin_amdgcn_readlane(v, k); }

// A page's hole mask in four named words: a dynamically indexed private
// array lives in scratch memory (k_page_merge stored and reloaded its mask
// there for every slot test)
struct HoleMask {
    uint64_t w0, w1, w2, w3;
    // (masks, not selects: a select chain over the four words is turned back
    // into an indexed private array)
    __device__ uint64_t word(int w) const {
        return (w0 & (0ull - (uint64_t)(w == 0))) | (w1 & (0ull - (uint64_t)(w == 1))) |
               (w2 & (0ull - (uint64_t)(w == 2))) | (w3 & (0ull - (uint64_t)(w == 3)));
    }
    __device__ bool bit(int i) const { return (word(i >> 6) >> (i & 63)) & 1; }
    __device__ int popc() const { return __popcll(w0) + __popcll(w1) + __popcll(w2) + __popcll(w3); }
};
static_assert(HM_WORDS == 4, "hole mask words");
__device__ inline HoleMask load_hole_mask_uniform(const Pool& p, int page) {
    uint64_t hm[HM_WORDS];
    load_hmask_uniform(p, page, hm);
    return HoleMask{hm[0], hm[1], hm[2], hm[3]};
}

// A part's first entry: its directory entry is stashed in LDS (written after
// the merge by one lane per part); parts beyond MAXP write it directly.
__device__ inline void part_dir(const Dir& D, const MergeArgs& A, int a, int y, int q, int per, int nout, int dp,
                                uint64_t h, uint64_t l, uint32_t mt, const uint8_t* tl) {
    const int n = min(per, nout - q * per);
    D.page[y] = dp; D.cnt[y] = spread_used(n); D.nr[y] = n;
    D.fhi[y] = h; D.flo[y] = l; D.fmeta[y] = mt; D.ftail[y] = tl;
    D.start[y] = A.aff_start[a] + (int64_t)q * per;
}

__device__ inline void part_first(WaveMerge& S, const Dir& D, const MergeArgs& A, int a, int doff, int q, int per,
                                  int nout, int dp, uint64_t h, uint64_t l, uint32_t mt, const uint8_t* tl) {
    if (q < MAXP) {
        S.f_hi[q] = h; S.f_lo[q] = l; S.f_meta[q] = mt; S.f_tail[q] = tl; S.f_dp[q] = dp;
    } else {
        part_dir(D, A, a, doff + q, q, per, nout, dp, h, l, mt, tl);
    }
}

// Plan of combined range j as one lane holds it.
struct RangePlan {
    int pb, ib, pe, ie;
    bool need;   // a node at e
    bool has_b;  // a node at b (not so for a range clipped at the shard's start)
    int64_t vb;  // (the keys are loaded where they are written: fewer live registers)
};

__device__ inline RangePlan load_plan(const MergeArgs& A, int j) {
    RangePlan r;
    r.pb = A.pb[j]; r.ib = A.ib[j]; r.pe = A.pe[j]; r.ie = A.ie[j];
    const uint8_t fl = A.need_e[j];
    r.need = fl & 1;
    r.has_b = (fl >> 1) & 1;
    r.vb = A.vb[j];
    return r;
}

// x -> max(x + d, L) packed as (d, L) in one 64-bit lane value; compose(x, e)
// applies e (an earlier stretch of slots) first, then x
__device__ inline uint64_t sat_pack(int d, int L) { return (uint64_t)(uint32_t)d | ((uint64_t)(uint32_t)L << 32); }
__device__ inline int sat_d(uint64_t f) { return (int)(uint32_t)f; }
__device__ inline int sat_L(uint64_t f) { return (int)(uint32_t)(f >> 32); }
constexpr int SAT_NONE = -(1 << 28);

// 2a.  Returns false (nothing written) if the new entries do not fit to the
// right of their insertion points; S.er / S.ins then still hold step 1's marks.
template <bool PX>
__device__ __forceinline__ bool merge_in_place(const MergeArgs& A, WaveMerge& S, int a, int p, int pg, int C, const HoleMask& hm,
                               int jlo, int jhi, const RangePlan& r0, bool has0, int doff, int nn) {
    const int lane = threadIdx.x & 63;
    const int i0 = 4 * lane;
    const int64_t pbase = (int64_t)pg * PAGE;
    const int64_t omax = A.dir.maxv[p];  // no boundary is erased: the maximum only grows
    int av[4], hv[4];
    uint64_t f = sat_pack(0, SAT_NONE);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = i0 + q;
        av[q] = S.ins[i];
        hv[q] = i >= C || hm.bit(i);  // (free slots past the used ones absorb like holes)
        const int d = av[q] - hv[q];
        f = sat_pack(sat_d(f) + d, max(sat_L(f) + d, 0));
    }
    const uint64_t incl = wave_incl_scan_op(f, sat_pack(0, SAT_NONE), [](uint64_t x, uint64_t e) {
        return sat_pack(sat_d(e) + sat_d(x), max(sat_L(e) + sat_d(x), sat_L(x)));
    });
    const uint64_t ex = __shfl_up(incl, 1);
    const uint64_t ex_fix = lane == 0 ? sat_pack(0, SAT_NONE) : ex;  // (lane 0: nothing before it)
    int c = max(sat_d(ex_fix), sat_L(ex_fix));  // carry arriving at slot i0 (none before slot 0)
    int cb[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        cb[q] = c;
        c = max(c + av[q] - hv[q], 0);
    }
    const int last = lane_read(c, 63);
    if (last != 0 || S.ins[PAGE] != 0) return false;  // some entries would run past the page
    // ---- positions
    const int isum = av[0] + av[1] + av[2] + av[3];
    int irun = wave_incl_scan(isum) - isum;
    uint32_t movem = 0, usem = 0;
    int maxout = -1;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = i0 + q;
        S.ins[i] = irun;  // new entries inserted before slot i
        S.er[i] = cb[q];  // carry arriving at slot i
        irun += av[q];
        if (i < C && !hv[q] && cb[q] + av[q] > 0) movem |= 1u << q;  // old boundary i moves
        if (i < C && hv[q] && cb[q] > 0) usem |= 1u << q;            // hole i absorbs one
        if ((movem >> q) & 1) maxout = max(maxout, i + cb[q] + av[q]);
    }
    if (lane == 0) {
        S.hm[0] = hm.w0; S.hm[1] = hm.w1; S.hm[2] = hm.w2; S.hm[3] = hm.w3;
    }
    wave_lds_sync();
    // ---- read the boundaries that move, then write them
    uint64_t ohi[4], olo[4];
    uint32_t ometa[4];
    int64_t over[4];
    const uint8_t* otail[4];
    // (<= 0: no prefix words to keep; PX false -- no long key yet -- compiles the
    // prefix-word moves out, so the plain path carries none of their registers)
    const int pskip = FDBCS_DIR_PX && PX ? A.pool.pskip[pg] : 0;
#pragma unroll
    for (int q = 0; q < 4; q++) {
        if (!((movem >> q) & 1)) continue;
        const int64_t sl = pbase + i0 + q;
        ohi[q] = A.pool.hi[sl]; olo[q] = A.pool.lo[sl]; ometa[q] = A.pool.meta[sl];
        over[q] = A.pool.ver[sl]; otail[q] = A.pool.tail[sl];
    }
    wave_loads_done();
    if (pskip > 0) {  // the moving slots' prefix words, in a pass of their own (fewer live registers)
        uint64_t opx[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            if ((movem >> q) & 1) opx[q] = A.pool.px[pbase + i0 + q];
        wave_loads_done();
#pragma unroll
        for (int q = 0; q < 4; q++)
            if ((movem >> q) & 1) put_px(A.pool, pbase + i0 + q + cb[q] + av[q], opx[q]);
    }
#pragma unroll
    for (int q = 0; q < 4; q++) {
        const int i = i0 + q;
        if ((movem >> q) & 1)
            put_entry(A.pool, pbase + i + cb[q] + av[q], ohi[q], olo[q], ometa[q], over[q], otail[q]);
        if ((usem >> q) & 1) atomicAnd(&S.hm[i >> 6], ~(1ull << (i & 63)));
    }
    // ---- the new entries, by the plan lanes: b_j (version now), then e_j
    int64_t vmax = omax;
    int base = 0;
    for (int j0 = jlo; j0 <= jhi; j0 += 64) {
        const int j = j0 + lane;
        const bool v = j <= jhi;
        RangePlan r{};
        if (v) r = j0 == jlo ? r0 : load_plan(A, j);
        const bool eb = v && r.pb == p && r.has_b;
        const bool ee = v && r.pe == p && r.need;
        const int cnt = (int)eb + (int)ee;
        const int inc = wave_incl_scan(cnt);
        int k = base + inc - cnt;  // new entries of this page before this lane's
#pragma unroll
        for (int w = 0; w < 2; w++) {
            if (!(w == 0 ? eb : ee)) continue;
            const Key kk = w == 0 ? A.rb.get(j) : A.re.get(j);
            const int at = w == 0 ? r.ib : r.ie;
            const int64_t ver = w == 0 ? A.now : r.vb;
            const int out = at + S.er[at] + (k - S.ins[at]);
            const uint8_t* tl;
            copy_tail(kk, A.arena, A.arena_cap, A.sc, &tl);
            put_entry(A.pool, pbase + out, kk.hi, kk.lo, kk.meta, ver, tl);
            if (pskip > 0) put_px(A.pool, pbase + out, key_bytes_at(kk, pskip));
            vmax = max(vmax, ver);
            maxout = max(maxout, out);
            if (out == 0) part_first(S, A.dst, A, a, doff, 0, 1, 1, pg, kk.hi, kk.lo, kk.meta, tl);
            k++;
        }
        base += lane_read(inc, 63);
    }
    vmax = wave_reduce_max(vmax);
    maxout = wave_reduce_max(maxout);
    wave_lds_sync();
    // ---- directory entry and hole mask
    const Dir& D = A.dst;
    if (lane < HM_WORDS) A.pool.hmask[(int64_t)pg * HM_WORDS + lane] = S.hm[lane];
    if (lane == 0) {
        const int holes = hm.popc();
        D.page[doff] = pg;
        D.cnt[doff] = max(C, maxout + 1);
        D.nr[doff] = C - holes + nn;
        D.maxv[doff] = vmax;
        D.start[doff] = A.aff_start[a];
        if (S.ins[1] == 0) {  // nothing inserted before slot 0: the pre-batch first key
            const Key first = dir_first(A.dir, p);
            D.fhi[doff] = first.hi; D.flo[doff] = first.lo; D.fmeta[doff] = first.meta; D.ftail[doff] = first.tail;
        } else {
            D.fhi[doff] = S.f_hi[0]; D.flo[doff] = S.f_lo[0]; D.fmeta[doff] = S.f_meta[0]; D.ftail[doff] = S.f_tail[0];
        }
    }
    return true;
}

// INPLACE: the first pass over every affected page (k_page_merge); pages it
// cannot do in place go on a list for the second (k_page_merge_full), which
// rewrites them -- two kernels, so the short in-place path is compiled apart
// from the register-heavy rewrite.  UNIFIED (FDBCS_PM_UNIFIED builds): a page
// the in-place pass cannot do is rewritten by the same wavefront at once (one
// launch; both paths fit 3 waves per SIMD).
#ifndef FDBCS_PM_REWRITE_AT  // (A/B: pages receiving this many new boundaries are rewritten, not shifted in place)
#define FDBCS_PM_REWRITE_AT (PAGE + 1)
#endif
template <bool INPLACE, bool UNIFIED = false, bool PX = true>
__device__ void merge_page_wave(const MergeArgs& A, WaveMerge& S, int a, int top0) {
    Scalars* sc = A.sc;
    const int lane = threadIdx.x & 63;
    const int p = A.aff_list[a];
    const int parts = A.parts[a];
    const int pg = A.aff_page[a], cntp = A.aff_cnt[a];  // cntp: slots in use
    if (INPLACE && parts == 0) {  // wholly erased: returns to the free stack in k_bmax_commit (after every pop)
        if (lane == 0) A.freed_list[A.free_off[a]] = pg;
        return;
    }
    const int jlo = A.jlo[a], jhi = A.jhi[a];
    const int nn = A.nn[a];
    const int xoff = A.extra_off[a], doff = A.parts_off[a];
    const int64_t pbase = (int64_t)pg * PAGE;
    const int i0 = 4 * lane;
    // ---- 0. the hole mask and the first 64 ranges' plans
    const HoleMask hm = load_hole_mask_uniform(A.pool, pg);
    const bool has0 = jlo + lane <= jhi;
    RangePlan r0{};
    if (has0) r0 = load_plan(A, jlo + lane);
#pragma unroll
    for (int q = 0; q < 4; q++) {
        S.er[i0 + q] = 0;
        S.ins[i0 + q] = 0;
    }
    if (lane == 0) {
        S.er[PAGE] = 0;
        S.ins[PAGE] = 0;
    }
    S.pmax[lane] = INT64_MIN;
    wave_lds_sync();
    // ---- 1. plan lanes: erased intervals and insertion counts
    bool erases = false;
    for (int j0 = jlo; j0 <= jhi; j0 += 64) {
        const int j = j0 + lane;
        if (j <= jhi) {
            const RangePlan r = j0 == jlo ? r0 : load_plan(A, j);
            const int s0 = r.pb < p ? 0 : r.ib, e0 = r.pe > p ? cntp : r.ie;
            if (e0 > s0) {
                atomicAdd(&S.er[s0], 1);
                atomicAdd(&S.er[e0], -1);
                erases = true;
            }
            if (r.pb == p && r.has_b) atomicAdd(&S.ins[r.ib], 1);
            if (r.pe == p && r.need) atomicAdd(&S.ins[r.ie], 1);
        }
    }
    wave_lds_sync();
    if (INPLACE) {
        if (parts == 1 && !__ballot(erases) && nn < FDBCS_PM_REWRITE_AT &&
            merge_in_place<PX>(A, S, a, p, pg, cntp, hm, jlo, jhi, r0, has0, doff, nn))
            return;
        if (!UNIFIED) {
            if (lane == 0) A.full_list[atomicAdd(&sc->n_full, 1)] = a;
            return;
        }
    }
    // ---- 2b. rewrite: every old slot, loaded before any write
    uint64_t ohi[4] = {}, olo[4] = {};
    int64_t over[4] = {};
    uint32_t ometa[4] = {};
    const uint8_t* otail[4] = {};
    if (i0 < cntp) {
        const longlong2* v2 = reinterpret_cast<const longlong2*>(A.pool.ver + pbase + i0);
        const ulonglong2* h2 = reinterpret_cast<const ulonglong2*>(A.pool.hi + pbase + i0);
        const ulonglong2* l2 = reinterpret_cast<const ulonglong2*>(A.pool.lo + pbase + i0);
        const ulonglong2* t2 = reinterpret_cast<const ulonglong2*>(A.pool.tail + pbase + i0);
        const uint4 m4 = *reinterpret_cast<const uint4*>(A.pool.meta + pbase + i0);
        const longlong2 va = v2[0], vb = v2[1];
        const ulonglong2 ha = h2[0], hb = h2[1], la = l2[0], lb = l2[1], ta = t2[0], tb = t2[1];
        over[0] = va.x; over[1] = va.y; over[2] = vb.x; over[3] = vb.y;
        ohi[0] = ha.x; ohi[1] = ha.y; ohi[2] = hb.x; ohi[3] = hb.y;
        olo[0] = la.x; olo[1] = la.y; olo[2] = lb.x; olo[3] = lb.y;
        ometa[0] = m4.x; ometa[1] = m4.y; ometa[2] = m4.z; ometa[3] = m4.w;
        otail[0] = (const uint8_t*)ta.x; otail[1] = (const uint8_t*)ta.y;
        otail[2] = (const uint8_t*)tb.x; otail[3] = (const uint8_t*)tb.y;
    }
    int ec[4], ic[4];
#pragma unroll
    for (int q = 0; q < 4; q++) {
        ec[q] = S.er[i0 + q];
        ic[q] = S.ins[i0 + q];
    }
    const int esum = ec[0] + ec[1] + ec[2] + ec[3], isum = ic[0] + ic[1] + ic[2] + ic[3];
    int erun = wave_incl_scan(esum) - esum;
    int irun = wave_incl_scan(isum) - isum;
    uint32_t keepm = 0;
    int newb[4];  // new entries at or before each slot
#pragma unroll
    for (int q = 0; q < 4; q++) {
        erun += ec[q];
        irun += ic[q];
        newb[q] = irun;
        if (i0 + q < cntp && erun == 0 && !hm.bit(i0 + q)) keepm |= 1u << q;
    }
    const int kc = __popc(keepm);
    const int kinc = wave_incl_scan(kc);
    const int kept = lane_read(kinc, 63);
    int kb[4];
    {
        int run = kinc - kc;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            kb[q] = run;
            S.er[i0 + q] = run;  // now: kept old entries before slot
            run += (keepm >> q) & 1;
        }
    }
    wave_lds_sync();
    if (lane == 0) S.er[cntp] = kept;
    wave_lds_sync();
    const int nout = kept + nn;
    const int per = cdiv(nout, parts);
    if (nout == 0 && lane == 0) {  // entry 0 emptied: an empty page whose first key sorts first
        S.f_hi[0] = 0; S.f_lo[0] = 0; S.f_meta[0] = 0; S.f_tail[0] = nullptr; S.f_dp[0] = pg;
    }
    const Dir& D = A.dst;
    auto dest = [&](int q) -> int { return q == 0 ? pg : A.free_stack[top0 - 1 - (xoff + q - 1)]; };
    // output entry m: part m / per, spread inside it (a hole after every g-th)
    auto place = [&](int m, uint64_t h, uint64_t l, uint32_t mt, int64_t ver, const uint8_t* tl, int64_t& vmax) {
        const int qq = m / per, r = m - qq * per;
        const int n = min(per, nout - qq * per), g = spread_gap(n);
        const int dp = dest(qq);
        const int64_t sl = (int64_t)dp * PAGE + spread_slot(r, g);
        put_entry(A.pool, sl, h, l, mt, ver, tl);
        if (spread_hole_after(r, n, g)) put_entry(A.pool, sl + 1, h, l, mt, ver, tl);
        if (parts == 1) vmax = max(vmax, ver);
        else if (qq < MAXP) atomicMax(&S.pmax[qq], (long long)ver);
        if (r == 0) part_first(S, D, A, a, doff, qq, per, nout, dp, h, l, mt, tl);
    };
    int64_t vmax = INT64_MIN;  // parts == 1: the page maximum by a wave reduction
    wave_loads_done();
    // ---- 3a. surviving old entries
#pragma unroll
    for (int q = 0; q < 4; q++)
        if ((keepm >> q) & 1) place(kb[q] + newb[q], ohi[q], olo[q], ometa[q], over[q], otail[q], vmax);
    // ---- 3b. new entries, by the plan lanes: b_j (version now), then e_j
    int base = 0;
    for (int j0 = jlo; j0 <= jhi; j0 += 64) {
        const int j = j0 + lane;
        const bool v = j <= jhi;
        RangePlan r{};
        if (v) r = j0 == jlo ? r0 : load_plan(A, j);
        const bool eb = v && r.pb == p && r.has_b;
        const bool ee = v && r.pe == p && r.need;
        const int c = (int)eb + (int)ee;
        const int inc = wave_incl_scan(c);
        int k = base + inc - c;  // new entries before this lane's
#pragma unroll
        for (int w = 0; w < 2; w++) {
            if (!(w == 0 ? eb : ee)) continue;
            const Key kk = w == 0 ? A.rb.get(j) : A.re.get(j);
            const int at = w == 0 ? r.ib : r.ie;
            const int64_t ver = w == 0 ? A.now : r.vb;
            const uint8_t* tl;
            copy_tail(kk, A.arena, A.arena_cap, sc, &tl);
            place(k + S.er[at], kk.hi, kk.lo, kk.meta, ver, tl, vmax);
            k++;
        }
        base += lane_read(inc, 63);
    }
    if (parts == 1) vmax = wave_reduce_max(vmax);
    wave_lds_sync();  // the LDS stash of part-first entries, written by any lane
    for (int q = lane; q < min(parts, MAXP); q += 64)  // directory entries of the parts
        part_dir(D, A, a, doff + q, q, per, nout, S.f_dp[q], S.f_hi[q], S.f_lo[q], S.f_meta[q], S.f_tail[q]);
    for (int x = lane; x < parts * HM_WORDS; x += 64) {  // the parts' hole masks
        const int q = x / HM_WORDS;
        A.pool.hmask[(int64_t)dest(q) * HM_WORDS + x % HM_WORDS] = spread_mask_word(min(per, nout - q * per), x % HM_WORDS);
    }
    if (FDBCS_DIR_PX)  // (the parts' key-prefix skips: k_page_px, after the batch)
        for (int q = lane; q < parts; q += 64) A.pool.pskip[dest(q)] = -1;
    if (parts == 1) {
        if (lane == 0) D.maxv[doff] = vmax;
        return;
    }
    if (parts > MAXP) __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");  // own pool writes, read below
    for (int q = lane; q < parts; q += 64) {
        int64_t mx;
        if (q < MAXP) {
            mx = S.pmax[q];
        } else {  // very large outputs (e.g. a first batch into an empty history)
            const int64_t bq = (int64_t)dest(q) * PAGE;
            const int c = spread_used(min(per, nout - q * per));
            mx = INT64_MIN;
            // (these slots were written by this wavefront above)
            for (int i = 0; i < c; i++) mx = max(mx, A.pool.ver[bq + i]);
        }
        D.maxv[doff + q] = mx;
    }
}

#ifndef FDBCS_PM_WAVES
#define FDBCS_PM_WAVES 3
#endif
#ifndef FDBCS_PM_UNIFIED
#define FDBCS_PM_UNIFIED 1
#endif
// PX: HistBufs::px_host (pages may hold prefix skips).  Two instantiations so
// that short-key histories (configs 2, 3, 5) never pay the long-key path's
// registers (its spill showed up as page-merge writes).
template <bool PX>
__global__ __launch_bounds__(256, FDBCS_PM_WAVES) void k_page_merge(MergeArgs A) {
    __shared__ WaveMerge S[MW_WAVES];
    Scalars* sc = A.sc;
    if (sc->err) return;
    const int naff = sc->n_aff;
    const int top0 = sc->free_top;
    const int w = threadIdx.x >> 6;
    for (int a = blockIdx.x * MW_WAVES + w; a < naff; a += gridDim.x * MW_WAVES)
        merge_page_wave<true, FDBCS_PM_UNIFIED != 0, PX>(A, S[w], a, top0);
}

__global__ __launch_bounds__(256, 2) void k_page_merge_full(MergeArgs A) {
    __shared__ WaveMerge S[MW_WAVES];
    Scalars* sc = A.sc;
    if (sc->err) return;
    const int nf = sc->n_full;
    const int top0 = sc->free_top;
    const int w = threadIdx.x >> 6;
    for (int x = blockIdx.x * MW_WAVES + w; x < nf; x += gridDim.x * MW_WAVES)
        merge_page_wave<false>(A, S[w], A.full_list[x], top0);
}

__device__ inline void dir_copy(const Dir& s, int x, const Dir& d, int y) {
    d.page[y] = s.page[x]; d.cnt[y] = s.cnt[x]; d.nr[y] = s.nr[x]; d.maxv[y] = s.maxv[x];
    d.fhi[y] = s.fhi[x]; d.flo[y] = s.flo[x]; d.fmeta[y] = s.fmeta[x]; d.ftail[y] = s.ftail[x];
}

__device__ inline void desc_copy(const DescArrays& s, int x, const Dir& d, int y) {
    d.page[y] = s.page[x]; d.cnt[y] = s.cnt[x]; d.nr[y] = s.nr[x]; d.maxv[y] = s.maxv[x];
    d.fhi[y] = s.fhi[x]; d.flo[y] = s.flo[x]; d.fmeta[y] = s.fmeta[x]; d.ftail[y] = s.ftail[x];
}

// Per-64-entry maxima of the new directory (one wavefront per group), pages
// the merge freed back onto the free stack (above the ones it took), then
// commit the directory size, free-stack top and history size.
// ------------------------------------------------------------ compaction ----
// removeBefore over the window driven by ConflictBatch::detectConflicts
// (SkipList.cpp:1198-1206, 665-702).  The window
// is the global index range [g0, g1) starting at the first boundary >=
// removalKey, budget 3*|combined|+10.  Node g is dropped iff g > g0 and both
// its version and the version of node g-1 (original values) are < oldest.
// removalKey becomes the key at g1, or "" at the end.  Survivors of the pages
// covering the window are repacked into fresh pages at FILL density.
//
// k_win_setup runs its searches with a whole wavefront: a 64-ary search over
// the directory (64 first keys compared per step), then over the page.
__device__ inline int wave_dir_search(const Dir& dir, int D, const Key& k) {
    // last j in [0, D) with j == 0 or first(j) <= k
    const int lane = threadIdx.x & 63;
    int lo = 1, hi = D;  // answer-1 in [lo-1, hi-1]; find first j in [lo, hi) with first(j) > k
    while (hi - lo > 64) {
        const int step = (hi - lo + 63) / 64;
        const int j = lo + lane * step;
        const bool le = j < hi && kcmp(dir_first(dir, j), k) <= 0;
        const uint64_t m = __ballot(le);
        const int cnt = __popcll(m);  // lanes 0..cnt-1 are <= k (monotone)
        if (cnt == 0) { hi = lo; break; }
        const int nlo = lo + (cnt - 1) * step + 1;
        const int nhi = min(hi, lo + cnt * step);
        lo = nlo;
        hi = nhi;
        if (cnt == 64) hi = min(hi, D);
    }
    const int j = lo + lane;
    const bool le = j < hi && kcmp(dir_first(dir, j), k) <= 0;
    return lo - 1 + __popcll(__ballot(le));
}

__device__ inline int wave_page_lb(const Pool& pool, int page, int cnt, const Key& k) {
    // first i with key(i) >= k: count of keys < k over up to 256 entries
    const int lane = threadIdx.x & 63;
    const int64_t b = (int64_t)page * PAGE;
    int c = 0;
    for (int i = lane; i < cnt; i += 64) c += kcmp(pool_key(pool, b + i), k) < 0;
    return wave_reduce_sum(c);
}

__device__ inline int wave_start_search(const int64_t* start, int D, int64_t g) {
    // last q in [0, D) with start[q] <= g
    const int lane = threadIdx.x & 63;
    int lo = 0, hi = D;  // find first q in [lo, hi) with start[q] > g
    while (hi - lo > 64) {
        const int step = (hi - lo + 63) / 64;
        const int q = lo + lane * step;
        const bool le = q < hi && start[q] <= g;
        const int cnt = __popcll(__ballot(le));
        if (cnt == 0) { hi = lo; break; }
        const int nlo = lo + (cnt - 1) * step + 1;
        hi = min(hi, lo + cnt * step);
        lo = nlo;
    }
    const int q = lo + lane;
    return lo - 1 + __popcll(__ballot(q < hi && start[q] <= g));
}

// The compaction window's end from its start (win_setup_wave): the last q
// with start[q] <= g and the last with start[q] <= g + 1, counted over 256
// entries a step from `from` (start[] never decreases, and start[from] <= g).
// A window of 3|C| + 10 boundaries spans ~160 directory entries at config 2:
// one round trip, where the 64-ary search over the whole directory took
// three or four dependent ones.
__device__ inline void wave_start_walk(const int64_t* start, int D, int64_t g, int from, int& le_g, int& le_g1) {
    const int lane = threadIdx.x & 63;
    for (int base = from;; base += 256) {
        int64_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {  // (every load issued before the compares)
            const int q = base + 64 * k + lane;
            v[k] = q < D ? start[q] : INT64_MAX;
        }
        int c0 = 0, c1 = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            c0 += __popcll(__ballot(v[k] <= g));
            c1 += __popcll(__ballot(v[k] <= g + 1));
        }
        if (c1 < 256 || base + 256 >= D) {
            le_g = base + c0 - 1;
            le_g1 = base + c1 - 1;
            return;
        }
    }
}

// pool slot of real boundary r of directory entry q (by one wavefront)
__device__ inline int64_t real_slot(const Pool& pool, const Dir& dir, int q, int64_t r) {
    const int pg = dir.page[q];
    uint64_t hm[HM_WORDS];
    load_hmask(pool, pg, hm);
    return (int64_t)pg * PAGE + wave_select_real(hm, dir.cnt[q], (int)r);
}

#ifndef FDBCS_WIN_SETUP_FUSED
#define FDBCS_WIN_SETUP_FUSED 1  // (A/B: scripts/build_variants.sh "old:-DFDBCS_WIN_SETUP_FUSED=0")
#endif

struct RemovalKey {
    uint64_t* hi;
    uint64_t* lo;
    uint32_t* meta;
    uint8_t* tail;
};

// The compaction window over the directory `dir` of D entries, by one
// wavefront (run by k_bmax_commit after the merge, before the commit).
// In the sharded mode (update_rk false) only g0 -- this shard's first
// boundary >= the global removalKey -- matters: the host assembles the global
// window from every shard's (H, g0) and sets removalKey itself.
__device__ void win_setup_wave(const Pool& pool, const Dir& dir, int D, Scalars* sc, const RemovalKey& rkey,
                               bool update_rk) {
    uint64_t* rk_hi = rkey.hi;
    uint64_t* rk_lo = rkey.lo;
    uint32_t* rk_meta = rkey.meta;
    uint8_t* rk_tail = rkey.tail;
    const int lane = threadIdx.x & 63;
    const int64_t H = dir.start[D];
    int64_t g0 = 0, g1 = 0;
    int pA = 1, pB = 0;
    bool has_key = false;
    Key nk{0, 0, 0, nullptr};
    if (!sc->err) {
        const Key rk{rk_hi[0], rk_lo[0], rk_meta[0], rk_tail};
#if FDBCS_WIN_SETUP_FUSED
        // After the search: the start / page / count of the 256 entries from
        // p0 in one round (the walk's, p0's own and usually q1's), p0's keys
        // and hole mask in the next, then q1's hole mask and the key at g1 --
        // two dependent round trips fewer than the separate steps below
        // (k_bmax_commit 13.6 -> 12.6 us, config 2,
        // profiles/r06_ab_win_setup.txt; a 1024-probe directory search in one
        // wavefront made it 30.9 us: 64 scattered loads a lane).
        const int p0 = wave_dir_search(dir, D, rk);
        int64_t st[4];
        int pgv[4], cnv[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
            const int q = p0 + 64 * k + lane;
            st[k] = q < D ? dir.start[q] : INT64_MAX;
            pgv[k] = q < D ? dir.page[q] : 0;
            cnv[k] = q < D ? dir.cnt[q] : 0;
        }
        const int pg0 = __shfl(pgv[0], 0), c0 = __shfl(cnv[0], 0);
        const int64_t s0 = __shfl(st[0], 0);
        uint64_t hm[HM_WORDS];
        load_hmask(pool, pg0, hm);
        const int i0 = wave_page_lb(pool, pg0, c0, rk);
        g0 = s0 + real_before(hm, i0);
        if (g0 < H) {
            const int64_t budget = 3 * (int64_t)sc->n_comb + 10;
            g1 = min(H, g0 + budget);
            pA = i0 < c0 ? p0 : p0 + 1;
            // the window's end (wave_start_walk's counts, over the entries loaded above first)
            int n0 = 0, n1 = 0;
#pragma unroll
            for (int k = 0; k < 4; k++) {
                n0 += __popcll(__ballot(st[k] <= g1 - 1));
                n1 += __popcll(__ballot(st[k] <= g1));
            }
            int q1 = p0 + n1 - 1;
            pB = p0 + n0 - 1;
            if (n1 == 256 && p0 + 256 < D) {  // (a window past 256 entries: the walk goes on from there)
                int a, b;
                wave_start_walk(dir.start, D, g1 - 1, p0 + 256, a, b);
                if (n0 == 256) pB = a;
                q1 = b;
            }
            if (g1 < H) {
                const int d = q1 - p0;  // (>= 0: start[p0] <= g0 < g1)
                int pq, cq;
                int64_t sq;
                if (d < 256) {
                    const int k = d >> 6, ln = d & 63;
                    pq = __shfl(k == 0 ? pgv[0] : k == 1 ? pgv[1] : k == 2 ? pgv[2] : pgv[3], ln);
                    cq = __shfl(k == 0 ? cnv[0] : k == 1 ? cnv[1] : k == 2 ? cnv[2] : cnv[3], ln);
                    sq = __shfl(k == 0 ? st[0] : k == 1 ? st[1] : k == 2 ? st[2] : st[3], ln);
                } else {
                    pq = dir.page[q1];
                    cq = dir.cnt[q1];
                    sq = dir.start[q1];
                }
                uint64_t hq[HM_WORDS];
                load_hmask(pool, pq, hq);
                nk = pool_key(pool, (int64_t)pq * PAGE + wave_select_real(hq, cq, (int)(g1 - sq)));
                has_key = true;
            }
        } else {
            g0 = g1 = H;
        }
#else
        const int p0 = wave_dir_search(dir, D, rk);
        const int i0 = wave_page_lb(pool, dir.page[p0], dir.cnt[p0], rk);
        uint64_t hm[HM_WORDS];
        load_hmask(pool, dir.page[p0], hm);
        g0 = dir.start[p0] + real_before(hm, i0);
        if (g0 < H) {
            const int64_t budget = 3 * (int64_t)sc->n_comb + 10;
            g1 = min(H, g0 + budget);
            pA = i0 < dir.cnt[p0] ? p0 : p0 + 1;
            int q1;  // the entry holding g1 (when g1 < H)
            wave_start_walk(dir.start, D, g1 - 1, p0, pB, q1);
            if (g1 < H) {
                nk = pool_key(pool, real_slot(pool, dir, q1, g1 - dir.start[q1]));
                has_key = true;
            }
        } else {
            g0 = g1 = H;
        }
#endif
    }
    if (lane == 0 && update_rk && !sc->err && g0 < g1) {  // tail arena GC: where this sweep stands
        int tf = sc->tail_flags;
        if (g0 == 0) tf = TF_FROM_START;  // a sweep from the first boundary starts here (it can move everything)
        if (g1 >= H) tf |= TF_WRAP;
        sc->tail_flags = tf;
    }
    if (lane == 0) {
        sc->win_g0 = g0;
        sc->win_r0 = g0 + 1;  // the first scanned node is never removed
        sc->win_prev = 0;     // (not needed: g0 + 1 > 0)
        sc->win_g1 = g1;
        sc->win_pA = pA;
        sc->win_pB = pB;
        sc->win_np = pB - pA + 1 > 0 ? pB - pA + 1 : 0;
        if (!sc->err && update_rk) {
            rk_hi[0] = has_key ? nk.hi : 0;
            rk_lo[0] = has_key ? nk.lo : 0;
            rk_meta[0] = has_key ? nk.meta : 0;
        }
    }
    if (!sc->err && update_rk && has_key && key_len(nk.meta) > 17) {
        const uint32_t words = (key_len(nk.meta) - 17 + 7) / 8;
        const uint64_t* s = reinterpret_cast<const uint64_t*>(nk.tail);
        uint64_t* d = reinterpret_cast<uint64_t*>(rk_tail);
        for (uint32_t w = lane; w < words; w += 64) d[w] = s[w];
    }
}

// level-1 entry i of the search index, and the entries of higher levels it
// starts (i a multiple of 16^(l-1))
__device__ inline void sidx_put(const Dir& d, int i, uint64_t v) {
    d.sidx[i] = v;
    int ii = i;
    for (int l = 2; l <= SIDX_LEVELS && (ii & (SIDX_B - 1)) == 0; l++) {
        ii >>= SIDX_LOG;
        d.sidx[sidx_off(d.cap, l) + ii] = v;
    }
}

__device__ inline void sidx_build(const Dir& d, int i) {
    const uint64_t v = d.fhi[(int64_t)i * SIDX_B];
    d.sidx[i] = v;
    int ii = i;
    for (int l = 2; l <= SIDX_LEVELS && (ii & (SIDX_B - 1)) == 0; l++) {
        ii >>= SIDX_LOG;
        d.sidx[sidx_off(d.cap, l) + ii] = v;
    }
}

__global__ __launch_bounds__(256) void k_sidx_build(Dir d, const int32_t* D) {
    const int n1 = cdiv(*D, SIDX_B);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n1; i += gridDim.x * blockDim.x) sidx_build(d, i);
}

// Dir::wsk / fpx / spx of a finished directory (common.h): a thread per
// entry of each level.  Window w of level l holds entries x = (16w + t) <<
// 4l; the searches reach it only with keys in [first(16w << 4l),
// first((16w + 16) << 4l)) -- except window 0, whose entry 0 is the default
// target of keys below every first key, and the last window -- so those two
// keys' common prefix is the query's too.  (Every thread of a window works
// its skip out from the same two keys.)  Level-0 threads also list the
// entries whose page was rewritten (Pool::pskip < 0) for k_page_px, where
// their window has a skip.
__device__ inline int window_skip(const Dir& d, int D, int l, int w) {
    const int64_t x0 = (int64_t)(SIDX_B * w) << (SIDX_LOG * l);
    const int64_t x1 = (int64_t)(SIDX_B * w + SIDX_B) << (SIDX_LOG * l);
    if (w == 0 || x1 >= D) return 0;
    const uint64_t h0 = d.fhi[x0], h1 = d.fhi[x1], l0 = d.flo[x0], l1 = d.flo[x1];
    const uint32_t m0 = d.fmeta[x0], m1 = d.fmeta[x1];
    if (h0 != h1 || l0 != l1 || (m0 >> 24) != (m1 >> 24) || key_len(m0) <= 17 || key_len(m1) <= 17) return 0;
    const int skip = key_lcp(Key{h0, l0, m0, d.ftail[x0]}, Key{h1, l1, m1, d.ftail[x1]});
    return skip < PX_MIN_SKIP ? 0 : min(skip, PX_MAX_SKIP);  // (a shorter skip is as valid)
}

// The levels lie side by side in one index space, each from a multiple of
// 16 (so a window never straddles a block): every level's windows at once,
// not one dependent pass per level.  Position f -> level l, its index i, and
// n = the level's entries (0 past the last level).
__device__ inline void px_level_of(int D, int f, int& l, int& i, int& n) {
    int base = 0;
    l = 0;
    n = D;
    for (;;) {
        const int span = (n + SIDX_B - 1) & ~(SIDX_B - 1);
        if (f < base + span) break;
        const int nn = l < SIDX_LEVELS ? sidx_n(D, l + 1) : 0;
        base += span;
        l++;
        if (nn <= 1) {  // (past the last level k_dir_px builds)
            n = 0;
            break;
        }
        n = nn;
    }
    i = f - base;
}
__device__ inline int px_positions(int D) {  // (the first position past the last level)
    int f = 0;
    for (int k = 0; k <= SIDX_LEVELS; k++) {
        const int nk = sidx_n(D, k);
        if (k > 0 && nk <= 1) break;
        f += (nk + SIDX_B - 1) & ~(SIDX_B - 1);
    }
    return f;
}

__global__ __launch_bounds__(256) void k_dir_px(Dir d, const int32_t* Dp, Pool pool, int32_t* list, int32_t* n_list,
                                              int32_t* n_next, const int32_t* px_on) {
    __shared__ int s_skip[256 / SIDX_B];
    const int D = *Dp;
    const int64_t cap = d.cap;
    if (blockIdx.x == 0 && threadIdx.x == 0) *n_next = 0;  // (the other parity's list: the next directory's)
    if (!*px_on) return;  // (no key past 17 bytes yet: every skip is still 0)
    const int nf = px_positions(D);
    // (block-uniform trip count: the barrier below)
    for (int f0 = blockIdx.x * blockDim.x; f0 < nf; f0 += gridDim.x * blockDim.x) {
        int l, i, n;
        px_level_of(D, f0 + (int)threadIdx.x, l, i, n);
        const int w = i >> SIDX_LOG;
        if ((i & (SIDX_B - 1)) == 0) {  // (levels start on a multiple of 16: i's window starts with f's)
            const int sk = i < n ? window_skip(d, D, l, w) : 0;
            s_skip[threadIdx.x / SIDX_B] = sk;
            if (i < n) d.wsk[wsk_off(cap, l) + w] = sk;
        }
        __syncthreads();
        const int skip = s_skip[threadIdx.x / SIDX_B];
        __syncthreads();
        if (i >= n || !skip) continue;
        const int x = (int)((int64_t)i << (SIDX_LOG * l));
        (l == 0 ? d.fpx : d.spx + sidx_off(cap, l))[i] = key_bytes_at(dir_first(d, x), skip);
        // (a page's skip counts only under a window skip: pages elsewhere
        // stay listed as rewritten until their window has one)
        if (l == 0 && pool.pskip[d.page[x]] < 0) {
            const int k = atomicAdd(n_list, 1);
            if (k < d.cap) list[k] = x;
        }
    }
}

// Pool::pskip / px / pxidx of the pages k_dir_px listed, a wavefront each:
// the skip is the common prefix of the page's first and last keys (so of
// all of them), used by the searches only where the page's directory window
// vouches for it (common.h Pool).
__global__ __launch_bounds__(256) void k_page_px(Dir d, Pool pool, const int32_t* list, const int32_t* n_list) {
    const int n = min(*n_list, d.cap);
    const int lane = threadIdx.x & 63;
    for (int k = blockIdx.x * 4 + (threadIdx.x >> 6); k < n; k += gridDim.x * 4) {
        const int x = list[k];
        const int pg = d.page[x], c = d.cnt[x];
        const int64_t b = (int64_t)pg * PAGE;
        int skip = 0;
        if (c > 1) {
            const Key a = pool_key(pool, b), z = pool_key(pool, b + c - 1);  // (the last used slot is real)
            if (a.hi == z.hi && a.lo == z.lo && (a.meta >> 24) == (z.meta >> 24) && key_len(a.meta) > 17 &&
                key_len(z.meta) > 17) {
                // (rounded down to 8 bytes: a page spans a sliver of its
                // window, so its own common prefix often runs a byte or two
                // past the window's -- then the window could not vouch for it)
                skip = min(key_lcp(a, z), PX_MAX_SKIP) & ~7;
                if (skip < PX_MIN_SKIP) skip = 0;
            }
        }
        if (skip) {
            // (every slot's words loaded before any store: a store between
            // them would keep the next slot's loads behind it, two round
            // trips a slot)
            uint64_t v[PAGE / 64];
#pragma unroll
            for (int q = 0; q < PAGE / 64; q++) {
                const int i = lane + 64 * q;
                v[q] = i < c ? key_bytes_at(pool_key(pool, b + i), skip) : 0;
            }
#pragma unroll
            for (int q = 0; q < PAGE / 64; q++) {
                const int i = lane + 64 * q;
                if (i >= c) continue;
                pool.px[b + i] = v[q];
                if ((i & (PIDX_STRIDE - 1)) == 0) pool.pxidx[(b + i) / PIDX_STRIDE] = v[q];
            }
        }
        if (lane == 0) pool.pskip[pg] = skip;
    }
}

// (the list's count alternates between two scalars: each k_dir_px zeroes the
// one the next k_dir_px counts into, so no memset node sits in the chain)
// Launched only once the host has seen a long key come through (the
// batch-ending kernel's mirror, one batch late at most): until then no skip
// was ever built, so the zero skips stay right and the two launches (~9 us
// of the update chain) are saved.
void launch_dir_px(HistBufs& h, int which, Scalars* sc, hipStream_t s) {
    if (!FDBCS_DIR_PX) return;
    if (!h.px_host && h.mirror_host && h.mirror_host->px_on) h.px_host = true;
    if (!h.px_host) return;
    const int par = h.px_par;
    h.px_par ^= 1;
    hipLaunchKernelGGL(k_dir_px, dim3(std::max(1, std::min(256, cdiv(h.cap_dir, 256)))), dim3(256), 0, s,
                       h.dir[which], &sc->D, h.pool, h.px_list, &sc->n_pxd[par], &sc->n_pxd[par ^ 1], &sc->px_on);
    hipLaunchKernelGGL(k_page_px, dim3(64), dim3(256), 0, s, h.dir[which], h.pool, (const int32_t*)h.px_list,
                       (const int32_t*)&sc->n_pxd[par]);
}

void launch_sidx_build(HistBufs& h, int which, Scalars* sc, hipStream_t s) {
    hipLaunchKernelGGL(k_sidx_build, dim3(cdiv(cdiv(h.cap_dir, SIDX_B), 256)), dim3(256), 0, s, h.dir[which], &sc->D);
    launch_dir_px(h, which, sc, s);
}

// the batch's load-metrics roll counters (common.h LmArgs) become the
// synchronized host's view; the next batch's ingest starts from zero
__device__ inline void lm_end_of_batch(Scalars* sc) {
    sc->lm_out_count = sc->lm_count;
    sc->lm_out_bytes = sc->lm_bytes;
    sc->lm_count = 0;
    sc->lm_bytes = 0;
}

// the scalars to the host-mapped mirror: one wavefront of a block whose
// thread 0 just committed (after a barrier), 8 bytes per lane
__device__ inline void publish_scalars(const Scalars* sc, Scalars* mirror) {
    const uint64_t* s = reinterpret_cast<const uint64_t*>(sc);
    uint64_t* m = reinterpret_cast<uint64_t*>(mirror);
    for (int i = threadIdx.x; i < (int)(sizeof(Scalars) / 8); i += 64) m[i] = s[i];
}

__global__ __launch_bounds__(256) void k_bmax_commit(Dir d, Scalars* sc, const int32_t* freed_list,
                                                     int32_t* free_stack, int end_of_batch, Pool pool,
                                                     RemovalKey rkey, Scalars* mirror, int sharded) {
    const int Dn = sc->D_next;
    // a compaction follows: its window over the new directory (one wavefront)
    if (!end_of_batch && blockIdx.x == 0 && threadIdx.x < 64) win_setup_wave(pool, d, Dn, sc, rkey, !sharded);
    if (freed_list) {
        // (free_base, not free_top: block 0 commits free_top below while later
        // blocks may not have started -- reading it here was a race that
        // corrupted the free stack under contention, e.g. two processes
        // sharing the GPU)
        const int base = sc->free_base;
        const int nf = sc->free_next - base;
        for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < nf; i += gridDim.x * blockDim.x)
            free_stack[base + i] = freed_list[i];
    }
    const int n1 = cdiv(Dn, SIDX_B);
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n1; i += gridDim.x * blockDim.x) sidx_build(d, i);
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (g * 64 < Dn) {
        const int x = g * 64 + lane;
        int64_t m = x < Dn ? d.maxv[x] : INT64_MIN;
        m = wave_reduce_max(m);
        if (lane == 0) d.bmax[g] = m;
    }
    // block 0 commits (no other block reads what it writes: D_next, free_base,
    // free_next and extra_total stay)
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        sc->D = Dn;
        sc->free_top = sc->free_next;
        sc->H = d.start[Dn];
        sc->last_ver = d.cnt[Dn - 1] > 0 ? pool.ver[(int64_t)d.page[Dn - 1] * PAGE + d.cnt[Dn - 1] - 1] : INT64_MIN;
        if (end_of_batch) {  // the next batch's encoder allocates from these
            sc->last_err = sc->err;
            sc->err = 0;
            if (sc->btail_used) sc->px_on = 1;  // (a long key came through: the prefix skips, from now on)
            sc->btail_used = 0;
            sc->ss_over[0] = sc->ss_over[1] = 0;  // (a sort overflow no guard ran for: not the next batch's)
            lm_end_of_batch(sc);
        }
    }
    if (end_of_batch && blockIdx.x == 0) {
        __syncthreads();
        if (threadIdx.x < 64) publish_scalars(sc, mirror);
    }
}

static void launch_bmax_commit(HistBufs& h, int which, Scalars* sc, hipStream_t s, bool end_of_batch,
                               const int32_t* freed_list = nullptr) {
    const int groups = cdiv(h.cap_dir, 64);
    const RemovalKey rk{h.rk_hi, h.rk_lo, h.rk_meta, h.rk_tail};
    hipLaunchKernelGGL(k_bmax_commit, dim3(cdiv(groups, 4)), dim3(256), 0, s, h.dir[which], sc, freed_list,
                       h.free_stack, (int)end_of_batch, h.pool, rk, h.mirror,
                       (int)(h.shard.has_lo | h.shard.has_hi));
    if (end_of_batch) launch_dir_px(h, which, sc, s);  // (else the compaction's k_win_dir builds the final directory)
}

void launch_dir_finish(HistBufs& h, int cur, Scalars* sc, BatchBufs& b, hipStream_t s) {
    // full recompute of start[] (used after reset / load)
    Dir& d = h.dir[cur];
    scan_i64_from_i32(d.nr, d.start, &sc->D, 0, &sc->H, b.scan_tmp, s);
    (void)hipMemcpyAsync(&sc->D_next, &sc->D, sizeof(int32_t), hipMemcpyDeviceToDevice, s);
    (void)hipMemcpyAsync(&sc->free_next, &sc->free_top, sizeof(int32_t), hipMemcpyDeviceToDevice, s);
    launch_bmax_commit(h, cur, sc, s, true);
}

int plan_blocks(int cap_dir) { return cdiv(cap_dir, PS_BLOCK); }

void launch_merge(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t now,
                  int64_t v0, bool end_of_batch, hipStream_t s) {
    const int W = v.write_count;
    Dir& src = h.dir[cur];
    Dir& dst = h.dir[cur ^ 1];
    if (W > 0) {
        hipLaunchKernelGGL(k_plan_ranges, dim3(cdiv(W, 256)), dim3(256), 0, s, (const int32_t*)b.cb_pos,
                           (const int32_t*)b.ce_pos, (const SRec*)b.sw, (const uint8_t* const*)b.keys.tail, b.wh,
                           write_base(b, v), v0, h.shard, sc, b.pb, b.ib, b.pe, b.ie, b.need_e, b.vb, b.acc, b.rkb, b.rke);
    }
    const int nblk = plan_blocks(h.cap_dir);
    hipLaunchKernelGGL(k_plan_aggr, dim3(nblk), dim3(PS_THREADS), 0, s, src, (const Scalars*)sc, b.acc, b.blk_agg,
                       b.blk_diff);
    PlanArgs P;
    P.src = src; P.dst = dst; P.sc = sc; P.acc = b.acc; P.blk_agg = b.blk_agg; P.blk_diff = b.blk_diff;
    P.aff_list = b.aff_list; P.aff_jlo = b.aff_jlo; P.aff_jhi = b.aff_jhi; P.aff_nn = b.aff_nn;
    P.aff_parts = b.aff_parts; P.aff_nn_off = b.aff_nn_off; P.aff_parts_off = b.aff_parts_off;
    P.aff_extra_off = b.aff_extra_off; P.aff_free_off = b.aff_free_off; P.aff_start = b.aff_start;
    P.aff_page = b.aff_page; P.aff_cnt = b.aff_cnt;
    hipLaunchKernelGGL(k_plan_scan, dim3(nblk), dim3(PS_THREADS), 0, s, P);
    if (W > 0) {
        const int max_aff = std::min<int64_t>(h.cap_dir, 4 * (int64_t)W + 4);
        MergeArgs A;
        A.pool = h.pool; A.dir = src; A.dst = dst; A.sc = sc; A.free_stack = h.free_stack; A.freed_list = b.freed_list;
        A.aff_list = b.aff_list; A.aff_page = b.aff_page; A.aff_cnt = b.aff_cnt;
        A.jlo = b.aff_jlo; A.jhi = b.aff_jhi; A.nn = b.aff_nn; A.nn_off = b.aff_nn_off; A.parts = b.aff_parts;
        A.parts_off = b.aff_parts_off; A.extra_off = b.aff_extra_off; A.free_off = b.aff_free_off;
        A.aff_start = b.aff_start;
        A.pb = b.pb; A.ib = b.ib; A.pe = b.pe; A.ie = b.ie; A.need_e = b.need_e; A.vb = b.vb;
        A.rb = b.rkb; A.re = b.rke; A.ne = b.ne; A.ne_ins = b.ne_ins;
        A.arena = h.tail_arena; A.arena_cap = h.tail_cap; A.now = now;
        A.px = h.px_host ? 1 : 0;
        A.full_list = b.full_list;
        const int grid = std::max(1, std::min(GRID_PAGES, cdiv(max_aff, MW_WAVES)));
        if (A.px)
            hipLaunchKernelGGL(k_page_merge<true>, dim3(grid), dim3(256), 0, s, A);
        else
            hipLaunchKernelGGL(k_page_merge<false>, dim3(grid), dim3(256), 0, s, A);
        if (!FDBCS_PM_UNIFIED) hipLaunchKernelGGL(k_page_merge_full, dim3(std::min(grid, 1024)), dim3(256), 0, s, A);
    }
    launch_bmax_commit(h, cur ^ 1, sc, s, end_of_batch, b.freed_list);
}

__global__ __launch_bounds__(256) void k_win_keep(Pool pool, Dir dir, const Scalars* sc, int64_t oldest,
                                                  uint8_t* __restrict__ keep_o, int32_t* __restrict__ cnt_o,
                                                  int64_t* __restrict__ part_max) {
    __shared__ int32_t tmp[256 / 64 + 1];
    const int64_t r0 = sc->win_r0, g1 = sc->win_g1, prev0 = sc->win_prev;
    const int pA = sc->win_pA, np = sc->win_np;
    for (int w = blockIdx.x; w < np; w += gridDim.x) {
        // the repack makes at most ceil(np * PAGE / FILL) <= 2 * np pages
        if (threadIdx.x < 2) part_max[2 * w + threadIdx.x] = INT64_MIN;
        const int q = pA + w;
        const int pg = dir.page[q], c = dir.cnt[q];
        const int64_t st = dir.start[q];
        const int i = threadIdx.x;
        // holes are dropped (the repack spreads fresh ones); global indices
        // count the real boundaries before slot i
        const bool real = i < c && !((pool.hmask[(int64_t)pg * HM_WORDS + (i >> 6)] >> (i & 63)) & 1);
        int nreal;
        const int ri = block_excl_scan((int)real, tmp, nreal);
        int keep = 0;
        if (i < c) keep_o[(int64_t)w * PAGE + i] = 0;
        if (real) {
            keep = 1;
            const int64_t g = st + ri;
            if (g >= r0 && g < g1) {
                const bool above = pool.ver[(int64_t)pg * PAGE + i] >= oldest;
                const int64_t pv = i > 0    ? pool.ver[(int64_t)pg * PAGE + i - 1]
                                   : q > 0 && dir.cnt[q - 1] > 0
                                       ? pool.ver[(int64_t)dir.page[q - 1] * PAGE + dir.cnt[q - 1] - 1]
                                       : prev0;  // (sharded: the previous shard's last node; only entry 0
                                                 // can be an empty page)
                keep = above || pv >= oldest;
            }
            keep_o[(int64_t)w * PAGE + i] = (uint8_t)keep;
        }
        const int tot = block_reduce_sum(keep, tmp);
        if (threadIdx.x == 0) cnt_o[w] = tot;
    }
}

// survivors -> fresh pages at FILL density, with their descriptors; each
// workgroup's survivors span at most 3 parts, reduced in LDS before one
// global atomic per part
__global__ __launch_bounds__(256) void k_win_repack(Pool pool, Dir dir, Scalars* sc,
                                                    const uint8_t* __restrict__ keep, const int32_t* __restrict__ cnt,
                                                    const int32_t* __restrict__ free_stack, DescArrays desc,
                                                    uint8_t* arena, uint64_t arena_cap, int gc) {
    __shared__ int32_t tmp[256 / 64 + 1];
    __shared__ long long lmax[4];
    const int np = sc->win_np;
    const int pA = sc->win_pA;
    const int top0 = sc->free_top;
    // this block's first page (usually its only one): its entry, keep flags
    // and slots loaded before the survivor sums below, so those loads do not
    // wait behind the sums' barriers (two dependent round trips)
    const int i = threadIdx.x;
    int pg0 = 0, c0 = 0, kp0 = 0;
    uint64_t hi0 = 0, lo0 = 0;
    uint32_t meta0 = 0;
    int64_t ver0 = 0;
    const uint8_t* tail0 = nullptr;
    if ((int)blockIdx.x < np) {
        pg0 = dir.page[pA + blockIdx.x];
        c0 = dir.cnt[pA + blockIdx.x];
        if (i < c0) {
            kp0 = keep[(int64_t)blockIdx.x * PAGE + i];
            const int64_t sidx = (int64_t)pg0 * PAGE + i;
            hi0 = pool.hi[sidx];
            lo0 = pool.lo[sidx];
            meta0 = pool.meta[sidx];
            ver0 = pool.ver[sidx];
            tail0 = pool.tail[sidx];
        }
    }
    // survivors in all window pages (S) and before this block's first page:
    // the window is a few hundred pages, so every block sums the counts
    int all = 0;
    for (int v = threadIdx.x; v < np; v += blockDim.x) all += cnt[v];
    const int S = block_reduce_sum(all, tmp);
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        sc->win_surv = S;
        if (!gc) atomicOr(&sc->tail_flags, TF_NOGC);  // (nothing moved: this sweep frees nothing)
    }
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    const int per = k > 0 ? cdiv(S, k) : 1;
    int before = 0;  // survivors in pages [0, w), advanced by the grid stride
    int wprev = 0;
    for (int w = blockIdx.x; w < np; w += gridDim.x) {
        int part_sum = 0;
        for (int v = wprev + threadIdx.x; v < w; v += blockDim.x) part_sum += cnt[v];
        before += block_reduce_sum(part_sum, tmp);
        wprev = w;
        const int offw = before;
        const bool first = w == (int)blockIdx.x;
        const int q = pA + w;
        const int pg = first ? pg0 : dir.page[q], c = first ? c0 : dir.cnt[q];
        if (i < 4) lmax[i] = INT64_MIN;
        const int kp = first ? kp0 : (i < c ? keep[(int64_t)w * PAGE + i] : 0);
        int tot;
        const int ex = block_excl_scan(kp, tmp, tot);
        const int part0 = offw / per;
        if (kp) {
            const int m = offw + ex;
            const int part = m / per, r = m - part * per;
            const int n = min(per, S - part * per), g = spread_gap(n);  // spread with fresh holes
            const int dp = free_stack[top0 - 1 - part];
            const int64_t sidx = (int64_t)pg * PAGE + i;
            const uint64_t hi = first ? hi0 : pool.hi[sidx], lo = first ? lo0 : pool.lo[sidx];
            const uint32_t meta = first ? meta0 : pool.meta[sidx];
            const int64_t ver = first ? ver0 : pool.ver[sidx];
            const uint8_t* tail = first ? tail0 : pool.tail[sidx];
            if (gc) tail = move_tail(tail, meta, arena, arena_cap, sc);
            const int64_t d = (int64_t)dp * PAGE + spread_slot(r, g);
            put_entry(pool, d, hi, lo, meta, ver, tail);
            if (spread_hole_after(r, n, g)) put_entry(pool, d + 1, hi, lo, meta, ver, tail);
            atomicMax(&lmax[min(3, part - part0)], (long long)ver);
            if (r == 0) {
                put_desc(desc, part, dp, n, hi, lo, meta, tail);
                for (int w2 = 0; w2 < HM_WORDS; w2++) pool.hmask[(int64_t)dp * HM_WORDS + w2] = spread_mask_word(n, w2);
                if (FDBCS_DIR_PX) pool.pskip[dp] = -1;  // (k_page_px, after the batch)
            }
        }
        __syncthreads();
        if (i < 4 && lmax[i] != INT64_MIN) atomicMax((long long*)&desc.maxv[part0 + i], lmax[i]);
        __syncthreads();
    }
}

// The directory after the compaction, its page-group maxima and search index
// (what k_bmax_commit does after a merge), and the commit by the last block.
__global__ __launch_bounds__(1024) void k_win_dir(Dir src, Dir dst, Scalars* sc, DescArrays desc,
                                                  int32_t* free_stack, Scalars* mirror, const int64_t* pool_ver) {
    __shared__ int last;
    const int np = sc->win_np;
    const int S = sc->win_surv;
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    const int per = k > 0 ? cdiv(S, k) : 1;
    const int D = sc->D, pA = sc->win_pA;
    // sharded mode can remove a shard's whole history: its first page then
    // stays as one empty entry (the directory never has zero entries)
    const int keep = (S == 0 && np == D && np > 0) ? 1 : 0;
    const int Dn = D - np + k + keep;
    const int64_t removed = np ? (src.start[pA + np] - src.start[pA]) - S : 0;
    const int free_next = sc->free_top - k + np - keep;
    const int64_t H = src.start[D] - removed;
    const int top = sc->free_top;
    if (blockIdx.x == 0 && threadIdx.x == 0) dst.start[Dn] = H;
    // grid-stride over entries (few blocks: each one bumps the commit counter)
    const int n = max(Dn, np);
    for (int y0 = blockIdx.x * blockDim.x; y0 < n; y0 += gridDim.x * blockDim.x) {
        const int y = y0 + threadIdx.x;
        int64_t mv = INT64_MIN;
        if (y < Dn) {
            // (the entry's fields in registers: its maximum and first key feed
            // the group maxima and the search index without reading back
            // what was just stored -- a round trip each)
            int pg, cn, nrr;
            int64_t st;
            uint64_t fh, fl;
            uint32_t fm;
            const uint8_t* ft;
            if (keep) {  // (Dn == 1)
                pg = src.page[0]; cn = 0; nrr = 0; mv = INT64_MIN;
                fh = 0; fl = 0; fm = 0; ft = nullptr; st = 0;
            } else if (np == 0 || y < pA || y >= pA + k) {
                const int x = np == 0 || y < pA ? y : y - k + np;
                pg = src.page[x]; cn = src.cnt[x]; nrr = src.nr[x]; mv = src.maxv[x];
                fh = src.fhi[x]; fl = src.flo[x]; fm = src.fmeta[x]; ft = src.ftail[x];
                st = np == 0 || y < pA ? src.start[x] : src.start[x] - removed;
            } else {
                const int x = y - pA;
                pg = desc.page[x]; cn = desc.cnt[x]; nrr = desc.nr[x]; mv = desc.maxv[x];
                fh = desc.fhi[x]; fl = desc.flo[x]; fm = desc.fmeta[x]; ft = desc.ftail[x];
                st = src.start[pA] + (int64_t)x * per;
            }
            dst.page[y] = pg; dst.cnt[y] = cn; dst.nr[y] = nrr; dst.maxv[y] = mv;
            dst.fhi[y] = fh; dst.flo[y] = fl; dst.fmeta[y] = fm; dst.ftail[y] = ft;
            dst.start[y] = st;
            if ((y & (SIDX_B - 1)) == 0) sidx_put(dst, y / SIDX_B, fh);
        }
        if (y < np - keep) free_stack[top - k + y] = src.page[pA + keep + y];
        mv = wave_reduce_max(mv);  // one wavefront = one 64-entry group
        if ((threadIdx.x & 63) == 0 && (y & ~63) < Dn) dst.bmax[y >> 6] = mv;
    }
    // commit once every block has read the pre-compaction scalars (no fence:
    // the values were consumed before the barrier, and the directory itself
    // is published by the kernel boundary -- a device-scope fence would write
    // back every XCD's L2)
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(&sc->blocks_done, 1) == (int)gridDim.x - 1;
    __syncthreads();
    if (!last) return;
    if (threadIdx.x == 0) {
        sc->blocks_done = 0;
        sc->D = Dn;
        sc->D_next = Dn;
        sc->free_top = free_next;
        sc->free_next = free_next;
        sc->H = H;
        {  // the last boundary: from the repacked pages when the window reached the end
            int lp = -1, lc = 0;
            if (np > 0 && pA + np == D) {
                if (k > 0) {
                    lp = desc.page[k - 1];
                    lc = desc.cnt[k - 1];
                } else if (pA > 0) {
                    lp = src.page[pA - 1];
                    lc = src.cnt[pA - 1];
                }
            } else {
                lp = src.page[D - 1];
                lc = src.cnt[D - 1];
            }
            sc->last_ver = lp >= 0 && lc > 0 ? pool_ver[(int64_t)lp * PAGE + lc - 1] : INT64_MIN;
        }
        sc->win_newpages = k;
        const int tf = sc->tail_flags;
        if (tf & TF_WRAP) {  // a sweep ended: if it covered everything and moved every tail, free the old half
            if ((tf & TF_FROM_START) && !(tf & TF_NOGC)) {
                sc->tail_half ^= 1;
                sc->tail_used = 0;
            }
            sc->tail_flags = 0;
        }
        sc->last_err = sc->err;  // end of batch: the next batch's encoder allocates from these
        sc->err = 0;
        if (sc->btail_used) sc->px_on = 1;
        sc->btail_used = 0;
        sc->ss_over[0] = sc->ss_over[1] = 0;  // (a sort overflow no guard ran for: not the next batch's)
        lm_end_of_batch(sc);
    }
    __syncthreads();
    if (threadIdx.x < 64) publish_scalars(sc, mirror);
}

// Sharded mode: the host hands this shard its part [a, b) of the global
// compaction window (local indices), whether a is the window's first node
// (never removed), and the version of the node before a when a == 0.
// Tail arena GC in a shard: the global sweep visits the shard's boundaries
// in key order, entering at its first (a == 0) and leaving at its last
// (b == H), so a shard's run of window parts from a == 0 to b == H has moved
// every tail alive when it entered -- the unsharded sweep's rule
// (k_bmax_commit) restricted to the shard's keys.
__device__ inline void shard_sweep_flags(Scalars* sc, int64_t a, int64_t b, int64_t H) {
    if (a >= b) return;
    int tf = sc->tail_flags;
    if (a == 0) tf = TF_FROM_START;
    if (b >= H) tf |= TF_WRAP;
    sc->tail_flags = tf;
}

__global__ __launch_bounds__(64) void k_win_explicit(Dir dir, Scalars* sc, int64_t a, int64_t b, int keep_first,
                                                     int64_t prev) {
    const int D = sc->D;
    const int pA = a < b ? wave_start_search(dir.start, D, a) : 1;
    const int pB = a < b ? wave_start_search(dir.start, D, b - 1) : 0;
    if (threadIdx.x == 0) {
        shard_sweep_flags(sc, a, b, dir.start[D]);
        sc->win_g0 = a;
        sc->win_r0 = keep_first ? a + 1 : a;
        sc->win_g1 = b;
        sc->win_prev = prev;
        sc->win_pA = pA;
        sc->win_pB = pB;
        sc->win_np = pB - pA + 1 > 0 ? pB - pA + 1 : 0;
    }
}

// the key at local index g (0 <= g < H) into out (hi, lo, meta) + out_tail
__global__ __launch_bounds__(64) void k_key_at(Pool pool, Dir dir, const Scalars* sc, int64_t g, uint64_t* out,
                                               uint8_t* out_tail) {
    const int D = sc->D;
    const int q = wave_start_search(dir.start, D, g);
    const Key k = pool_key(pool, real_slot(pool, dir, q, g - dir.start[q]));
    if (threadIdx.x == 0) {
        out[0] = k.hi;
        out[1] = k.lo;
        out[2] = k.meta;
    }
    const uint32_t L = key_len(k.meta);
    if (L > 17)
        for (uint32_t w = threadIdx.x; w < (L - 17 + 7) / 8; w += 64)
            reinterpret_cast<uint64_t*>(out_tail)[w] = reinterpret_cast<const uint64_t*>(k.tail)[w];
}

void launch_key_at(HistBufs& h, int cur, Scalars* sc, int64_t g, uint64_t* out, uint8_t* out_tail, hipStream_t s) {
    hipLaunchKernelGGL(k_key_at, dim3(1), dim3(64), 0, s, h.pool, h.dir[cur], (const Scalars*)sc, g, out, out_tail);
}

static constexpr int WIN_DIR_BLOCKS = 128;

void launch_compact(BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t oldest, hipStream_t s,
                    const WinExplicit* win) {
    Dir& src = h.dir[cur];
    Dir& dst = h.dir[cur ^ 1];
    const int win_cap = b.win_cap_pages;
    if (win)
        hipLaunchKernelGGL(k_win_explicit, dim3(1), dim3(64), 0, s, src, sc, win->a, win->b, win->keep_first,
                           win->prev);
    hipLaunchKernelGGL(k_win_keep, dim3(std::min(GRID_PAGES, win_cap)), dim3(256), 0, s, h.pool, src, sc, oldest,
                       b.win_keep, b.win_cnt, b.desc_max);
    DescArrays da{b.desc_page, b.desc_cnt, b.desc_nr, b.desc_max, b.desc_fhi, b.desc_flo, b.desc_fmeta, b.desc_ftail};
    // (FDBCS_NO_SHARD_GC: a shard's windows move no tails and free no half -- A/B and fault hunting)
    static const bool no_shard_gc = getenv("FDBCS_NO_SHARD_GC") != nullptr;
    const int gc = (h.shard.has_lo | h.shard.has_hi) && no_shard_gc ? 0 : 1;
    hipLaunchKernelGGL(k_win_repack, dim3(std::min(GRID_PAGES, win_cap)), dim3(256), 0, s, h.pool, src, sc,
                       b.win_keep, b.win_cnt, h.free_stack, da, h.tail_arena, h.tail_cap, gc);
    hipLaunchKernelGGL(k_win_dir, dim3(std::min(WIN_DIR_BLOCKS, cdiv(h.cap_dir, 1024))), dim3(1024), 0, s, src, dst,
                       sc, da, h.free_stack, h.mirror, (const int64_t*)h.pool.ver);
    launch_dir_px(h, cur ^ 1, sc, s);
}

// --------------------------------------------------------- nth after ----
// fdbcs_nth_after: per query (a wavefront each) the key of the boundary
// `step` positions after the first boundary >= key, or "none" past the end.
__global__ __launch_bounds__(64) void k_nth_after(NthArgs A) {
    const int q = blockIdx.x;
    if (q >= A.n) return;
    const int lane = threadIdx.x;
    const Key k{A.qhi[q], A.qlo[q], A.qmeta[q], A.qtail[q]};
    const int D = A.sc->D;
    const int64_t H = A.dir.start[D];
    const int p0 = wave_dir_search(A.dir, D, k);
    const int i0 = wave_page_lb(A.pool, A.dir.page[p0], A.dir.cnt[p0], k);
    uint64_t hm[HM_WORDS];
    load_hmask(A.pool, A.dir.page[p0], hm);
    const int64_t j = A.dir.start[p0] + real_before(hm, i0) + A.steps[q];
    if (j < 0 || j >= H) {
        if (lane == 0) A.out[3 * (int64_t)q + 2] = ~0ull;
        return;
    }
    const int qq = wave_start_search(A.dir.start, D, j);
    const Key r = pool_key(A.pool, real_slot(A.pool, A.dir, qq, j - A.dir.start[qq]));
    if (lane == 0) {
        A.out[3 * (int64_t)q] = r.hi;
        A.out[3 * (int64_t)q + 1] = r.lo;
        A.out[3 * (int64_t)q + 2] = r.meta;
    }
    const uint32_t L = key_len(r.meta);
    if (L > 17)
        for (uint32_t w = lane; w < (L - 17 + 7) / 8 && 8 * (w + 1) <= A.tail_stride; w += 64)
            reinterpret_cast<uint64_t*>(A.out_tail + (int64_t)q * A.tail_stride)[w] =
                reinterpret_cast<const uint64_t*>(r.tail)[w];
}

void launch_nth_after(HistBufs& h, int cur, const Scalars* sc, const NthArgs& a0, hipStream_t s) {
    NthArgs a = a0;
    a.pool = h.pool;
    a.dir = h.dir[cur];
    a.sc = sc;
    if (a.n > 0) hipLaunchKernelGGL(k_nth_after, dim3(a.n), dim3(64), 0, s, a);
}

// ------------------------------------------------ fdbcs_sharded (device) ----
// SURVEY.md §8e protocol A with its exchanges and host-side arithmetic moved
// onto the device (foundationdb_amd/sharded.py holds the same steps in
// Python): slots of exchange 1 (k_sh_slot_out), the apply carry-in
// (k_sh_carry), this shard's (H, g0, last, own begins) for exchange 2
// (k_sh_info_out), and the compaction plan over global indices + the next
// removalKey's owner (k_sh_plan, SkipList.cpp:665-702 over the concatenated
// shards).  Slots / infos are SH_WORDS int64 per shard.
__global__ __launch_bounds__(64) void k_sh_init(Scalars* sc, int64_t v0, int reset_owner) {
    if (threadIdx.x == 0) {
        sc->carry_dev = 1;
        sc->carry_check = v0;
        sc->carry_apply = v0;
        if (reset_owner) sc->sh_rk_owner = -1;
    }
}

// after a batch: this shard's (H, last version) in its slot, zeros elsewhere
// (exchange 1 is a byte-wise MAX all-reduce, so it delivers every slot)
__global__ __launch_bounds__(64) void k_sh_slot_out(const Scalars* sc, int64_t* slots, int rank, int G) {
    for (int i = threadIdx.x; i < SH_WORDS * G; i += blockDim.x) {
        const int k = i % SH_WORDS;
        int64_t v = 0;
        if (i / SH_WORDS == rank) v = k == 0 ? sc->H : (k == 1 ? (sc->H ? sc->last_ver : INT64_MIN) : 0);
        slots[i] = v;
    }
}

// step 4: the carry-in of the apply -- the last version of the nearest
// earlier non-empty shard after the previous compaction, or v0
__global__ __launch_bounds__(64) void k_sh_carry(Scalars* sc, const int64_t* slots, int rank, int64_t v0) {
    if (threadIdx.x != 0) return;
    int64_t cur = v0;
    for (int g = 0; g < rank; g++)
        if (slots[g * SH_WORDS] > 0) cur = slots[g * SH_WORDS + 1];
    sc->carry_apply = cur;
}

// exchange 2's contribution after the merge: (H, g0, last, own begins).  g0 =
// the first local index >= removalKey: only the owner searches (k_bmax_commit
// before a compaction); shards below the owner hold only smaller keys (H),
// shards above only larger ones (0); "" (no owner): 0
__global__ __launch_bounds__(64) void k_sh_info_out(const Scalars* sc, int64_t* send, int rank, int bounded) {
    if (threadIdx.x != 0) return;
    const int owner = sc->sh_rk_owner;
    const int64_t H = sc->H;
    send[0] = H;
    send[1] = owner == rank ? sc->win_g0 : (owner < 0 ? 0 : (rank < owner ? H : 0));
    send[2] = H ? sc->last_ver : INT64_MIN;
    send[3] = bounded ? sc->n_comb_own : sc->n_comb;  // (one unbounded shard: every range begins in it)
}

// steps 6-7 from exchange 2's infos: the carry-in of the next check, and with
// a compaction the window's part in this shard (as k_win_explicit) and the
// boundary that becomes removalKey (copied into rk by its owner)
__global__ __launch_bounds__(64) void k_sh_plan(Pool pool, Dir dir, Scalars* sc, const int64_t* infos, int rank,
                                                int G, int64_t v0, int compact, RemovalKey rk) {
    __shared__ int64_t s_part[4];
    __shared__ int64_t s_owner[2];
    if (sc->err == E_SH_RETRY) {  // (a short edge exchange: this attempt changes nothing; no window)
        if (threadIdx.x == 0) sc->win_np = 0;
        return;
    }
    if (threadIdx.x == 0) {
        int64_t tot = 0, carry = v0, cur = v0;
        for (int g = 0; g < G; g++) {
            if (g == rank) carry = cur;
            if (infos[g * SH_WORDS] > 0) cur = infos[g * SH_WORDS + 2];
        }
        sc->carry_check = carry;
        int64_t n_comb = 0, G0 = -1, off_me = 0, H_me = infos[rank * SH_WORDS];
        for (int g = 0; g < G; g++) {
            const int64_t H = infos[g * SH_WORDS], g0 = infos[g * SH_WORDS + 1];
            if (g == rank) off_me = tot;
            if (G0 < 0 && g0 < H) G0 = tot + g0;
            tot += H;
            n_comb += infos[g * SH_WORDS + 3];
        }
        int64_t a = 0, b = 0, keep = 0, prev = 0, og = -1, oi = 0;
        if (G0 >= 0) {
            const int64_t G1 = min(tot, G0 + 3 * n_comb + 10);
            a = min(max(G0 - off_me, (int64_t)0), H_me);
            b = min(max(G1 - off_me, (int64_t)0), H_me);
            keep = off_me <= G0 && G0 < off_me + H_me;
            if (a == 0 && a < b && !keep) {  // the node before a: the nearest earlier non-empty shard's last
                int64_t pl = 0;
                for (int g = 0; g < rank; g++)
                    if (infos[g * SH_WORDS] > 0) pl = infos[g * SH_WORDS + 2];
                prev = pl;
            }
            if (G1 < tot) {
                int64_t o = 0;
                for (int g = 0; g < G; g++) {
                    const int64_t H = infos[g * SH_WORDS];
                    if (o <= G1 && G1 < o + H) {
                        og = g;
                        oi = G1 - o;
                        break;
                    }
                    o += H;
                }
            }
        }
        s_part[0] = a; s_part[1] = b; s_part[2] = keep; s_part[3] = prev;
        s_owner[0] = og; s_owner[1] = oi;
    }
    __syncthreads();
    if (!compact) return;
    const int64_t a = s_part[0], b = s_part[1];
    const int D = sc->D;
    const int pA = a < b ? wave_start_search(dir.start, D, a) : 1;
    const int pB = a < b ? wave_start_search(dir.start, D, b - 1) : 0;
    const int og = (int)s_owner[0];
    if (og == rank) {  // this shard holds the next removalKey: read it before the compaction moves it
        const int64_t g = s_owner[1];
        const int q = wave_start_search(dir.start, D, g);
        const Key k = pool_key(pool, real_slot(pool, dir, q, g - dir.start[q]));
        if (threadIdx.x == 0) {
            rk.hi[0] = k.hi;
            rk.lo[0] = k.lo;
            rk.meta[0] = k.meta;
        }
        const uint32_t L = key_len(k.meta);
        if (L > 17)
            for (uint32_t w = threadIdx.x; w < (L - 17 + 7) / 8; w += 64)
                reinterpret_cast<uint64_t*>(rk.tail)[w] = reinterpret_cast<const uint64_t*>(k.tail)[w];
    }
    if (threadIdx.x == 0) {
        shard_sweep_flags(sc, a, b, dir.start[D]);
        sc->win_g0 = a;
        sc->win_r0 = s_part[2] ? a + 1 : a;
        sc->win_g1 = b;
        sc->win_prev = s_part[3];
        sc->win_pA = pA;
        sc->win_pB = pB;
        sc->win_np = pB - pA + 1 > 0 ? pB - pA + 1 : 0;
        sc->sh_rk_owner = og;
    }
}

void launch_sh_init(Scalars* sc, int64_t v0, bool reset_owner, hipStream_t s) {
    hipLaunchKernelGGL(k_sh_init, dim3(1), dim3(64), 0, s, sc, v0, (int)reset_owner);
}
void launch_sh_slot_out(const Scalars* sc, int64_t* slots, int rank, int G, hipStream_t s) {
    hipLaunchKernelGGL(k_sh_slot_out, dim3(1), dim3(64), 0, s, sc, slots, rank, G);
}
void launch_sh_carry(Scalars* sc, const int64_t* slots, int rank, int64_t v0, hipStream_t s) {
    hipLaunchKernelGGL(k_sh_carry, dim3(1), dim3(64), 0, s, sc, slots, rank, v0);
}
void launch_sh_info_out(const Scalars* sc, int64_t* send, int rank, bool bounded, hipStream_t s) {
    hipLaunchKernelGGL(k_sh_info_out, dim3(1), dim3(64), 0, s, sc, send, rank, (int)bounded);
}
void launch_sh_plan(HistBufs& h, int cur, Scalars* sc, const int64_t* infos, int rank, int G, int64_t v0, bool compact,
                    hipStream_t s) {
    const RemovalKey rk{h.rk_hi, h.rk_lo, h.rk_meta, h.rk_tail};
    hipLaunchKernelGGL(k_sh_plan, dim3(1), dim3(64), 0, s, h.pool, h.dir[cur], sc, infos, rank, G, v0, (int)compact,
                       rk);
}

// ---- protocol B: the overlap edges' exchange ----------------
// Exchange 1 carries this shard's edge count (slot word 2) and whether its
// edge list overflowed (word 3); the other shards' words are zero, so the MAX
// all-reduce delivers every shard's.
__global__ __launch_bounds__(64) void k_sh_edges_count(const Scalars* sc, int64_t* slots, int rank, int G,
                                                       int64_t edge_cap) {
    for (int g = threadIdx.x; g < G; g += blockDim.x) {
        int64_t n = 0, ovf = 0;
        if (g == rank) {
            n = sc->edges_total;
            ovf = n < 0 || n > edge_cap;  // (the counter wraps past 2^31 pairs)
            if (n < 0) n = INT32_MAX;
        }
        slots[g * SH_WORDS + 2] = n;
        slots[g * SH_WORDS + 3] = ovf;
    }
}

// this shard's list, zero padded to M pairs: [readers M | writers M]
__global__ __launch_bounds__(256) void k_sh_edges_pack(const int32_t* __restrict__ et, const int32_t* __restrict__ eu,
                                                       const Scalars* sc, int64_t M, int32_t* __restrict__ send) {
    const int64_t n = min((int64_t)sc->edges_total, M);
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < M; i += (int64_t)gridDim.x * blockDim.x) {
        send[i] = i < n ? et[i] : 0;
        send[M + i] = i < n ? eu[i] : 0;
    }
}

// The fixed-capacity form (one host wait per batch, sh_exchange_b): every
// shard sent min(count, M) pairs; one block concatenates the gathered lists
// in shard order into (cat_et, cat_eu) and sets edges_total.  If some shard's
// count exceeded M, or some shard's own list overflowed, the batch cannot be
// decided from these: err = E_SH_RETRY (the history stages then change
// nothing) and sh_need = the largest count.
__global__ __launch_bounds__(1024) void k_sh_edges_cat_fixed(const int32_t* __restrict__ recv, const int64_t* slots,
                                                             int G, int64_t M, int32_t* __restrict__ cat_et,
                                                             int32_t* __restrict__ cat_eu, Scalars* sc) {
    int64_t off = 0, mx = 0;
    int64_t ovf = 0;
    for (int g = 0; g < G; g++) {
        const int64_t c = slots[g * SH_WORDS + 2], n = min(c, M);
        mx = max(mx, c);
        ovf |= slots[g * SH_WORDS + 3];
        const int32_t* src = recv + 2 * M * g;
        for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
            cat_et[off + i] = src[i];
            cat_eu[off + i] = src[M + i];
        }
        off += n;
    }
    if (threadIdx.x == 0) {
        sc->edges_total = (int32_t)off;
        sc->sh_max = (int32_t)min<int64_t>(mx, INT32_MAX);
        if (mx > M || ovf) {
            sc->sh_need = (int32_t)min<int64_t>(mx, INT32_MAX);
            atomicCAS(&sc->err, 0, E_SH_RETRY);
        }
    }
}

void launch_sh_edges_count(const Scalars* sc, int64_t* slots, int rank, int G, int64_t edge_cap, hipStream_t s) {
    hipLaunchKernelGGL(k_sh_edges_count, dim3(1), dim3(64), 0, s, sc, slots, rank, G, edge_cap);
}
void launch_sh_edges_pack(const BatchBufs& b, const Scalars* sc, int64_t M, int32_t* send, hipStream_t s) {
    const int nb = (int)std::min<int64_t>(1024, (M + 255) / 256);
    hipLaunchKernelGGL(k_sh_edges_pack, dim3(std::max(1, nb)), dim3(256), 0, s, b.et, b.eu, sc, M, send);
}
void launch_sh_edges_cat_fixed(const int32_t* recv, const int64_t* slots, int G, int64_t M, int32_t* cat_et,
                               int32_t* cat_eu, Scalars* sc, hipStream_t s) {
    hipLaunchKernelGGL(k_sh_edges_cat_fixed, dim3(1), dim3(1024), 0, s, recv, slots, G, M, cat_et, cat_eu, sc);
}
// ------------------------------------------------------------------ reset ----
__global__ __launch_bounds__(256) void k_reset(Dir d, int32_t* free_stack, int cap_pages, Scalars* sc,
                                              uint64_t* hmask, int32_t* pskip) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < HM_WORDS) hmask[i] = 0;  // page 0: empty
    if (i < cap_pages - 1) free_stack[i] = cap_pages - 1 - i;  // pops yield page 1, 2, ...
    if (i < cap_pages) pskip[i] = 0;
    if (i == 0) {
        d.page[0] = 0; d.cnt[0] = 0; d.nr[0] = 0; d.maxv[0] = INT64_MIN; d.start[0] = 0; d.start[1] = 0;
        d.fhi[0] = 0; d.flo[0] = 0; d.fmeta[0] = 0; d.ftail[0] = nullptr; d.bmax[0] = INT64_MIN;
        sc->D = 1;
        sc->free_top = cap_pages - 1;
        sc->H = 0;
        sc->tail_used = 0;
        sc->tail_half = 0;
        sc->tail_flags = 0;
        sc->err = 0;
        sc->lm_count = 0;
        sc->lm_bytes = 0;
    }
}

void launch_reset_history(HistBufs& h, int cur, Scalars* sc, hipStream_t s) {
    hipLaunchKernelGGL(k_reset, dim3(cdiv(h.cap_pages, 256)), dim3(256), 0, s, h.dir[cur], h.free_stack,
                       h.cap_pages, sc, h.pool.hmask, h.pool.pskip);
}

}  // namespace fdbcs_dev

namespace fdbcs_dev {

// --------------------------------------------------------- dump / growth ----
__global__ __launch_bounds__(256) void k_gather(Pool pool, Dir dir, const Scalars* sc, Pool out) {
    const int D = sc->D;
    __shared__ int32_t tmp[256 / 64 + 1];
    for (int x = blockIdx.x; x < D; x += gridDim.x) {  // (a thread per slot: PAGE == blockDim)
        const int c = dir.cnt[x], pg = dir.page[x];
        const int64_t b = (int64_t)pg * PAGE;
        const int i = threadIdx.x;
        const bool real = i < c && !((pool.hmask[(int64_t)pg * HM_WORDS + (i >> 6)] >> (i & 63)) & 1);
        int tot;
        const int64_t o = dir.start[x] + block_excl_scan((int)real, tmp, tot);
        if (real) {
            out.hi[o] = pool.hi[b + i];
            out.lo[o] = pool.lo[b + i];
            out.meta[o] = pool.meta[b + i];
            out.ver[o] = pool.ver[b + i];
            out.tail[o] = pool.tail[b + i];
        }
    }
}

void launch_gather(HistBufs& h, int cur, Scalars* sc, Pool out, hipStream_t s) {
    hipLaunchKernelGGL(k_gather, dim3(GRID_PAGES), dim3(256), 0, s, h.pool, h.dir[cur], sc, out);
}

__global__ void k_push_free(int32_t* free_stack, int32_t from_top, int32_t first_id, int32_t count) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < count) free_stack[from_top + i] = first_id + count - 1 - i;
}

void launch_push_free(HistBufs& h, int32_t from_top, int32_t first_id, int32_t count, hipStream_t s) {
    if (count <= 0) return;
    hipLaunchKernelGGL(k_push_free, dim3(cdiv(count, 256)), dim3(256), 0, s, h.free_stack, from_top, first_id, count);
}

__global__ __launch_bounds__(256) void k_relocate(const uint8_t** p, int64_t n, const uint8_t* old_base,
                                                  uint64_t old_half, const uint8_t* new_base, uint64_t new_half) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* t = p[i];
    if (t >= old_base && t < old_base + old_half) p[i] = new_base + (t - old_base);
    else if (t >= old_base + old_half && t < old_base + 2 * old_half) p[i] = new_base + new_half + (t - old_base - old_half);
}
// tail pointers into an arena of old_cap bytes -> one of new_cap bytes (each half to its half)
void launch_relocate_tails(HistBufs& h, const uint8_t* old_base, uint64_t old_cap, const uint8_t* new_base,
                           uint64_t new_cap, hipStream_t s) {
    const int64_t n = (int64_t)h.cap_pages * PAGE;
    const uint64_t oh = tail_half_bytes(old_cap), nh = tail_half_bytes(new_cap);
    hipLaunchKernelGGL(k_relocate, dim3(cdiv(n, 256)), dim3(256), 0, s, h.pool.tail, n, old_base, oh, new_base, nh);
    for (int d = 0; d < 2; d++)
        hipLaunchKernelGGL(k_relocate, dim3(cdiv(h.cap_dir, 256)), dim3(256), 0, s, h.dir[d].ftail,
                           (int64_t)h.cap_dir, old_base, oh, new_base, nh);
}

}  // namespace fdbcs_dev
