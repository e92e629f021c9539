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
#include <algorithm>
#include "kernels.h"
#include "devutil.h"
#include "hist_search.h"

namespace fdbcs_dev {

static constexpr int GRID_PAGES = 2048;  // workgroups for per-page kernels (grid-stride)

// ------------------------------------------------ small single-block scan ----
template <int NA>
struct ScanArgs {
    const int32_t* in[NA];
    int32_t* out[NA];
};

// Exclusive scans of NA int32 arrays of the same device-resident length n;
// out[k][n] receives the total.  One workgroup, contiguous segment per thread.
template <int NA>
__global__ __launch_bounds__(1024) void k_scan_small(ScanArgs<NA> a, const int32_t* n_ptr) {
    __shared__ int32_t tmp[1024 / 64 + 1];
    const int n = *n_ptr;
    const int per = (n + blockDim.x - 1) / blockDim.x;
    const int beg = min(n, (int)threadIdx.x * per), end = min(n, beg + per);
#pragma unroll
    for (int k = 0; k < NA; k++) {
        int s = 0;
        for (int i = beg; i < end; i++) s += a.in[k][i];
        int tot;
        int run = block_excl_scan(s, tmp, tot);
        for (int i = beg; i < end; i++) {
            const int x = a.in[k][i];
            a.out[k][i] = run;
            run += x;
        }
        if (threadIdx.x == 0) a.out[k][n] = tot;
    }
}

// ------------------------------------------------------- insertion plan ----
// Per combined range j: where b and e fall in the pre-batch history, whether
// e needs a node, and the value it keeps.  Marks the pages [pb, pe] touched.
__global__ __launch_bounds__(256) void k_bounds(KeyArrays cb, KeyArrays ce, Pool pool, Dir dir, Scalars* sc,
                                                int64_t v0, int32_t* __restrict__ pb_o, int32_t* __restrict__ ib_o,
                                                int32_t* __restrict__ pe_o, int32_t* __restrict__ ie_o,
                                                uint8_t* __restrict__ need_o, int64_t* __restrict__ vb_o,
                                                int32_t* __restrict__ aff_flag) {
    if (sc->err) return;
    const int nC = sc->n_comb;
    const int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= nC) return;
    const int D = sc->D;
    const Key b = cb.get(j), e = ce.get(j);
    const int p_b = dir_search(dir, D, b, 1);
    const int c_b = dir.cnt[p_b], g_b = dir.page[p_b];
    const int i_b = page_lb(pool, g_b, 0, c_b, b);
    int p_e = p_b;
    if (p_b + 1 < D && kcmp(dir_first(dir, p_b + 1), e) <= 0) p_e = dir_search(dir, D, e, p_b + 1);
    const int c_e = dir.cnt[p_e], g_e = dir.page[p_e];
    const int i_e = page_lb(pool, g_e, p_e == p_b ? i_b : 0, c_e, e);
    const bool found = i_e < c_e && kcmp(pool_key(pool, (int64_t)g_e * PAGE + i_e), e) == 0;
    int64_t vb;
    if (i_e > 0) vb = pool.ver[(int64_t)g_e * PAGE + i_e - 1];
    else if (p_e > 0) vb = pool.ver[(int64_t)dir.page[p_e - 1] * PAGE + dir.cnt[p_e - 1] - 1];
    else vb = v0;
    const bool touch = j + 1 < nC && kcmp(cb.get(j + 1), e) == 0;
    pb_o[j] = p_b;
    ib_o[j] = i_b;
    pe_o[j] = p_e;
    ie_o[j] = i_e;
    need_o[j] = (!found && !touch) ? 1 : 0;
    vb_o[j] = vb;
    for (int p = p_b; p <= p_e; p++) aff_flag[p] = 1;
}

__global__ __launch_bounds__(256) void k_aff_scatter(const int32_t* __restrict__ flag, const int32_t* __restrict__ pos,
                                                     int32_t* __restrict__ list, const Scalars* sc) {
    const int p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < sc->D && flag[p]) list[pos[p]] = p;
}

// Per affected page: the range of combined writes touching it, surviving old
// entries, new entries landing in it, and how many output pages it becomes.
__global__ __launch_bounds__(256) void k_aff_plan(Dir dir, const Scalars* sc, const int32_t* __restrict__ aff_list,
                                                  const int32_t* __restrict__ pb, const int32_t* __restrict__ ib,
                                                  const int32_t* __restrict__ pe, const int32_t* __restrict__ ie,
                                                  const uint8_t* __restrict__ need_e, int32_t* __restrict__ jlo_o,
                                                  int32_t* __restrict__ jhi_o, int32_t* __restrict__ nn_o,
                                                  int32_t* __restrict__ parts_o, int32_t* __restrict__ extra_o,
                                                  int32_t* __restrict__ freed_o) {
    __shared__ int32_t tmp[256 / 64 + 1];
    const int naff = sc->err ? 0 : sc->n_aff, nC = sc->n_comb;
    for (int a = blockIdx.x; a < naff; a += gridDim.x) {
        const int p = aff_list[a], cntp = dir.cnt[p];
        int lo = 0, hi = nC;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (pe[mid] < p) lo = mid + 1; else hi = mid;
        }
        const int jlo = lo;
        lo = 0; hi = nC;
        while (lo < hi) {
            int mid = (lo + hi) >> 1;
            if (pb[mid] <= p) lo = mid + 1; else hi = mid;
        }
        const int jhi = lo - 1;
        int erased = 0, nn = 0;
        for (int j = jlo + threadIdx.x; j <= jhi; j += blockDim.x) {
            const int s = pb[j] < p ? 0 : ib[j];
            const int en = pe[j] > p ? cntp : ie[j];
            erased += max(0, en - s);
            nn += (pb[j] == p) + (pe[j] == p && need_e[j]);
        }
        erased = block_reduce_sum(erased, tmp);
        nn = block_reduce_sum(nn, tmp);
        if (threadIdx.x == 0) {
            const int nout = cntp - erased + nn;
            const int parts = nout == 0 ? 0 : (nout <= PAGE ? 1 : cdiv(nout, FILL));
            jlo_o[a] = jlo;
            jhi_o[a] = jhi;
            nn_o[a] = nn;
            parts_o[a] = parts;
            extra_o[a] = parts > 1 ? parts - 1 : 0;
            freed_o[a] = parts == 0;
        }
        __syncthreads();
    }
}

__device__ inline void copy_tail(const Key& k, uint8_t* arena, uint64_t cap, Scalars* sc, const uint8_t** out) {
    const uint32_t L = key_len(k.meta);
    if (L <= 17) {
        *out = nullptr;
        return;
    }
    const uint64_t padded = ((uint64_t)(L - 17) + 7) & ~7ull;
    const uint64_t o = atomicAdd((unsigned long long*)&sc->tail_used, (unsigned long long)padded);
    if (o + padded > cap) {
        atomicCAS(&sc->err, 0, FDBCS_E_CAPACITY);
        *out = nullptr;
        return;
    }
    const uint64_t* src = reinterpret_cast<const uint64_t*>(k.tail);
    uint64_t* dst = reinterpret_cast<uint64_t*>(arena + o);
    for (uint64_t w = 0; w < padded / 8; w++) dst[w] = src[w];
    *out = arena + o;
}

struct MergeArgs {
    Pool pool;
    Dir dir;
    Scalars* sc;
    const int32_t* free_stack;
    const int32_t* aff_list;
    const int32_t *jlo, *jhi, *nn, *nn_off, *parts, *parts_off, *extra_off;
    const int32_t *pb, *ib, *pe, *ie;
    const uint8_t* need_e;
    const int64_t* vb;
    KeyArrays cb, ce;
    Pool ne;
    int32_t* ne_ins;
    int32_t* desc_page;
    int32_t* desc_cnt;
    int64_t* desc_max;
    uint64_t* desc_fhi;
    uint64_t* desc_flo;
    uint32_t* desc_fmeta;
    const uint8_t** desc_ftail;
    uint8_t* arena;
    uint64_t arena_cap;
    int64_t now;
};

// One workgroup per affected page: load it into LDS, drop erased entries,
// merge in the new boundaries, write 0..k output pages (the first in place,
// the others from the free stack) and their directory descriptors.
__global__ __launch_bounds__(256) void k_page_merge(MergeArgs A) {
    __shared__ uint64_t o_hi[PAGE], o_lo[PAGE];
    __shared__ uint32_t o_meta[PAGE];
    __shared__ int64_t o_ver[PAGE];
    __shared__ const uint8_t* o_tail[PAGE];
    __shared__ int32_t kb[PAGE + 1];
    __shared__ int32_t tmp[256 / 64 + 1];
    Scalars* sc = A.sc;
    if (sc->err) return;
    const int naff = sc->n_aff;
    const int top0 = sc->free_top;
    const int tid = threadIdx.x;
    for (int a = blockIdx.x; a < naff; a += gridDim.x) {
        const int p = A.aff_list[a];
        const int pg = A.dir.page[p], cntp = A.dir.cnt[p];
        const int jlo = A.jlo[a], jhi = A.jhi[a];
        const int nn = A.nn[a], nn_off = A.nn_off[a];
        const int parts = A.parts[a];
        const int64_t pbase = (int64_t)pg * PAGE;
        if (tid < cntp) {
            o_hi[tid] = A.pool.hi[pbase + tid];
            o_lo[tid] = A.pool.lo[pbase + tid];
            o_meta[tid] = A.pool.meta[pbase + tid];
            o_ver[tid] = A.pool.ver[pbase + tid];
            o_tail[tid] = A.pool.tail[pbase + tid];
        }
        // erased iff inside [(pb_j, ib_j), (pe_j, ie_j)) for the last j starting at or before (p, tid)
        int keep = 0;
        if (tid < cntp) {
            int lo = jlo, hi = jhi + 1;
            while (lo < hi) {
                int mid = (lo + hi) >> 1;
                if (pos_le(A.pb[mid], A.ib[mid], p, tid)) lo = mid + 1; else hi = mid;
            }
            const int j = lo - 1;
            const bool erased = j >= jlo && pos_lt(p, tid, A.pe[j], A.ie[j]);
            keep = !erased;
        }
        int kept;
        const int kex = block_excl_scan(keep, tmp, kept);
        if (tid < cntp) kb[tid] = kex;
        if (tid == 0) kb[cntp] = kept;
        // new entries landing here, in key order: b_j (version now), then e_j
        int local = 0;
        for (int jb = jlo; jb <= jhi; jb += blockDim.x) {
            const int j = jb + tid;
            const bool eb = j <= jhi && A.pb[j] == p;
            const bool ee = j <= jhi && A.pe[j] == p && A.need_e[j];
            int t2;
            const int ex = block_excl_scan((int)eb + (int)ee, tmp, t2);
            int k = nn_off + local + ex;
            if (eb) {
                const Key kk = A.cb.get(j);
                A.ne.hi[k] = kk.hi; A.ne.lo[k] = kk.lo; A.ne.meta[k] = kk.meta; A.ne.ver[k] = A.now;
                copy_tail(kk, A.arena, A.arena_cap, sc, &A.ne.tail[k]);
                A.ne_ins[k] = A.ib[j];
                k++;
            }
            if (ee) {
                const Key kk = A.ce.get(j);
                A.ne.hi[k] = kk.hi; A.ne.lo[k] = kk.lo; A.ne.meta[k] = kk.meta; A.ne.ver[k] = A.vb[j];
                copy_tail(kk, A.arena, A.arena_cap, sc, &A.ne.tail[k]);
                A.ne_ins[k] = A.ie[j];
            }
            local += t2;
        }
        __threadfence_block();
        __syncthreads();
        const int nout = kept + nn;
        const int per = parts > 0 ? cdiv(nout, parts) : 1;
        const int xoff = A.extra_off[a];
        auto dest = [&](int q) -> int { return q == 0 ? pg : A.free_stack[top0 - 1 - (xoff + q - 1)]; };
        if (tid < cntp && keep) {
            int lo = 0, hi = nn;
            while (lo < hi) {
                int mid = (lo + hi) >> 1;
                if (A.ne_ins[nn_off + mid] <= tid) lo = mid + 1; else hi = mid;
            }
            const int m = kb[tid] + lo;
            const int q = m / per;
            const int64_t d = (int64_t)dest(q) * PAGE + (m - q * per);
            A.pool.hi[d] = o_hi[tid]; A.pool.lo[d] = o_lo[tid]; A.pool.meta[d] = o_meta[tid];
            A.pool.ver[d] = o_ver[tid]; A.pool.tail[d] = o_tail[tid];
        }
        for (int k = tid; k < nn; k += blockDim.x) {
            const int s = nn_off + k;
            const int m = k + kb[A.ne_ins[s]];
            const int q = m / per;
            const int64_t d = (int64_t)dest(q) * PAGE + (m - q * per);
            A.pool.hi[d] = A.ne.hi[s]; A.pool.lo[d] = A.ne.lo[s]; A.pool.meta[d] = A.ne.meta[s];
            A.pool.ver[d] = A.ne.ver[s]; A.pool.tail[d] = A.ne.tail[s];
        }
        __threadfence_block();
        __syncthreads();
        const int doff = A.parts_off[a];
        for (int q = tid; q < parts; q += blockDim.x) {
            const int c = min(per, nout - q * per);
            const int pgq = dest(q);
            const int64_t bq = (int64_t)pgq * PAGE;
            int64_t mx = INT64_MIN;
            for (int i = 0; i < c; i++) mx = max(mx, A.pool.ver[bq + i]);
            A.desc_page[doff + q] = pgq;
            A.desc_cnt[doff + q] = c;
            A.desc_max[doff + q] = mx;
            A.desc_fhi[doff + q] = A.pool.hi[bq];
            A.desc_flo[doff + q] = A.pool.lo[bq];
            A.desc_fmeta[doff + q] = A.pool.meta[bq];
            A.desc_ftail[doff + q] = A.pool.tail[bq];
        }
        __syncthreads();
    }
}

__device__ inline void dir_copy(const Dir& s, int x, const Dir& d, int y) {
    d.page[y] = s.page[x]; d.cnt[y] = s.cnt[x]; d.maxv[y] = s.maxv[x];
    d.fhi[y] = s.fhi[x]; d.flo[y] = s.flo[x]; d.fmeta[y] = s.fmeta[x]; d.ftail[y] = s.ftail[x];
}

struct DescArrays {
    const int32_t* page;
    const int32_t* cnt;
    const int64_t* maxv;
    const uint64_t* fhi;
    const uint64_t* flo;
    const uint32_t* fmeta;
    const uint8_t* const* ftail;
};

__device__ inline void desc_copy(const DescArrays& s, int x, const Dir& d, int y) {
    d.page[y] = s.page[x]; d.cnt[y] = s.cnt[x]; d.maxv[y] = s.maxv[x];
    d.fhi[y] = s.fhi[x]; d.flo[y] = s.flo[x]; d.fmeta[y] = s.fmeta[x]; d.ftail[y] = s.ftail[x];
}

// Directory after the merge: unaffected entries move by the number of extra
// pages inserted before them; affected entries are replaced by their parts.
__global__ __launch_bounds__(256) void k_dir_rebuild(Dir src, Dir dst, const Scalars* sc, DescArrays desc,
                                                     const int32_t* __restrict__ aff_list,
                                                     const int32_t* __restrict__ parts,
                                                     const int32_t* __restrict__ parts_off,
                                                     const int32_t* __restrict__ freed,
                                                     const int32_t* __restrict__ free_off,
                                                     const int32_t* __restrict__ extra_off, int32_t* free_stack) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const int D = sc->D;
    if (x >= D) return;
    const int naff = sc->err ? 0 : sc->n_aff;
    if (naff == 0) {
        dir_copy(src, x, dst, x);
        return;
    }
    int lo = 0, hi = naff;
    while (lo < hi) {
        int mid = (lo + hi) >> 1;
        if (aff_list[mid] < x) lo = mid + 1; else hi = mid;
    }
    const int na = lo;
    const int base = x - na + parts_off[na];
    if (na < naff && aff_list[na] == x) {
        const int np = parts[na], off = parts_off[na];
        for (int q = 0; q < np; q++) desc_copy(desc, off + q, dst, base + q);
        if (freed[na]) free_stack[sc->free_top - extra_off[naff] + free_off[na]] = src.page[x];
    } else {
        dir_copy(src, x, dst, base);
    }
}

__global__ void k_dir_commit(Scalars* sc, const int32_t* parts_off, const int32_t* extra_off,
                             const int32_t* free_off) {
    const int naff = sc->err ? 0 : sc->n_aff;
    if (naff > 0) {
        sc->D = sc->D - naff + parts_off[naff];
        sc->free_top = sc->free_top - extra_off[naff] + free_off[naff];
    }
}

__global__ __launch_bounds__(256) void k_bmax(Dir d, const Scalars* sc) {
    const int g = blockIdx.x * blockDim.x + threadIdx.x;
    const int D = sc->D;
    if (g * 64 >= D) return;
    int64_t m = INT64_MIN;
    for (int x = g * 64; x < min(D, g * 64 + 64); x++) m = max(m, d.maxv[x]);
    d.bmax[g] = m;
}

void launch_dir_finish(HistBufs& h, int cur, Scalars* sc, BatchBufs& b, hipStream_t s) {
    Dir& d = h.dir[cur];
    scan_i64_from_i32(d.cnt, d.start, &sc->D, 0, &sc->H, b.scan_tmp, s);
    hipLaunchKernelGGL(k_bmax, dim3(cdiv(cdiv(h.cap_dir, 64), 256)), dim3(256), 0, s, d, sc);
}

void launch_merge(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t now,
                  int64_t v0, hipStream_t s) {
    const int W = v.write_count;
    Dir& src = h.dir[cur];
    Dir& dst = h.dir[cur ^ 1];
    hipMemsetAsync(&sc->n_aff, 0, sizeof(int32_t), s);
    if (W > 0) {
        hipMemsetAsync(b.aff_flag, 0, sizeof(int32_t) * (size_t)(h.cap_dir + 1), s);
        hipLaunchKernelGGL(k_bounds, dim3(cdiv(W, 256)), dim3(256), 0, s, b.cb, b.ce, h.pool, src, sc, v0, b.pb,
                           b.ib, b.pe, b.ie, b.need_e, b.vb, b.aff_flag);
        scan_i32(b.aff_flag, b.aff_pos, &sc->D, 0, &sc->n_aff, b.scan_tmp, s);
        hipLaunchKernelGGL(k_aff_scatter, dim3(cdiv(h.cap_dir, 256)), dim3(256), 0, s, b.aff_flag, b.aff_pos,
                           b.aff_list, sc);
        hipLaunchKernelGGL(k_aff_plan, dim3(GRID_PAGES), dim3(256), 0, s, src, sc, b.aff_list, b.pb, b.ib, b.pe,
                           b.ie, b.need_e, b.aff_jlo, b.aff_jhi, b.aff_nn, b.aff_parts, b.aff_extra, b.aff_freed);
        ScanArgs<4> sa;
        sa.in[0] = b.aff_nn; sa.out[0] = b.aff_nn_off;
        sa.in[1] = b.aff_parts; sa.out[1] = b.aff_parts_off;
        sa.in[2] = b.aff_extra; sa.out[2] = b.aff_extra_off;
        sa.in[3] = b.aff_freed; sa.out[3] = b.aff_free_off;
        hipLaunchKernelGGL(k_scan_small<4>, dim3(1), dim3(1024), 0, s, sa, &sc->n_aff);
        MergeArgs A;
        A.pool = h.pool; A.dir = src; A.sc = sc; A.free_stack = h.free_stack; A.aff_list = b.aff_list;
        A.jlo = b.aff_jlo; A.jhi = b.aff_jhi; A.nn = b.aff_nn; A.nn_off = b.aff_nn_off; A.parts = b.aff_parts;
        A.parts_off = b.aff_parts_off; A.extra_off = b.aff_extra_off;
        A.pb = b.pb; A.ib = b.ib; A.pe = b.pe; A.ie = b.ie; A.need_e = b.need_e; A.vb = b.vb;
        A.cb = b.cb; A.ce = b.ce; A.ne = b.ne; A.ne_ins = b.ne_ins;
        A.desc_page = b.desc_page; A.desc_cnt = b.desc_cnt; A.desc_max = b.desc_max; A.desc_fhi = b.desc_fhi;
        A.desc_flo = b.desc_flo; A.desc_fmeta = b.desc_fmeta; A.desc_ftail = b.desc_ftail;
        A.arena = h.tail_arena; A.arena_cap = h.tail_cap; A.now = now;
        hipLaunchKernelGGL(k_page_merge, dim3(GRID_PAGES), dim3(256), 0, s, A);
    }
    DescArrays da{b.desc_page, b.desc_cnt, b.desc_max, b.desc_fhi, b.desc_flo, b.desc_fmeta, b.desc_ftail};
    hipLaunchKernelGGL(k_dir_rebuild, dim3(cdiv(h.cap_dir, 256)), dim3(256), 0, s, src, dst, sc, da, b.aff_list,
                       b.aff_parts, b.aff_parts_off, b.aff_freed, b.aff_free_off, b.aff_extra_off, h.free_stack);
    hipLaunchKernelGGL(k_dir_commit, dim3(1), dim3(1), 0, s, sc, b.aff_parts_off, b.aff_extra_off, b.aff_free_off);
    launch_dir_finish(h, cur ^ 1, sc, b, s);
}

// ------------------------------------------------------------ compaction ----
// removeBefore over the window driven by ConflictBatch::detectConflicts
// (SkipList.cpp:1198-1206, 665-702).  The window
// is the global index range [g0, g1) starting at the first boundary >=
// removalKey, budget 3*|combined|+10.  Node g is dropped iff g > g0 and both
// its version and the version of node g-1 (original values) are < oldest.
// removalKey becomes the key at g1, or "" at the end.  Survivors of the pages
// covering the window are repacked into fresh pages at FILL density.
struct WinState {
    int64_t g0, g1;
    int32_t pA, pB, np;
};

__global__ __launch_bounds__(256) void k_win_setup(Pool pool, Dir dir, Scalars* sc, uint64_t* rk_hi, uint64_t* rk_lo,
                                                   uint32_t* rk_meta, uint8_t* rk_tail, int32_t* win_np) {
    __shared__ Key nk;
    __shared__ int has_key;
    if (threadIdx.x == 0) {
        const int D = sc->D;
        const int64_t H = dir.start[D];
        int64_t g0 = 0, g1 = 0;
        int pA = 1, pB = 0;
        has_key = 0;
        if (!sc->err) {
            const Key rk{rk_hi[0], rk_lo[0], rk_meta[0], rk_tail};
            const int p0 = dir_search(dir, D, rk, 1);
            const int i0 = page_lb(pool, dir.page[p0], 0, dir.cnt[p0], rk);
            g0 = dir.start[p0] + i0;
            if (g0 < H) {
                const int64_t budget = 3 * (int64_t)sc->n_comb + 10;
                g1 = min(H, g0 + budget);
                pA = i0 < dir.cnt[p0] ? p0 : p0 + 1;
                int lo = 0, hi = D;  // last q with start[q] <= g1 - 1
                while (lo < hi) {
                    int mid = (lo + hi) >> 1;
                    if (dir.start[mid] <= g1 - 1) lo = mid + 1; else hi = mid;
                }
                pB = lo - 1;
                if (g1 < H) {
                    lo = 0; hi = D;
                    while (lo < hi) {
                        int mid = (lo + hi) >> 1;
                        if (dir.start[mid] <= g1) lo = mid + 1; else hi = mid;
                    }
                    const int q1 = lo - 1;
                    nk = pool_key(pool, (int64_t)dir.page[q1] * PAGE + (g1 - dir.start[q1]));
                    has_key = 1;
                }
            } else {
                g0 = g1 = H;
            }
        }
        sc->win_g0 = g0;
        sc->win_g1 = g1;
        sc->win_pA = pA;
        sc->win_pB = pB;
        *win_np = pB - pA + 1 > 0 ? pB - pA + 1 : 0;
    }
    __syncthreads();
    if (sc->err) return;
    if (threadIdx.x == 0) {
        rk_hi[0] = has_key ? nk.hi : 0;
        rk_lo[0] = has_key ? nk.lo : 0;
        rk_meta[0] = has_key ? nk.meta : 0;
    }
    if (has_key && key_len(nk.meta) > 17) {
        const uint32_t words = (key_len(nk.meta) - 17 + 7) / 8;
        const uint64_t* s = reinterpret_cast<const uint64_t*>(nk.tail);
        uint64_t* d = reinterpret_cast<uint64_t*>(rk_tail);
        for (uint32_t w = threadIdx.x; w < words; w += blockDim.x) d[w] = s[w];
    }
}

__global__ __launch_bounds__(256) void k_win_keep(Pool pool, Dir dir, const Scalars* sc, int64_t oldest,
                                                  uint8_t* __restrict__ keep_o, int32_t* __restrict__ cnt_o) {
    __shared__ int32_t tmp[256 / 64 + 1];
    const int64_t g0 = sc->win_g0, g1 = sc->win_g1;
    const int pA = sc->win_pA, pB = sc->win_pB;
    for (int w = blockIdx.x; w <= pB - pA; w += gridDim.x) {
        const int q = pA + w;
        const int pg = dir.page[q], c = dir.cnt[q];
        const int64_t st = dir.start[q];
        const int i = threadIdx.x;
        int keep = 0;
        if (i < c) {
            keep = 1;
            const int64_t g = st + i;
            if (g > g0 && g < g1) {
                const bool above = pool.ver[(int64_t)pg * PAGE + i] >= oldest;
                const int64_t pv = i > 0 ? pool.ver[(int64_t)pg * PAGE + i - 1]
                                         : pool.ver[(int64_t)dir.page[q - 1] * PAGE + dir.cnt[q - 1] - 1];
                keep = above || pv >= oldest;
            }
            keep_o[(int64_t)w * PAGE + i] = (uint8_t)keep;
        }
        const int tot = block_reduce_sum(keep, tmp);
        if (threadIdx.x == 0) cnt_o[w] = tot;
    }
}

__global__ __launch_bounds__(256) void k_win_repack(Pool pool, Dir dir, const Scalars* sc,
                                                    const uint8_t* __restrict__ keep, const int32_t* __restrict__ off,
                                                    const int32_t* win_np, const int32_t* __restrict__ free_stack) {
    __shared__ int32_t tmp[256 / 64 + 1];
    const int np = *win_np;
    const int pA = sc->win_pA;
    const int top0 = sc->free_top;
    const int S = off[np];
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    const int per = k > 0 ? cdiv(S, k) : 1;
    for (int w = blockIdx.x; w < np; w += gridDim.x) {
        const int q = pA + w;
        const int pg = dir.page[q], c = dir.cnt[q];
        const int i = threadIdx.x;
        const int kp = i < c ? keep[(int64_t)w * PAGE + i] : 0;
        int tot;
        const int ex = block_excl_scan(kp, tmp, tot);
        if (kp) {
            const int m = off[w] + ex;
            const int part = m / per;
            const int64_t d = (int64_t)free_stack[top0 - 1 - part] * PAGE + (m - part * per);
            const int64_t sidx = (int64_t)pg * PAGE + i;
            pool.hi[d] = pool.hi[sidx]; pool.lo[d] = pool.lo[sidx]; pool.meta[d] = pool.meta[sidx];
            pool.ver[d] = pool.ver[sidx]; pool.tail[d] = pool.tail[sidx];
        }
    }
}

__global__ __launch_bounds__(256) void k_win_desc(Pool pool, const int32_t* __restrict__ off, const int32_t* win_np,
                                                  const Scalars* sc, const int32_t* __restrict__ free_stack,
                                                  int32_t* desc_page, int32_t* desc_cnt, int64_t* desc_max,
                                                  uint64_t* desc_fhi, uint64_t* desc_flo, uint32_t* desc_fmeta,
                                                  const uint8_t** desc_ftail) {
    const int np = *win_np;
    const int S = off[np];
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    const int per = k > 0 ? cdiv(S, k) : 1;
    const int top0 = sc->free_top;
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= k) return;
    const int c = min(per, S - q * per);
    const int pg = free_stack[top0 - 1 - q];
    const int64_t b = (int64_t)pg * PAGE;
    int64_t mx = INT64_MIN;
    for (int i = 0; i < c; i++) mx = max(mx, pool.ver[b + i]);
    desc_page[q] = pg; desc_cnt[q] = c; desc_max[q] = mx;
    desc_fhi[q] = pool.hi[b]; desc_flo[q] = pool.lo[b]; desc_fmeta[q] = pool.meta[b]; desc_ftail[q] = pool.tail[b];
}

__global__ __launch_bounds__(256) void k_win_dir(Dir src, Dir dst, const Scalars* sc, DescArrays desc,
                                                 const int32_t* __restrict__ off, const int32_t* win_np,
                                                 int32_t* free_stack) {
    const int np = *win_np;
    const int S = off[np];
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    const int D = sc->D, pA = sc->win_pA;
    const int Dn = D - np + k;
    const int y = blockIdx.x * blockDim.x + threadIdx.x;
    if (y < Dn) {
        if (np == 0 || y < pA) dir_copy(src, y, dst, y);
        else if (y < pA + k) desc_copy(desc, y - pA, dst, y);
        else dir_copy(src, y - k + np, dst, y);
    }
    if (y < np) free_stack[sc->free_top - k + y] = src.page[pA + y];
}

__global__ void k_win_commit(Scalars* sc, const int32_t* off, const int32_t* win_np) {
    const int np = *win_np;
    const int S = off[np];
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    sc->D = sc->D - np + k;
    sc->free_top = sc->free_top - k + np;
    sc->win_newpages = k;
    sc->win_surv = S;
}

void launch_compact(BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t oldest, hipStream_t s) {
    Dir& src = h.dir[cur];
    Dir& dst = h.dir[cur ^ 1];
    int32_t* win_np = b.win_off + b.win_cap_pages + 1;  // scalar slot after the offsets
    hipLaunchKernelGGL(k_win_setup, dim3(1), dim3(256), 0, s, h.pool, src, sc, h.rk_hi, h.rk_lo, h.rk_meta,
                       h.rk_tail, win_np);
    hipLaunchKernelGGL(k_win_keep, dim3(GRID_PAGES), dim3(256), 0, s, h.pool, src, sc, oldest, b.win_keep,
                       b.win_cnt);
    ScanArgs<1> sa;
    sa.in[0] = b.win_cnt;
    sa.out[0] = b.win_off;
    hipLaunchKernelGGL(k_scan_small<1>, dim3(1), dim3(1024), 0, s, sa, win_np);
    hipLaunchKernelGGL(k_win_repack, dim3(GRID_PAGES), dim3(256), 0, s, h.pool, src, sc, b.win_keep, b.win_off,
                       win_np, h.free_stack);
    hipLaunchKernelGGL(k_win_desc, dim3(cdiv(b.win_cap_pages, 256)), dim3(256), 0, s, h.pool, b.win_off, win_np, sc,
                       h.free_stack, b.desc_page, b.desc_cnt, b.desc_max, b.desc_fhi, b.desc_flo, b.desc_fmeta,
                       b.desc_ftail);
    DescArrays da{b.desc_page, b.desc_cnt, b.desc_max, b.desc_fhi, b.desc_flo, b.desc_fmeta, b.desc_ftail};
    hipLaunchKernelGGL(k_win_dir, dim3(cdiv(h.cap_dir, 256)), dim3(256), 0, s, src, dst, sc, da, b.win_off, win_np,
                       h.free_stack);
    hipLaunchKernelGGL(k_win_commit, dim3(1), dim3(1), 0, s, sc, b.win_off, win_np);
    launch_dir_finish(h, cur ^ 1, sc, b, s);
}

// ------------------------------------------------------------------ reset ----
__global__ __launch_bounds__(256) void k_reset(Dir d, int32_t* free_stack, int cap_pages, Scalars* sc) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < cap_pages - 1) free_stack[i] = cap_pages - 1 - i;  // pops yield page 1, 2, ...
    if (i == 0) {
        d.page[0] = 0; d.cnt[0] = 0; d.maxv[0] = INT64_MIN; d.start[0] = 0; d.start[1] = 0;
        d.fhi[0] = 0; d.flo[0] = 0; d.fmeta[0] = 0; d.ftail[0] = nullptr; d.bmax[0] = INT64_MIN;
        sc->D = 1;
        sc->free_top = cap_pages - 1;
        sc->H = 0;
        sc->tail_used = 0;
        sc->err = 0;
    }
}

void launch_reset_history(HistBufs& h, int cur, Scalars* sc, hipStream_t s) {
    hipLaunchKernelGGL(k_reset, dim3(cdiv(h.cap_pages, 256)), dim3(256), 0, s, h.dir[cur], h.free_stack,
                       h.cap_pages, sc);
}

}  // namespace fdbcs_dev

namespace fdbcs_dev {

// --------------------------------------------------------- dump / growth ----
__global__ __launch_bounds__(256) void k_gather(Pool pool, Dir dir, const Scalars* sc, Pool out) {
    const int D = sc->D;
    for (int x = blockIdx.x; x < D; x += gridDim.x) {
        const int c = dir.cnt[x];
        const int64_t b = (int64_t)dir.page[x] * PAGE, o = dir.start[x];
        for (int i = threadIdx.x; i < c; i += blockDim.x) {
            out.hi[o + i] = pool.hi[b + i];
            out.lo[o + i] = pool.lo[b + i];
            out.meta[o + i] = pool.meta[b + i];
            out.ver[o + i] = pool.ver[b + i];
            out.tail[o + i] = pool.tail[b + i];
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
                                                  uint64_t old_cap, const uint8_t* new_base) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint8_t* t = p[i];
    if (t >= old_base && t < old_base + old_cap) p[i] = new_base + (t - old_base);
}

void launch_relocate_tails(HistBufs& h, const uint8_t* old_base, uint64_t old_cap, const uint8_t* new_base,
                           hipStream_t s) {
    const int64_t n = (int64_t)h.cap_pages * PAGE;
    hipLaunchKernelGGL(k_relocate, dim3(cdiv(n, 256)), dim3(256), 0, s, h.pool.tail, n, old_base, old_cap, new_base);
    for (int d = 0; d < 2; d++)
        hipLaunchKernelGGL(k_relocate, dim3(cdiv(h.cap_dir, 256)), dim3(256), 0, s, h.dir[d].ftail,
                           (int64_t)h.cap_dir, old_base, old_cap, new_base);
}

}  // namespace fdbcs_dev
