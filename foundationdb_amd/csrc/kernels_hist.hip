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
// Launches per batch: merge = bounds, aff_build, aff_plan, scan, page_merge,
// dir_rebuild, bmax_commit; compaction = win_setup, win_keep, scan,
// win_repack, win_dir, bmax_commit.  Directory `start[]` (global index of a
// page's first boundary) is carried forward incrementally, never rescanned.
#include <algorithm>
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
// Per combined range j: where b and e fall in the pre-batch history, whether
// e needs a node, and the value it keeps.
__global__ __launch_bounds__(256) void k_bounds(IndirectKeys cb, IndirectKeys ce, Pool pool, Dir dir, Scalars* sc,
                                                int64_t v0, int32_t* __restrict__ pb_o, int32_t* __restrict__ ib_o,
                                                int32_t* __restrict__ pe_o, int32_t* __restrict__ ie_o,
                                                uint8_t* __restrict__ need_o, int64_t* __restrict__ vb_o) {
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
}

// The affected pages are the union of the intervals [pb_j, pe_j], which are
// nondecreasing in j; range j contributes the pages after the previous
// range's pe.  One workgroup: a scan over the contributions.  aff_jlo[a] = the
// first range touching page a (the contributing one).
__global__ __launch_bounds__(1024) void k_aff_build(const int32_t* __restrict__ pb, const int32_t* __restrict__ pe,
                                                    Scalars* sc, int32_t* __restrict__ aff_list,
                                                    int32_t* __restrict__ aff_jlo) {
    __shared__ int32_t s_pb[4096], s_pe[4097];
    __shared__ int32_t tmp[1024 / 64 + 1];
    const int nC = sc->err ? 0 : sc->n_comb;
    const int tid = threadIdx.x;
    int carry = 0;
    for (int base = 0; base < nC; base += 4096) {
        const int n = min(4096, nC - base);
        // s_pe[0] = pe of the range before the tile (or -1)
        if (tid == 0) s_pe[0] = base > 0 ? pe[base - 1] : -1;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = j * 1024 + tid;
            if (i < n) {
                s_pb[i] = pb[base + i];
                s_pe[i + 1] = pe[base + i];
            }
        }
        __syncthreads();
        int s = 0;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = tid * 4 + j;
            if (i < n) s += max(0, s_pe[i + 1] - max(s_pb[i], s_pe[i] + 1) + 1);
        }
        int tot;
        int pos = carry + block_excl_scan(s, tmp, tot);
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = tid * 4 + j;
            if (i < n) {
                for (int p = max(s_pb[i], s_pe[i] + 1); p <= s_pe[i + 1]; p++) {
                    aff_list[pos] = p;
                    aff_jlo[pos] = base + i;
                    pos++;
                }
            }
        }
        carry += tot;
        __syncthreads();
    }
    if (tid == 0) sc->n_aff = carry;
}

// One wavefront per affected page: the last range touching it, surviving old
// entries, new entries landing in it, and how many output pages it becomes.
__global__ __launch_bounds__(256) void k_aff_plan(Dir dir, const Scalars* sc, const int32_t* __restrict__ aff_list,
                                                  const int32_t* __restrict__ pb, const int32_t* __restrict__ ib,
                                                  const int32_t* __restrict__ pe, const int32_t* __restrict__ ie,
                                                  const uint8_t* __restrict__ need_e, const int32_t* __restrict__ jlo_i,
                                                  int32_t* __restrict__ jhi_o, int32_t* __restrict__ nn_o,
                                                  int32_t* __restrict__ parts_o, int32_t* __restrict__ extra_o,
                                                  int32_t* __restrict__ freed_o, int32_t* __restrict__ delta_o) {
    const int naff = sc->err ? 0 : sc->n_aff, nC = sc->n_comb;
    const int lane = threadIdx.x & 63;
    const int wpb = blockDim.x >> 6;
    for (int a = blockIdx.x * wpb + (threadIdx.x >> 6); a < naff; a += gridDim.x * wpb) {
        const int p = aff_list[a], cntp = dir.cnt[p];
        const int jlo = jlo_i[a];
        int lo = jlo, hi = nC;  // last j with pb[j] <= p
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (pb[mid] <= p) lo = mid + 1; else hi = mid;
        }
        const int jhi = lo - 1;
        int erased = 0, nn = 0;
        for (int j = jlo + lane; j <= jhi; j += 64) {
            const int s = pb[j] < p ? 0 : ib[j];
            const int en = pe[j] > p ? cntp : ie[j];
            erased += max(0, en - s);
            nn += (pb[j] == p) + (pe[j] == p && need_e[j]);
        }
        erased = wave_reduce_sum(erased);
        nn = wave_reduce_sum(nn);
        if (lane == 0) {
            const int nout = cntp - erased + nn;
            const int parts = nout == 0 ? 0 : (nout <= PAGE ? 1 : cdiv(nout, FILL));
            jhi_o[a] = jhi;
            nn_o[a] = nn;
            parts_o[a] = parts;
            extra_o[a] = parts > 1 ? parts - 1 : 0;
            freed_o[a] = parts == 0;
            delta_o[a] = nout - cntp;
        }
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

struct DescArrays {
    int32_t* page;
    int32_t* cnt;
    int64_t* maxv;
    uint64_t* fhi;
    uint64_t* flo;
    uint32_t* fmeta;
    const uint8_t** ftail;
};

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
    IndirectKeys cb, ce;
    Pool ne;
    int32_t* ne_ins;
    DescArrays desc;
    uint8_t* arena;
    uint64_t arena_cap;
    int64_t now;
};

__device__ inline void put_entry(const Pool& pool, int64_t d, uint64_t hi, uint64_t lo, uint32_t meta, int64_t ver,
                                 const uint8_t* tail) {
    pool.hi[d] = hi; pool.lo[d] = lo; pool.meta[d] = meta; pool.ver[d] = ver; pool.tail[d] = tail;
}

__device__ inline void put_desc(const DescArrays& D, int x, int page, int cnt, uint64_t hi, uint64_t lo,
                                uint32_t meta, const uint8_t* tail) {
    D.page[x] = page; D.cnt[x] = cnt; D.fhi[x] = hi; D.flo[x] = lo; D.fmeta[x] = meta; D.ftail[x] = tail;
}

// One workgroup per affected page: load it into LDS, drop erased entries,
// merge in the new boundaries, write 0..k output pages (the first in place,
// the others from the free stack) and their directory descriptors.  Part
// maxima come from LDS atomics as the entries are written.
//
// Fast path (<= JCAP combined ranges touch the page -- the common case): the
// ranges' insertion plan and the page's new entries are staged in LDS, so a
// page costs ~3 dependent global round trips.  Otherwise the new entries go
// through the global scratch list (A.ne) and the plan is read from global.
static constexpr int JCAP = 64;

struct MergeShared {
    uint64_t o_hi[PAGE], o_lo[PAGE];
    int64_t o_ver[PAGE];
    const uint8_t* o_tail[PAGE];
    uint32_t o_meta[PAGE];
    int32_t kb[PAGE + 1];
    long long pmax[MAXP];
    int32_t tmp[256 / 64 + 1];
    int32_t j_pb[JCAP], j_ib[JCAP], j_pe[JCAP], j_ie[JCAP];
    int64_t j_vb[JCAP];
    uint8_t j_need[JCAP];
    uint64_t n_hi[2 * JCAP], n_lo[2 * JCAP];
    int64_t n_ver[2 * JCAP];
    const uint8_t* n_tail[2 * JCAP];
    uint32_t n_meta[2 * JCAP];
    int32_t n_ins[2 * JCAP];
};

template <bool FAST>
__device__ void merge_page(const MergeArgs& A, MergeShared& S, int a, int top0) {
    Scalars* sc = A.sc;
    const int tid = threadIdx.x;
    const int p = A.aff_list[a];
    const int pg = A.dir.page[p], cntp = A.dir.cnt[p];
    const int jlo = A.jlo[a], jhi = A.jhi[a];
    const int nj = jhi - jlo + 1;
    const int nn = A.nn[a], nn_off = A.nn_off[a];
    const int parts = A.parts[a];
    const int xoff = A.extra_off[a];
    const int doff = A.parts_off[a];
    const int64_t pbase = (int64_t)pg * PAGE;
    if (tid < cntp) {
        S.o_hi[tid] = A.pool.hi[pbase + tid];
        S.o_lo[tid] = A.pool.lo[pbase + tid];
        S.o_meta[tid] = A.pool.meta[pbase + tid];
        S.o_ver[tid] = A.pool.ver[pbase + tid];
        S.o_tail[tid] = A.pool.tail[pbase + tid];
    }
    if (tid < MAXP) S.pmax[tid] = INT64_MIN;
    if (FAST && tid < nj) {
        const int j = jlo + tid;
        S.j_pb[tid] = A.pb[j];
        S.j_ib[tid] = A.ib[j];
        S.j_pe[tid] = A.pe[j];
        S.j_ie[tid] = A.ie[j];
        S.j_need[tid] = A.need_e[j];
        S.j_vb[tid] = A.vb[j];
    }
    if (FAST) __syncthreads();
    auto PB = [&](int j) { return FAST ? S.j_pb[j - jlo] : A.pb[j]; };
    auto IB = [&](int j) { return FAST ? S.j_ib[j - jlo] : A.ib[j]; };
    auto PE = [&](int j) { return FAST ? S.j_pe[j - jlo] : A.pe[j]; };
    auto IE = [&](int j) { return FAST ? S.j_ie[j - jlo] : A.ie[j]; };
    auto NEED = [&](int j) { return FAST ? S.j_need[j - jlo] : A.need_e[j]; };
    auto VB = [&](int j) { return FAST ? S.j_vb[j - jlo] : A.vb[j]; };
    // erased iff inside [(pb_j, ib_j), (pe_j, ie_j)) for the last j starting at or before (p, tid)
    int keep = 0;
    if (tid < cntp) {
        int lo = jlo, hi = jhi + 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (pos_le(PB(mid), IB(mid), p, tid)) lo = mid + 1; else hi = mid;
        }
        const int j = lo - 1;
        keep = !(j >= jlo && pos_lt(p, tid, PE(j), IE(j)));
    }
    int kept;
    const int kex = block_excl_scan(keep, S.tmp, kept);
    if (tid < cntp) S.kb[tid] = kex;
    if (tid == 0) S.kb[cntp] = kept;
    // new entries landing here, in key order: b_j (version now), then e_j
    uint64_t* NHI = FAST ? S.n_hi : A.ne.hi + nn_off;
    uint64_t* NLO = FAST ? S.n_lo : A.ne.lo + nn_off;
    uint32_t* NMETA = FAST ? S.n_meta : A.ne.meta + nn_off;
    int64_t* NVER = FAST ? S.n_ver : A.ne.ver + nn_off;
    const uint8_t** NTAIL = FAST ? S.n_tail : A.ne.tail + nn_off;
    int32_t* NINS = FAST ? S.n_ins : A.ne_ins + nn_off;
    int local = 0;
    for (int jb = jlo; jb <= jhi; jb += blockDim.x) {
        const int j = jb + tid;
        const bool eb = j <= jhi && PB(j) == p;
        const bool ee = j <= jhi && PE(j) == p && NEED(j);
        int t2;
        int k = local + block_excl_scan((int)eb + (int)ee, S.tmp, t2);
        if (eb) {
            const Key kk = A.cb.get(j);
            NHI[k] = kk.hi; NLO[k] = kk.lo; NMETA[k] = kk.meta; NVER[k] = A.now;
            copy_tail(kk, A.arena, A.arena_cap, sc, &NTAIL[k]);
            NINS[k] = IB(j);
            k++;
        }
        if (ee) {
            const Key kk = A.ce.get(j);
            NHI[k] = kk.hi; NLO[k] = kk.lo; NMETA[k] = kk.meta; NVER[k] = VB(j);
            copy_tail(kk, A.arena, A.arena_cap, sc, &NTAIL[k]);
            NINS[k] = IE(j);
        }
        local += t2;
    }
    __threadfence_block();
    __syncthreads();
    const int nout = kept + nn;
    const int per = parts > 0 ? cdiv(nout, parts) : 1;
    auto dest = [&](int q) -> int { return q == 0 ? pg : A.free_stack[top0 - 1 - (xoff + q - 1)]; };
    if (tid < cntp && keep) {
        int lo = 0, hi = nn;  // new entries that go before old entry tid
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (NINS[mid] <= tid) lo = mid + 1; else hi = mid;
        }
        const int m = S.kb[tid] + lo;
        const int q = m / per, slot = m - q * per;
        const int dp = dest(q);
        put_entry(A.pool, (int64_t)dp * PAGE + slot, S.o_hi[tid], S.o_lo[tid], S.o_meta[tid], S.o_ver[tid],
                  S.o_tail[tid]);
        if (q < MAXP) atomicMax(&S.pmax[q], (long long)S.o_ver[tid]);
        if (slot == 0)
            put_desc(A.desc, doff + q, dp, min(per, nout - q * per), S.o_hi[tid], S.o_lo[tid], S.o_meta[tid],
                     S.o_tail[tid]);
    }
    for (int k = tid; k < nn; k += blockDim.x) {
        const int m = k + S.kb[NINS[k]];
        const int q = m / per, slot = m - q * per;
        const int dp = dest(q);
        const uint64_t hi = NHI[k], lo = NLO[k];
        const uint32_t meta = NMETA[k];
        const int64_t ver = NVER[k];
        const uint8_t* tail = NTAIL[k];
        put_entry(A.pool, (int64_t)dp * PAGE + slot, hi, lo, meta, ver, tail);
        if (q < MAXP) atomicMax(&S.pmax[q], (long long)ver);
        if (slot == 0) put_desc(A.desc, doff + q, dp, min(per, nout - q * per), hi, lo, meta, tail);
    }
    __threadfence_block();
    __syncthreads();
    for (int q = tid; q < parts; q += blockDim.x) {
        int64_t mx;
        if (q < MAXP) {
            mx = S.pmax[q];
        } else {  // very large outputs (e.g. a first batch into an empty history)
            const int64_t bq = (int64_t)dest(q) * PAGE;
            const int c = min(per, nout - q * per);
            mx = INT64_MIN;
            for (int i = 0; i < c; i++) mx = max(mx, A.pool.ver[bq + i]);
        }
        A.desc.maxv[doff + q] = mx;
    }
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_page_merge(MergeArgs A) {
    __shared__ MergeShared S;
    Scalars* sc = A.sc;
    if (sc->err) return;
    const int naff = sc->n_aff;
    const int top0 = sc->free_top;
    for (int a = blockIdx.x; a < naff; a += gridDim.x) {
        if (A.jhi[a] - A.jlo[a] + 1 <= JCAP) merge_page<true>(A, S, a, top0);
        else merge_page<false>(A, S, a, top0);
    }
}

__device__ inline void dir_copy(const Dir& s, int x, const Dir& d, int y) {
    d.page[y] = s.page[x]; d.cnt[y] = s.cnt[x]; d.maxv[y] = s.maxv[x];
    d.fhi[y] = s.fhi[x]; d.flo[y] = s.flo[x]; d.fmeta[y] = s.fmeta[x]; d.ftail[y] = s.ftail[x];
}

__device__ inline void desc_copy(const DescArrays& s, int x, const Dir& d, int y) {
    d.page[y] = s.page[x]; d.cnt[y] = s.cnt[x]; d.maxv[y] = s.maxv[x];
    d.fhi[y] = s.fhi[x]; d.flo[y] = s.flo[x]; d.fmeta[y] = s.fmeta[x]; d.ftail[y] = s.ftail[x];
}

struct RebuildArgs {
    Dir src, dst;
    Scalars* sc;
    DescArrays desc;
    const int32_t *aff_list, *parts, *parts_off, *freed, *free_off, *extra_off, *delta_off;
    int32_t* free_stack;
};

// Directory after the merge: unaffected entries move by the number of extra
// pages inserted before them; affected entries are replaced by their parts.
// start[] moves by the boundary-count change of the affected pages before.
__global__ __launch_bounds__(256) void k_dir_rebuild(RebuildArgs A) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    const Scalars* sc = A.sc;
    const int D = sc->D;
    const int naff = sc->err ? 0 : sc->n_aff;
    const int Dn = naff ? D - naff + A.parts_off[naff] : D;
    if (x == 0) {
        A.sc->D_next = Dn;
        A.sc->free_next = naff ? sc->free_top - A.extra_off[naff] + A.free_off[naff] : sc->free_top;
        A.dst.start[Dn] = A.src.start[D] + (naff ? A.delta_off[naff] : 0);
    }
    if (x >= D) return;
    if (naff == 0) {
        dir_copy(A.src, x, A.dst, x);
        A.dst.start[x] = A.src.start[x];
        return;
    }
    int lo = 0, hi = naff;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (A.aff_list[mid] < x) lo = mid + 1; else hi = mid;
    }
    const int na = lo;
    const int base = x - na + A.parts_off[na];
    const int64_t st = A.src.start[x] + A.delta_off[na];
    if (na < naff && A.aff_list[na] == x) {
        const int np = A.parts[na], off = A.parts_off[na];
        int64_t s = st;
        for (int q = 0; q < np; q++) {
            desc_copy(A.desc, off + q, A.dst, base + q);
            A.dst.start[base + q] = s;
            s += A.desc.cnt[off + q];
        }
        if (A.freed[na]) A.free_stack[sc->free_top - A.extra_off[naff] + A.free_off[na]] = A.src.page[x];
    } else {
        dir_copy(A.src, x, A.dst, base);
        A.dst.start[base] = st;
    }
}

// Per-64-entry maxima of the new directory (one wavefront per group), then
// commit the directory size, free-stack top and history size.
__global__ __launch_bounds__(256) void k_bmax_commit(Dir d, Scalars* sc) {
    const int Dn = sc->D_next;
    const int lane = threadIdx.x & 63;
    const int g = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    if (g * 64 < Dn) {
        const int x = g * 64 + lane;
        int64_t m = x < Dn ? d.maxv[x] : INT64_MIN;
        m = wave_reduce_max(m);
        if (lane == 0) d.bmax[g] = m;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        sc->D = Dn;
        sc->free_top = sc->free_next;
        sc->H = d.start[Dn];
    }
}

static void launch_bmax_commit(HistBufs& h, int which, Scalars* sc, hipStream_t s) {
    const int groups = cdiv(h.cap_dir, 64);
    hipLaunchKernelGGL(k_bmax_commit, dim3(cdiv(groups, 4)), dim3(256), 0, s, h.dir[which], sc);
}

void launch_dir_finish(HistBufs& h, int cur, Scalars* sc, BatchBufs& b, hipStream_t s) {
    // full recompute of start[] (used after reset / load)
    Dir& d = h.dir[cur];
    scan_i64_from_i32(d.cnt, d.start, &sc->D, 0, &sc->H, b.scan_tmp, s);
    hipMemcpyAsync(&sc->D_next, &sc->D, sizeof(int32_t), hipMemcpyDeviceToDevice, s);
    hipMemcpyAsync(&sc->free_next, &sc->free_top, sizeof(int32_t), hipMemcpyDeviceToDevice, s);
    launch_bmax_commit(h, cur, sc, s);
}

void launch_merge(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t now,
                  int64_t v0, hipStream_t s) {
    const int W = v.write_count;
    Dir& src = h.dir[cur];
    Dir& dst = h.dir[cur ^ 1];
    if (W > 0) {
        const IndirectKeys cbk{b.keys, b.cb_slot}, cek{b.keys, b.ce_slot};
        hipLaunchKernelGGL(k_bounds, dim3(cdiv(W, 256)), dim3(256), 0, s, cbk, cek, h.pool, src, sc, v0, b.pb,
                           b.ib, b.pe, b.ie, b.need_e, b.vb);
    }
    hipLaunchKernelGGL(k_aff_build, dim3(1), dim3(1024), 0, s, b.pb, b.pe, sc, b.aff_list, b.aff_jlo);
    if (W > 0) {
        const int max_aff = std::min<int64_t>(h.cap_dir, 4 * (int64_t)W + 4);
        hipLaunchKernelGGL(k_aff_plan, dim3(std::max(1, std::min(GRID_PAGES, cdiv(max_aff, 4)))), dim3(256), 0, s,
                           src, sc, b.aff_list, b.pb, b.ib, b.pe, b.ie, b.need_e, b.aff_jlo, b.aff_jhi, b.aff_nn,
                           b.aff_parts, b.aff_extra, b.aff_freed, b.aff_delta);
        ScanArgs<5> sa;
        sa.in[0] = b.aff_nn; sa.out[0] = b.aff_nn_off;
        sa.in[1] = b.aff_parts; sa.out[1] = b.aff_parts_off;
        sa.in[2] = b.aff_extra; sa.out[2] = b.aff_extra_off;
        sa.in[3] = b.aff_freed; sa.out[3] = b.aff_free_off;
        sa.in[4] = b.aff_delta; sa.out[4] = b.aff_delta_off;
        hipLaunchKernelGGL(k_scan_small<5>, dim3(1), dim3(1024), 0, s, sa, &sc->n_aff);
        MergeArgs A;
        A.pool = h.pool; A.dir = src; A.sc = sc; A.free_stack = h.free_stack; A.aff_list = b.aff_list;
        A.jlo = b.aff_jlo; A.jhi = b.aff_jhi; A.nn = b.aff_nn; A.nn_off = b.aff_nn_off; A.parts = b.aff_parts;
        A.parts_off = b.aff_parts_off; A.extra_off = b.aff_extra_off;
        A.pb = b.pb; A.ib = b.ib; A.pe = b.pe; A.ie = b.ie; A.need_e = b.need_e; A.vb = b.vb;
        A.cb = IndirectKeys{b.keys, b.cb_slot}; A.ce = IndirectKeys{b.keys, b.ce_slot}; A.ne = b.ne; A.ne_ins = b.ne_ins;
        A.desc = DescArrays{b.desc_page, b.desc_cnt, b.desc_max, b.desc_fhi, b.desc_flo, b.desc_fmeta, b.desc_ftail};
        A.arena = h.tail_arena; A.arena_cap = h.tail_cap; A.now = now;
        hipLaunchKernelGGL(k_page_merge, dim3(std::max(1, std::min(GRID_PAGES, max_aff))), dim3(256), 0, s, A);
    }
    RebuildArgs R;
    R.src = src; R.dst = dst; R.sc = sc;
    R.desc = DescArrays{b.desc_page, b.desc_cnt, b.desc_max, b.desc_fhi, b.desc_flo, b.desc_fmeta, b.desc_ftail};
    R.aff_list = b.aff_list; R.parts = b.aff_parts; R.parts_off = b.aff_parts_off; R.freed = b.aff_freed;
    R.free_off = b.aff_free_off; R.extra_off = b.aff_extra_off; R.delta_off = b.aff_delta_off;
    R.free_stack = h.free_stack;
    hipLaunchKernelGGL(k_dir_rebuild, dim3(cdiv(h.cap_dir, 256)), dim3(256), 0, s, R);
    launch_bmax_commit(h, cur ^ 1, sc, s);
}

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

__global__ __launch_bounds__(64) void k_win_setup(Pool pool, Dir dir, Scalars* sc, uint64_t* rk_hi, uint64_t* rk_lo,
                                                  uint32_t* rk_meta, uint8_t* rk_tail) {
    const int lane = threadIdx.x;
    const int D = sc->D;
    const int64_t H = dir.start[D];
    int64_t g0 = 0, g1 = 0;
    int pA = 1, pB = 0;
    bool has_key = false;
    Key nk{0, 0, 0, nullptr};
    if (!sc->err) {
        const Key rk{rk_hi[0], rk_lo[0], rk_meta[0], rk_tail};
        const int p0 = wave_dir_search(dir, D, rk);
        const int i0 = wave_page_lb(pool, dir.page[p0], dir.cnt[p0], rk);
        g0 = dir.start[p0] + i0;
        if (g0 < H) {
            const int64_t budget = 3 * (int64_t)sc->n_comb + 10;
            g1 = min(H, g0 + budget);
            pA = i0 < dir.cnt[p0] ? p0 : p0 + 1;
            pB = wave_start_search(dir.start, D, g1 - 1);
            if (g1 < H) {
                const int q1 = wave_start_search(dir.start, D, g1);
                nk = pool_key(pool, (int64_t)dir.page[q1] * PAGE + (g1 - dir.start[q1]));
                has_key = true;
            }
        } else {
            g0 = g1 = H;
        }
    }
    if (lane == 0) {
        sc->win_g0 = g0;
        sc->win_g1 = g1;
        sc->win_pA = pA;
        sc->win_pB = pB;
        sc->win_np = pB - pA + 1 > 0 ? pB - pA + 1 : 0;
        if (!sc->err) {
            rk_hi[0] = has_key ? nk.hi : 0;
            rk_lo[0] = has_key ? nk.lo : 0;
            rk_meta[0] = has_key ? nk.meta : 0;
        }
    }
    if (!sc->err && has_key && key_len(nk.meta) > 17) {
        const uint32_t words = (key_len(nk.meta) - 17 + 7) / 8;
        const uint64_t* s = reinterpret_cast<const uint64_t*>(nk.tail);
        uint64_t* d = reinterpret_cast<uint64_t*>(rk_tail);
        for (uint32_t w = lane; w < words; w += 64) d[w] = s[w];
    }
}

__global__ __launch_bounds__(256) void k_win_keep(Pool pool, Dir dir, const Scalars* sc, int64_t oldest,
                                                  uint8_t* __restrict__ keep_o, int32_t* __restrict__ cnt_o,
                                                  int64_t* __restrict__ part_max) {
    __shared__ int32_t tmp[256 / 64 + 1];
    const int64_t g0 = sc->win_g0, g1 = sc->win_g1;
    const int pA = sc->win_pA, np = sc->win_np;
    for (int w = blockIdx.x; w < np; w += gridDim.x) {
        // the repack makes at most ceil(np * PAGE / FILL) <= 2 * np pages
        if (threadIdx.x < 2) part_max[2 * w + threadIdx.x] = INT64_MIN;
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

// survivors -> fresh pages at FILL density, with their descriptors; each
// workgroup's survivors span at most 3 parts, reduced in LDS before one
// global atomic per part
__global__ __launch_bounds__(256) void k_win_repack(Pool pool, Dir dir, const Scalars* sc,
                                                    const uint8_t* __restrict__ keep, const int32_t* __restrict__ off,
                                                    const int32_t* __restrict__ free_stack, DescArrays desc) {
    __shared__ int32_t tmp[256 / 64 + 1];
    __shared__ long long lmax[4];
    const int np = sc->win_np;
    const int pA = sc->win_pA;
    const int top0 = sc->free_top;
    const int S = off[np];
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    const int per = k > 0 ? cdiv(S, k) : 1;
    for (int w = blockIdx.x; w < np; w += gridDim.x) {
        const int q = pA + w;
        const int pg = dir.page[q], c = dir.cnt[q];
        const int i = threadIdx.x;
        if (i < 4) lmax[i] = INT64_MIN;
        const int kp = i < c ? keep[(int64_t)w * PAGE + i] : 0;
        int tot;
        const int ex = block_excl_scan(kp, tmp, tot);
        const int part0 = off[w] / per;
        if (kp) {
            const int m = off[w] + ex;
            const int part = m / per, slot = m - part * per;
            const int dp = free_stack[top0 - 1 - part];
            const int64_t sidx = (int64_t)pg * PAGE + i;
            const uint64_t hi = pool.hi[sidx], lo = pool.lo[sidx];
            const uint32_t meta = pool.meta[sidx];
            const int64_t ver = pool.ver[sidx];
            const uint8_t* tail = pool.tail[sidx];
            put_entry(pool, (int64_t)dp * PAGE + slot, hi, lo, meta, ver, tail);
            atomicMax(&lmax[min(3, part - part0)], (long long)ver);
            if (slot == 0) put_desc(desc, part, dp, min(per, S - part * per), hi, lo, meta, tail);
        }
        __syncthreads();
        if (i < 4 && lmax[i] != INT64_MIN) atomicMax((long long*)&desc.maxv[part0 + i], lmax[i]);
        __syncthreads();
    }
}

__global__ __launch_bounds__(256) void k_win_dir(Dir src, Dir dst, Scalars* sc, DescArrays desc,
                                                 const int32_t* __restrict__ off, int32_t* free_stack) {
    const int np = sc->win_np;
    const int S = off[np];
    const int k = S > 0 ? cdiv(S, FILL) : 0;
    const int per = k > 0 ? cdiv(S, k) : 1;
    const int D = sc->D, pA = sc->win_pA;
    const int Dn = D - np + k;
    const int64_t removed = np ? (src.start[pA + np] - src.start[pA]) - S : 0;
    const int y = blockIdx.x * blockDim.x + threadIdx.x;
    if (y == 0) {
        sc->D_next = Dn;
        sc->free_next = sc->free_top - k + np;
        dst.start[Dn] = src.start[D] - removed;
        sc->win_newpages = k;
        sc->win_surv = S;
    }
    if (y < Dn) {
        if (np == 0 || y < pA) {
            dir_copy(src, y, dst, y);
            dst.start[y] = src.start[y];
        } else if (y < pA + k) {
            desc_copy(desc, y - pA, dst, y);
            dst.start[y] = src.start[pA] + (int64_t)(y - pA) * per;
        } else {
            dir_copy(src, y - k + np, dst, y);
            dst.start[y] = src.start[y - k + np] - removed;
        }
    }
    if (y < np) free_stack[sc->free_top - k + y] = src.page[pA + y];
}

void launch_compact(BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t oldest, hipStream_t s) {
    Dir& src = h.dir[cur];
    Dir& dst = h.dir[cur ^ 1];
    const int win_cap = b.win_cap_pages;
    hipLaunchKernelGGL(k_win_setup, dim3(1), dim3(64), 0, s, h.pool, src, sc, h.rk_hi, h.rk_lo, h.rk_meta,
                       h.rk_tail);
    hipLaunchKernelGGL(k_win_keep, dim3(std::min(GRID_PAGES, win_cap)), dim3(256), 0, s, h.pool, src, sc, oldest,
                       b.win_keep, b.win_cnt, b.desc_max);
    ScanArgs<1> sa;
    sa.in[0] = b.win_cnt;
    sa.out[0] = b.win_off;
    hipLaunchKernelGGL(k_scan_small<1>, dim3(1), dim3(1024), 0, s, sa, &sc->win_np);
    DescArrays da{b.desc_page, b.desc_cnt, b.desc_max, b.desc_fhi, b.desc_flo, b.desc_fmeta, b.desc_ftail};
    hipLaunchKernelGGL(k_win_repack, dim3(std::min(GRID_PAGES, win_cap)), dim3(256), 0, s, h.pool, src, sc,
                       b.win_keep, b.win_off, h.free_stack, da);
    hipLaunchKernelGGL(k_win_dir, dim3(cdiv(h.cap_dir, 256)), dim3(256), 0, s, src, dst, sc, da, b.win_off,
                       h.free_stack);
    launch_bmax_commit(h, cur ^ 1, sc, s);
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
