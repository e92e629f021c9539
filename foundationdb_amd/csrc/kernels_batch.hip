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
#include <cstdlib>
#include "kernels.h"
#include "devutil.h"
#include "hist_search.h"

namespace fdbcs_dev {

// Write-through (sc1) stores and loads of values handed between workgroups
// inside one launch (MI355X_MICROARCH.md, inter-workgroup visibility): the
// fused edge lanes (k_decide_rounds) and the sort-overflow flag the live
// kernel's poller watches.
template <class T>
__device__ inline void st1(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ inline T ld1(const T* p) {
    return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}


// -------------------------------------------------------------- ingest ----
// One launch, two kinds of blocks:
//   prep   (lane per txn):   addTransaction's tooOld rule (SkipList.cpp:979-1008)
//                            and the range -> txn maps;
//   encode (lane per range): both endpoints -> (hi, lo, meta, tail) records
//                            (replaces KeyInfo/getCharacter, :134-177) and the
//                            begin < end precondition.
// The per-batch scalars the encoder allocates from (err, btail_used) were
// reset by the previous batch's last kernel (k_bmax_commit, end of batch).
// 8 bytes at p (any alignment) as a little-endian word, from the aligned
// words that hold them: w0 = the word at p & ~7, w1 the next one
__device__ inline uint64_t funnel8(uint64_t w0, uint64_t w1, uint32_t sh) {
    return sh ? (w0 >> (8 * sh)) | (w1 << (64 - 8 * sh)) : w0;
}

// The fixed part of a key at p (any alignment) from up to three aligned
// 8-byte loads instead of 17 byte loads, and its tail (bytes 17..) copied a
// word at a time into the batch's tail buffer (8-byte aligned, zero padded).
// Only the aligned words that hold key bytes are read (a key can end a
// buffer), and bytes past L are masked to zero.
__device__ inline Key encode_key(const uint8_t* p, uint32_t L, uint8_t* btail, uint64_t btail_cap, Scalars* sc) {
    if (L > FDBCS_MAX_KEY) {
        atomicCAS(&sc->err, 0, FDBCS_E_KEY);
        L = FDBCS_MAX_KEY;
    }
    const uint32_t n = L < 17 ? L : 17;
    const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 7);
    const uint64_t* w = reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(7));
    const uint64_t w0 = n ? w[0] : 0, w1 = sh + n > 8 ? w[1] : 0, w2 = sh + n > 16 ? w[2] : 0;
    uint64_t hi = __builtin_bswap64(funnel8(w0, w1, sh)), lo = __builtin_bswap64(funnel8(w1, w2, sh));
    uint32_t b16 = n == 17 ? (uint32_t)((w2 >> (8 * sh)) & 0xFF) : 0;
    if (n < 8) hi = n ? hi & (~0ull << (64 - 8 * n)) : 0;  // (big-endian: byte i at bits 56-8i)
    if (n < 16) lo = n > 8 ? lo & (~0ull << (64 - 8 * (n - 8))) : 0;
    const uint8_t* tail = nullptr;
    if (L > 17) {
        const uint64_t m = L - 17, words = (m + 7) >> 3;
        const uint64_t o = atomicAdd((unsigned long long*)&sc->btail_used, (unsigned long long)(8 * words));
        if (o + 8 * words > btail_cap) {
            // the batch fails; later kernels still compare this key, so it
            // points at readable bytes (the buffer holds >= 64 KB > any tail)
            atomicCAS(&sc->err, 0, FDBCS_E_CAPACITY);
            tail = btail;
        } else {
            uint64_t* d = reinterpret_cast<uint64_t*>(btail + o);
            const uint8_t* q = p + 17;
            const uint32_t qs = (uint32_t)(reinterpret_cast<uintptr_t>(q) & 7);
            const uint64_t* qw = reinterpret_cast<const uint64_t*>(reinterpret_cast<uintptr_t>(q) & ~uintptr_t(7));
            const uint64_t qwords = (qs + m + 7) >> 3;  // aligned words holding the tail's bytes
            uint64_t cur = qw[0];
            for (uint64_t i = 0; i < words; i++) {
                const uint64_t nxt = i + 1 < qwords ? qw[i + 1] : 0;
                uint64_t x = funnel8(cur, nxt, qs);
                if (i + 1 == words && (m & 7)) x &= ~0ull >> (64 - 8 * (m & 7));  // zero padding past L
                d[i] = x;
                cur = nxt;
            }
            tail = reinterpret_cast<const uint8_t*>(d);
        }
    }
    return Key{hi, lo, (b16 << 24) | L, tail};
}

struct IngestArgs {
    int T, R, W, prep_blocks, bmax2_blocks;
    int64_t wbase;  // slot of write 0's begin (write_base: 2R, or a live batch's 2 caps.R)
    Dir hd;  // bmax2 blocks: the history directory of this batch's read check
    const int64_t* snap;
    const int32_t* ro;
    const int32_t* wo;
    const uint64_t* koff;
    const uint32_t* klen;
    const uint8_t* bytes;
    int64_t oldest;
    uint8_t* too_old;
    uint8_t* hist;
    int32_t* deg;
    int32_t* read_txn;
    int64_t* read_snap;
    int32_t* write_txn;
    KeyArrays keys;
    uint8_t* btail;
    uint64_t btail_cap;
    Scalars* sc;
    LmArgs lm;  // the attached sample's roll (per-transaction path; lm.on = 0 otherwise)
};

// A sampled range of the load-metrics roll (common.h LmArgs): its entry and
// begin key into pinned host memory, at places claimed by two counters (the
// host orders the ~200 entries of a batch by position afterwards).
// The key's bytes come from its encoding (Key: hi, lo big-endian, byte 16 in
// meta, bytes 17.. in the 8-aligned zero-padded tail), written 16 at a time.
__device__ inline void lm_append(const LmArgs& L, Scalars* sc, int64_t amt, const Key& k, uint64_t pos) {
    const uint32_t len = key_len(k.meta);
    const uint64_t padded = ((uint64_t)len + 15) & ~15ull;
    const uint32_t i = (uint32_t)atomicAdd(&sc->lm_count, 1);
    const uint64_t o = atomicAdd((unsigned long long*)&sc->lm_bytes, (unsigned long long)padded);
    if (i >= L.cap_n) return;  // (the host sees the count past the capacity and rolls the batch again)
    uint4* e = reinterpret_cast<uint4*>(L.ent + i);
    e[0] = make_uint4((uint32_t)amt, (uint32_t)((uint64_t)amt >> 32), (uint32_t)pos, len);
    e[1] = make_uint4((uint32_t)o, (uint32_t)(o >> 32), 0, 0);
    // (the empty key claims no bytes: its offset is the next key's, whose
    // bytes a store here would zero)
    if (padded == 0 || o + padded > L.cap_b) return;
    uint64_t* d = reinterpret_cast<uint64_t*>(L.bytes + o);
    const uint64_t w0 = __builtin_bswap64(k.hi), w1 = __builtin_bswap64(k.lo);
    *reinterpret_cast<uint4*>(d) = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
    if (len <= 16) return;
    // bytes 16.. : byte 16, then the tail's words shifted up one byte
    const uint64_t* t = reinterpret_cast<const uint64_t*>(k.tail);
    const uint32_t rest = len - 16, words = (rest + 7) / 8;
    uint64_t prev = (uint64_t)(k.meta >> 24);
    for (uint32_t w = 0; w < words; w += 2) {
        uint64_t x[2];
        for (int h = 0; h < 2; h++) {
            const uint32_t ww = w + h;
            const uint64_t tw = ww < words && len > 17 && ww < (len - 17 + 7) / 8 ? t[ww] : 0;
            x[h] = ww < words ? (prev | (tw << 8)) : 0;
            prev = tw >> 56;
        }
        *reinterpret_cast<uint4*>(d + 2 + w) =
            make_uint4((uint32_t)x[0], (uint32_t)(x[0] >> 32), (uint32_t)x[1], (uint32_t)(x[1] >> 32));
    }
}

// ---------------------------------------------------------- read check ----
// Per read range: conflict iff max(version over boundaries in
// [b, e), plus valueBefore(b) if b is not a boundary) > snapshot -- the
// predicate CheckMax evaluates on the skip list (SkipList.cpp:755-837;
// SURVEY.md Appendix A step 1).  Pages fully inside the range are skipped
// through the directory's per-page maxima (the skip list's upper-level
// maxVersion plays this role in the reference).
// A group of RC_G lanes per read: both endpoints are searched in lockstep
// (directory, then page, hist_search.h), then the group scans the versions
// covering [b, e) -- the slot b falls in, the slots up to e, and between the
// two pages the directory's page maxima (64-entry block maxima for long
// ranges) -- and ORs the result.
static constexpr int RC_G = SIDX_B;
#ifndef FDBCS_RC_WIDE
#define FDBCS_RC_WIDE 1  // (0: the two-level range maximum, kept for A/B)
#endif

struct ReadCheckArgs {
    int R;
    KeyArrays keys;
    const int32_t* read_txn;
    const int64_t* read_snap;  // INT64_MAX: the transaction is too old, nothing to check
    uint8_t* hist;
    Pool pool;
    Dir dir;
    const Scalars* sc;
    int64_t v0;            // version before the first boundary (sharded: the shard's carry-in)
    ShardBounds shard;     // reads are clipped to it (sharded mode)
    const int32_t* qx;     // large batches: directory entry of every read's begin (k_dir_join), else null
};

// The directory entry of e given that of b (<= e): a 16-entry window after
// it, one 128-byte line of first keys; past the window, the full search.
__device__ inline int dir_entry_after(const Group<RC_G>& g, const Dir& dir, int D, int xb, const Key& e) {
    const int j = xb + 1 + g.lane;
    const int c = __popc(g.ballot(j < D && dir_le(dir, j, e)));
    if (c < RC_G) return xb + c;
    DirHit h1, h2;
    grp_dir_find2(g, dir, D, e, e, h1, h2);
    return h1.x;
}

// read r, checked by the RC_G lanes of its group (g.lane).  WIDE: the range
// maximum between the edge pages has a third level (bmax2, 4096-entry
// groups), so a read costs at most 63 words per edge of each level at any
// span.
template <bool WIDE>
__device__ inline void read_check_group(const ReadCheckArgs& A, const Group<RC_G>& g, int r) {
    if (r >= A.R) return;
    const Pool& pool = A.pool;
    const Dir& dir = A.dir;
    const int t = A.read_txn[r];
    const int64_t s = A.read_snap[r];
    Key b = A.keys.get(2 * (int64_t)r), e = A.keys.get(2 * (int64_t)r + 1);
    const int D = A.sc->D;
    const int64_t v0 = A.sc->carry_dev ? A.sc->carry_check : A.v0;
    if (s == INT64_MAX) return;
    if (A.shard.has_lo | A.shard.has_hi) {  // the part of [b, e) in this shard (protocol A step 2)
        if (A.shard.below(b)) b = A.shard.lo;
        if (A.shard.at_or_above(e)) e = A.shard.hi;
        if (kcmp(b, e) >= 0) return;
    }
    DirHit hb, he;
    if (A.qx) {  // the begin's entry from the merge-join; the end's from the entries after it
        const int xb = A.qx[r];
        const int xe = dir_entry_after(g, dir, D, xb, e);
        hb = DirHit{xb, dir.page[xb], dir.cnt[xb]};
        he = DirHit{xe, dir.page[xe], dir.cnt[xe]};
    }
    const bool px = FDBCS_DIR_PX && A.sc->px_on;  // (long keys: the searches' prefix skips)
    if (!A.qx) {
        if (px) grp_dir_find2<true>(g, dir, D, b, e, hb, he);
        else grp_dir_find2<false>(g, dir, D, b, e, hb, he);
    }
    const int pb = hb.x, pe = he.x, cb = hb.cnt;
    int ib, ie;
    bool eqb, eqe;
    if (px) grp_page_find2<true>(g, pool, dir, hb.x, hb.page, hb.cnt, b, he.x, he.page, he.cnt, e, ib, eqb, ie, eqe);
    else grp_page_find2<false>(g, pool, dir, hb.x, hb.page, hb.cnt, b, he.x, he.page, he.cnt, e, ib, eqb, ie, eqe);
    const int64_t baseb = (int64_t)hb.page * PAGE, basee = (int64_t)he.page * PAGE;
    const int i0 = eqb ? ib : ib - 1;  // the slot whose version covers b
    bool c = i0 < 0 && v0 > s;
    const int lo = max(i0, 0);
    if (pe == pb) {
        for (int i = lo + g.lane; i < ie; i += RC_G) c |= pool.ver[baseb + i] > s;
    } else {
        for (int i = lo + g.lane; i < cb; i += RC_G) c |= pool.ver[baseb + i] > s;
        for (int i = g.lane; i < ie; i += RC_G) c |= pool.ver[basee + i] > s;
        const int q0 = pb + 1, q1 = pe;  // the entries strictly between
        const int qa = min(q1, (q0 + 63) & ~63), qz = max(qa, q1 & ~63);
        for (int q = q0 + g.lane; q < qa; q += RC_G) c |= dir.maxv[q] > s;
        for (int q = qz + g.lane; q < q1; q += RC_G) c |= dir.maxv[q] > s;
        if constexpr (WIDE) {
            const int g0 = qa >> 6, g1 = qz >> 6;
            const int ga = min(g1, (g0 + 63) & ~63), gz = max(ga, g1 & ~63);
            for (int q = g0 + g.lane; q < ga; q += RC_G) c |= dir.bmax[q] > s;
            for (int q = gz + g.lane; q < g1; q += RC_G) c |= dir.bmax[q] > s;
            for (int q = (ga >> 6) + g.lane; q < (gz >> 6); q += RC_G) c |= dir.bmax2[q] > s;
        } else {
            for (int q = (qa >> 6) + g.lane; q < (qz >> 6); q += RC_G) c |= dir.bmax[q] > s;
        }
    }
    if (g.ballot(c) && g.lane == 0) A.hist[t] = 1;
}

// ---------------------------------------------------------------- sort ----
// Two sorts per batch, in the same launches: the begin keys of all reads
// (slots 2r) and all write endpoints (slots 2R+i, begins even, ends odd).
// The order is total: key, then write END before write BEGIN at equal keys
// (the reference's tie digit, SkipList.cpp:169-172, which makes touching
// ranges stay separate in the combine), then slot.  A total order means no
// ties, so a record's output position is simply its rank.
//
// Sample sort (replaces the reference's MSD radix sort, sortPoints
// SkipList.cpp:227-279):
//   k_ss_scatter: splitters = every (1024/nb)-th of the 1024 quantile records
//                 kept from the previous batch's sorted output (LDS); lane per
//                 record: binary search -> bucket, atomicAdd -> slot in the
//                 bucket's staging row.
//   k_ss_bucket : one wavefront per bucket (~24 records): offset = sum of the
//                 earlier buckets' counts, bitonic sort of <= 128 records held
//                 two per lane in registers (partners exchanged by shuffles --
//                 no LDS, no barriers), write out[offset ...] and the
//                 quantiles the next batch splits by.
//   k_ss_sample : only when no quantiles exist yet (first batch, after an
//                 unbalanced batch): one workgroup per job bitonic-sorts 1024
//                 strided samples in LDS and keeps them as the quantiles.
// Splitters from an earlier batch are valid for any input (they only decide
// balance); a bucket above 128 records is sorted in LDS by its wavefront and
// flags a re-sample, above SS_ROW it is ranked from global memory.  Ties are
// broken by slot, so duplicated keys (Zipf hot keys) spread over buckets.
static constexpr int SS_MAXB = 1024;     // buckets per job (power of two)
static constexpr int SS_Q = 1024;        // quantile records kept per job
static constexpr int SS_WAVE = 128;      // bucket size sorted in registers
static constexpr int SS_ROW = 512;       // staging row per bucket (LDS path)
static constexpr int SS_CNT = 3 * SS_MAXB;  // counter words per parity: counts of both jobs, job 1's cover deltas

// A sort record's tail: the pointer its scatter kept in `pad` (the batch's
// tail bytes, one load fewer per tail compare of a sorted record), else the
// key arrays' (records rebuilt from LDS or loaded by slot carry pad 0;
// quantiles, which outlive the batch, are stored with pad 0).
__device__ inline uint64_t rec_pad(const Key& k) { return (uint64_t)(uintptr_t)k.tail; }
__device__ inline const uint8_t* rec_tail(const SRec& a, const uint8_t* const* tails) {
    return a.pad ? reinterpret_cast<const uint8_t*>(a.pad) : tails[a.idx];
}

// Total order on sort records: key, then END (odd slot) before BEGIN, then
// slot.  Branch-free on the fixed-width part; the tails are consulted only
// when both keys are > 17 bytes and equal on 17 bytes.  (hi, lo, meta) as
// integers is the key order otherwise: meta = byte16 << 24 | len.
// (out of line with scalar arguments: a record passed by reference to an
// out-of-line call is spilled to the stack)
__device__ __noinline__ bool rec_lt_tail_at(const uint8_t* ta, uint32_t ma, uint32_t ia, const uint8_t* tb,
                                            uint32_t mb, uint32_t ib) {
    const int c = tail_cmp(ta, key_len(ma), tb, key_len(mb));
    if (c) return c < 0;
    const uint32_t pa = ia & 1, pb = ib & 1;
    return pa != pb ? pa > pb : ia < ib;
}
__device__ inline bool rec_lt_tail(const SRec& a, const SRec& b, const uint8_t* const* tails) {
    return rec_lt_tail_at(rec_tail(a, tails), a.meta, a.idx, rec_tail(b, tails), b.meta, b.idx);
}

__device__ inline bool rec_lt(const SRec& a, const SRec& b, const uint8_t* const* tails) {
    const bool heq = a.hi == b.hi, leq = a.lo == b.lo;
    const bool tail_case = heq & leq & ((a.meta >> 24) == (b.meta >> 24)) & (key_len(a.meta) > 17) &
                           (key_len(b.meta) > 17);
    if (__builtin_expect(tail_case, 0)) return rec_lt_tail(a, b, tails);
    const uint32_t pa = a.idx & 1, pb = b.idx & 1;
    const bool tlt = (pa > pb) | ((pa == pb) & (a.idx < b.idx));
    const bool mlt = (a.meta < b.meta) | ((a.meta == b.meta) & tlt);
    const bool llt = (a.lo < b.lo) | (leq & mlt);
    return (a.hi < b.hi) | (heq & llt);
}

// key-only three-way compare of a record against a key
__device__ __noinline__ int tail_cmp_at(const uint8_t* ta, uint32_t la, const uint8_t* tb, uint32_t lb) {
    return tail_cmp(ta, la, tb, lb);
}
__device__ inline int rec_vs_key_tail(const SRec& a, const Key& k, const uint8_t* const* tails) {
    return tail_cmp_at(rec_tail(a, tails), key_len(a.meta), k.tail, key_len(k.meta));
}

__device__ inline int rec_vs_key(const SRec& a, const Key& k, const uint8_t* const* tails) {
    const bool heq = a.hi == k.hi, leq = a.lo == k.lo;
    const bool tail_case = heq & leq & ((a.meta >> 24) == (k.meta >> 24)) & (key_len(a.meta) > 17) &
                           (key_len(k.meta) > 17);
    if (__builtin_expect(tail_case, 0)) return rec_vs_key_tail(a, k, tails);
    const bool lt = (a.hi < k.hi) | (heq & ((a.lo < k.lo) | (leq & (a.meta < k.meta))));
    const bool eq = heq & leq & (a.meta == k.meta);
    return lt ? -1 : (eq ? 0 : 1);
}

struct SortJobs {
    int32_t n[2];          // records per job
    int32_t nb[2];         // buckets per job (power of two, <= SS_MAXB)
    int32_t blocks0;       // scatter blocks of job 0
    int64_t sbase[2];      // slot of record 0
    int32_t sstride[2];    // slot step per record
    SRec* out[2];          // sorted output
    uint32_t* out_slot;    // [n1] slots of job 1's sorted records (compact copy)
    SRec* quant;           // [2][SS_Q] quantiles (persist across batches)
    uint8_t* qtail;        // [2][SS_Q][SS_QT] their first SS_QT tail bytes
    int32_t* cnt;          // [SS_CNT] this batch's bucket counts: [2][SS_MAXB], then job 1's cover deltas
    int32_t* cnt_next;     // [SS_CNT] the next batch's (zeroed here)
    int32_t* dcnt;         // [SS_MAXB] = cnt + 2 SS_MAXB: per bucket of job 1, write begins minus write ends
    int32_t* wcov;         // [2W] or null: per sorted write endpoint, the begins minus ends at or before it
    int32_t* bkt;          // [n0 + n1] bucket of each record
    SRec* tmp;             // [2][SS_MAXB][SS_ROW] staging rows
    Scalars* sc;
};

// Quantiles outlive the batch whose keys they are, so their tails are kept
// (first SS_QT bytes) beside them.  x < splitter q, in the record order; a
// splitter whose tail was cut stands for the prefix it kept (the smallest key
// with that prefix), which is still a consistent split point.
__device__ inline void put_quantile(const SortJobs& J, int job, int q, const SRec& x, const uint8_t* const* tails) {
    SRec y = x;
    y.pad = 0;  // (the batch's tail pointer: quantiles outlive the batch, qtail keeps their bytes)
    J.quant[job * SS_Q + q] = y;
    const uint32_t L = key_len(x.meta);
    if (L > 17) {
        const int words = (int)min<uint32_t>((L - 17 + 7) / 8, SS_QT / 8);
        const uint64_t* src = reinterpret_cast<const uint64_t*>(rec_tail(x, tails));
        uint64_t* dst = reinterpret_cast<uint64_t*>(J.qtail + (int64_t)(job * SS_Q + q) * SS_QT);
        // (every word loaded before any store: a store between them would
        // keep the next load behind it, a round trip a word)
        uint64_t v[SS_QT / 8];
#pragma unroll
        for (int w = 0; w < SS_QT / 8; w++) v[w] = w < words ? src[w] : 0;
#pragma unroll
        for (int w = 0; w < SS_QT / 8; w++)
            if (w < words) dst[w] = v[w];
    }
}

__device__ __noinline__ bool rec_lt_quant_tail_at(const uint8_t* xt, uint32_t xm, uint32_t xi, uint32_t qm, uint32_t qi,
                                                  const uint8_t* qt) {
    const uint32_t lx = key_len(xm), lq = key_len(qm);
    if (lq - 17 > (uint32_t)SS_QT) {  // q was cut: compare with its kept prefix
        const uint32_t lp = 17 + SS_QT;
        const int c = tail_cmp(xt, lx, qt, lp);
        return c < 0;  // (a key that starts with the prefix is not below it)
    }
    const int c = tail_cmp(xt, lx, qt, lq);
    if (c) return c < 0;
    const uint32_t px = xi & 1, pq = qi & 1;
    return px != pq ? px > pq : xi < qi;
}
__device__ inline bool rec_lt_quant_tail(const SRec& x, const SRec& q, const uint8_t* qt,
                                         const uint8_t* const* tails) {
    return rec_lt_quant_tail_at(rec_tail(x, tails), x.meta, x.idx, q.meta, q.idx, qt);
}

__device__ inline bool rec_lt_quant(const SRec& x, const SRec& q, const uint8_t* qt, const uint8_t* const* tails) {
    const bool heq = x.hi == q.hi, leq = x.lo == q.lo;
    const bool tail_case = heq & leq & ((x.meta >> 24) == (q.meta >> 24)) & (key_len(x.meta) > 17) &
                           (key_len(q.meta) > 17);
    if (__builtin_expect(tail_case, 0)) return rec_lt_quant_tail(x, q, qt, tails);
    return rec_lt(x, q, tails);  // (decided without tails)
}

__device__ inline SRec load_rec(const KeyArrays& keys, int64_t slot) {
    return SRec{keys.hi[slot], keys.lo[slot], keys.meta[slot], (uint32_t)slot, 0};
}

// LDS record image: three 8-byte arrays; idx == REC_INF marks +infinity
// (padding), which compares above everything without touching a tail.
struct LdsRecs {
    uint64_t* hi;
    uint64_t* lo;
    uint64_t* mi;  // meta << 32 | idx
    __device__ SRec get(int i) const {
        const uint64_t m = mi[i];
        return SRec{hi[i], lo[i], (uint32_t)(m >> 32), (uint32_t)m, 0};
    }
    __device__ void put(int i, const SRec& r) const {
        hi[i] = r.hi;
        lo[i] = r.lo;
        mi[i] = ((uint64_t)r.meta << 32) | r.idx;
    }
};
constexpr uint32_t REC_INF = 0xFFFFFFFFu;
__device__ inline SRec rec_inf() { return SRec{~0ull, ~0ull, ~0u, REC_INF, 0}; }

__device__ inline bool rec_lt_inf(const SRec& a, const SRec& b, const uint8_t* const* tails) {
    if (b.idx == REC_INF) return a.idx != REC_INF;
    if (a.idx == REC_INF) return false;
    return rec_lt(a, b, tails);
}

// Ascending bitonic sort of P (power of two) records in LDS; every thread of
// the workgroup calls it.
__device__ void lds_bitonic(const LdsRecs& L, int P, const uint8_t* const* tails) {
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < (P >> 1); i += blockDim.x) {
                const int a = ((i & ~(j - 1)) << 1) | (i & (j - 1));
                const int b = a | j;
                const SRec x = L.get(a), y = L.get(b);
                const bool up = (a & k) == 0;
                const bool sw = up ? rec_lt_inf(y, x, tails) : rec_lt_inf(x, y, tails);
                if (sw) {
                    L.put(a, y);
                    L.put(b, x);
                }
            }
            __syncthreads();
        }
    }
}

__device__ inline SRec shfl_xor_rec(const SRec& r, int m) {
    return SRec{__shfl_xor(r.hi, m, 64), __shfl_xor(r.lo, m, 64), (uint32_t)__shfl_xor((int)r.meta, m, 64),
                (uint32_t)__shfl_xor((int)r.idx, m, 64), 0};
}

// Ascending bitonic sort of P <= 128 records held by one wavefront, element
// e = 2*lane + q in r[q].  Partners at distance j >= 2 live in lane ^ (j/2).
__device__ void wave_bitonic(SRec r[2], int P, const uint8_t* const* tails) {
    const int lane = threadIdx.x & 63;
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j == 1) {
                const bool up = ((2 * lane) & k) == 0;
                const bool sw = up ? rec_lt_inf(r[1], r[0], tails) : rec_lt_inf(r[0], r[1], tails);
                if (sw) {
                    const SRec t = r[0];
                    r[0] = r[1];
                    r[1] = t;
                }
            } else {
#pragma unroll
                for (int q = 0; q < 2; q++) {
                    const int e = 2 * lane + q;
                    const SRec o = shfl_xor_rec(r[q], j >> 1);
                    const bool up = (e & k) == 0, lower = (e & j) == 0;
                    const bool take = (lower == up) ? rec_lt_inf(o, r[q], tails) : rec_lt_inf(r[q], o, tails);
                    if (take) r[q] = o;
                }
            }
        }
    }
}

// Splitters drawn from the batch itself: SS_S strided samples (4x the
// quantiles kept, so a bucket between two splitters holds ~4 sample gaps and
// its size concentrates) sorted in LDS.  Returns the sample count.
static constexpr int SS_S = 4096;
__device__ int sample_quantiles(const SortJobs& J, int job, const KeyArrays& keys, const LdsRecs& L) {
    const int n = J.n[job];
    const int ns = min(n, SS_S);
    for (int k = threadIdx.x; k < SS_S; k += blockDim.x) {
        if (k < ns) {
            const int64_t r = ((int64_t)k * n + n / (2 * ns)) / ns;
            L.put(k, load_rec(keys, J.sbase[job] + r * J.sstride[job]));
        } else {
            L.put(k, rec_inf());
        }
    }
    __syncthreads();
    lds_bitonic(L, SS_S, keys.tail);
    for (int q = threadIdx.x; q < SS_Q; q += blockDim.x)
        put_quantile(J, job, q, L.get((int)((int64_t)q * ns / SS_Q)), keys.tail);
    return ns;
}

// record i of a job goes to bucket b: count, bucket id, staging row
__device__ inline void place_rec(const SortJobs& J, int job, int i, int b, const SRec& x) {
    const int slot = atomicAdd(&J.cnt[job * SS_MAXB + b], 1);
    if (job && J.wcov) atomicAdd(&J.dcnt[b], (x.idx & 1) ? -1 : 1);  // (the write cover: a begin opens, an end closes)
    J.bkt[(job ? J.n[0] : 0) + i] = b;
    if (slot < SS_ROW) J.tmp[((int64_t)job * SS_MAXB + b) * SS_ROW + slot] = x;
    else if (slot == SS_ROW) J.sc->ss_over[job] = 1;  // the bucket kernel would rank it from global memory
}

// One workgroup per job.  guard == 0: the first batch -- splitters from a
// sample of this batch.  guard == 1 (after every scatter): nothing, unless a
// bucket overflowed its staging row (the key distribution moved away from the
// previous batch's quantiles); then splitters from this batch's own sample
// and every record of the job is bucketed again, so the batch keeps the fast
// bucket paths instead of an O(bucket x n) global-memory ranking.
__device__ void ss_sample_job(const SortJobs& J, const KeyArrays& keys, const LdsRecs& L, int guard) {
    const int job = blockIdx.x;
    const int n = J.n[job];
    if (guard && !J.sc->ss_over[job]) return;
    if (n == 0) return;
    const int ns = sample_quantiles(J, job, keys, L);
    if (!guard) return;
    const int nb = J.nb[job], step = SS_Q / nb;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        J.cnt[job * SS_MAXB + b] = 0;
        if (job) J.dcnt[b] = 0;
    }
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) J.sc->ss_resample = 1;  // (stats: the batch was bucketed twice)
    for (int i = threadIdx.x; i < n; i += blockDim.x) {
        const SRec x = load_rec(keys, J.sbase[job] + (int64_t)i * J.sstride[job]);
        int lo = 0, len = nb - 1;  // bucket = number of splitters <= x
        while (len > 0) {
            const int half = len >> 1, k = lo + half;
            const SRec sp = L.get((int)((int64_t)((k + 1) * step) * ns / SS_Q));
            if (!rec_lt(x, sp, keys.tail)) {
                lo += half + 1;
                len -= half + 1;
            } else {
                len = half;
            }
        }
        place_rec(J, job, i, lo, x);
    }
    __syncthreads();
    if (threadIdx.x == 0) J.sc->ss_over[job] = 0;  // (a bucket may still exceed its row: ranked globally)
}

__global__ __launch_bounds__(1024) void k_ss_sample(SortJobs J, KeyArrays keys, int guard) {
    __shared__ uint64_t s_hi[SS_S], s_lo[SS_S], s_mi[SS_S];
    ss_sample_job(J, keys, LdsRecs{s_hi, s_lo, s_mi}, guard);
}

// The guard after every scatter, without the 96 KiB of LDS (whose allocation
// made even the usual immediate return cost ~4.6 us): the rare resample sorts
// its sample in global scratch (3 * SS_S words per job).
__global__ __launch_bounds__(1024) void k_ss_guard(SortJobs J, KeyArrays keys, uint64_t* scratch) {
    PHASE(J.sc, 12);  // (FDBCS_PHASES builds: the first launch after the live kernel, scripts/diag_live.py)
    uint64_t* g = scratch + (int64_t)blockIdx.x * 3 * SS_S;
    ss_sample_job(J, keys, LdsRecs{g, g + SS_S, g + 2 * SS_S}, 1);
}

// Splitter s of a job is quantile (s + 1) * SS_Q / nb.  Scatter kernels keep
// the splitters' first key words in LDS and fetch the whole quantile only on
// a tie of those words.
__device__ inline void splitter_fill(const SortJobs& J, int job, uint64_t* sp) {
    const int nb = J.nb[job], step = SS_Q / max(nb, 1);
    for (int k = threadIdx.x; k < nb - 1; k += blockDim.x) sp[k] = J.quant[job * SS_Q + (k + 1) * step].hi;
}

// rec_lt_quant for an x longer than 17 bytes whose tail is xt: the splitter,
// its kept tail and x's first tail words are loaded together -- one round
// trip a search step where rec_lt_quant takes two (the splitter, then both
// tails); config 4's keys tie on their first 64 bytes, so every step of
// their splitter search compares tails.  (x's words past the compared ones
// are loaded and ignored: every compare stops within SS_QT tail bytes.)
__device__ inline bool rec_lt_quant_long(const SRec& x, const uint8_t* xt, const SRec* qp, const uint8_t* qt,
                                         const uint8_t* const* tails) {
    constexpr int NW = SS_QT / 8;
    const uint32_t lx = key_len(x.meta);
    const int xwords = (int)min<uint32_t>((lx - 17 + 7) >> 3, (uint32_t)NW);
    const uint64_t* a = reinterpret_cast<const uint64_t*>(xt);
    const uint64_t* b = reinterpret_cast<const uint64_t*>(qt);
    uint64_t xa[NW], yb[NW];
#pragma unroll
    for (int k = 0; k < NW; k++) {
        xa[k] = k < xwords ? a[k] : 0;
        yb[k] = k < xwords ? b[k] : 0;
    }
    const SRec q = *qp;
    const bool tail_case = (x.hi == q.hi) & (x.lo == q.lo) & ((x.meta >> 24) == (q.meta >> 24)) &
                           (key_len(q.meta) > 17);
    if (!tail_case) return rec_lt(x, q, tails);  // (decided without tails)
    // as rec_lt_quant_tail: a cut splitter stands for its kept prefix
    const uint32_t lq = key_len(q.meta);
    const bool cut = lq - 17 > (uint32_t)SS_QT;
    const uint32_t lb = cut ? 17 + SS_QT : lq;
    const int words = (int)(((lx < lb ? lx : lb) - 17 + 7) >> 3);  // (<= xwords)
    int c = 0;
#pragma unroll
    for (int k = NW - 1; k >= 0; k--)  // (the first differing word decides)
        if (k < words && xa[k] != yb[k]) c = __builtin_bswap64(xa[k]) < __builtin_bswap64(yb[k]) ? -1 : 1;
    if (c == 0) c = lx < lb ? -1 : (lx > lb ? 1 : 0);
    if (cut || c) return c < 0;
    const uint32_t px = x.idx & 1, pq = q.idx & 1;
    return px != pq ? px > pq : x.idx < q.idx;
}

// bucket of record x = number of splitters <= x (splitters nondecreasing)
__device__ inline int bucket_of(const SortJobs& J, int job, const uint64_t* sp, const SRec& x,
                                const uint8_t* const* tails) {
    const int nb = J.nb[job], step = SS_Q / nb;
    const uint8_t* xt = key_len(x.meta) > 17 ? rec_tail(x, tails) : nullptr;  // (once, not per step)
    int lo = 0, len = nb - 1;
    while (len > 0) {
        const int half = len >> 1, k = lo + half;
        const uint64_t h = sp[k];
        bool le;
        if (h != x.hi) {
            le = h < x.hi;
        } else {
            const int q = job * SS_Q + (k + 1) * step;
            const uint8_t* qt = J.qtail + (int64_t)q * SS_QT;
            le = xt ? !rec_lt_quant_long(x, xt, J.quant + q, qt, tails) : !rec_lt_quant(x, J.quant[q], qt, tails);
        }
        if (le) {
            lo += half + 1;
            len -= half + 1;
        } else {
            len = half;
        }
    }
    return lo;
}

// record i of a job into its bucket's staging row
__device__ inline void scatter_rec(const SortJobs& J, int job, int i, const SRec& x, const uint8_t* const* tails,
                                   const uint64_t* sp) {
    place_rec(J, job, i, bucket_of(J, job, sp, x, tails), x);
}

__global__ __launch_bounds__(256) void k_ss_scatter(SortJobs J, KeyArrays keys) {
    __shared__ uint64_t sp[SS_MAXB];
    const int job = blockIdx.x < J.blocks0 ? 0 : 1;
    const int i = (job ? blockIdx.x - J.blocks0 : blockIdx.x) * blockDim.x + threadIdx.x;
    splitter_fill(J, job, sp);
    __syncthreads();
    if (i >= J.n[job]) return;
    scatter_rec(J, job, i, load_rec(keys, J.sbase[job] + (int64_t)i * J.sstride[job]), keys.tail, sp);
}

// Ingest: one launch, two kinds of blocks.  Transaction blocks: tooOld
// (SkipList.cpp:985: the previous batch's oldestVersion, >= 1 read), the
// per-range transaction maps and snapshots.  Range blocks: encode both keys
// of a range (the begin < end precondition), and -- in steady state, when
// splitters from an earlier batch exist (SCATTER) -- scatter the range's sort
// records straight into their buckets (reads: the begin; writes: both ends).
#ifndef FDBCS_INGEST_BLOCK
#define FDBCS_INGEST_BLOCK 256
#endif
// The top level of the read check's range maximum: bmax2[k] = max of maxv over
// directory entries [4096k, 4096k + 4096), from independent loads (16 per
// thread of a 256-thread block) and one block reduction.
__device__ inline void bmax2_block(const Dir& d, int D, int k) {
    __shared__ int64_t red[1024 / 64];
    const int base = k * BMAX2_SPAN;
    if (base >= D) return;
    const int end = min(D, base + BMAX2_SPAN);
    int64_t m = INT64_MIN;
#pragma unroll 4
    for (int x = base + (int)threadIdx.x; x < end; x += blockDim.x) m = max(m, d.maxv[x]);
    m = wave_reduce_max(m);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < (int)(blockDim.x >> 6); w++) m = max(m, red[w]);
        d.bmax2[k] = m;
    }
}
template <bool SCATTER>
__global__ __launch_bounds__(FDBCS_INGEST_BLOCK) void k_ingest(IngestArgs A, SortJobs J) {
    if ((int)blockIdx.x < A.prep_blocks) {
        const int t = blockIdx.x * blockDim.x + threadIdx.x;
        if (t == 0) {
            A.sc->n_comb = 0;  // stays 0 if the batch has no transactions
            A.sc->n_comb_own = 0;
            A.sc->ss_resample = 0;
            A.sc->ss_maxc = 0;
        }
        if (t >= A.T) return;
        const int r0 = A.ro[t], r1 = A.ro[t + 1];
        const int64_t sn = A.snap[t];
        const bool too = sn < A.oldest && r1 > r0;
        A.too_old[t] = too ? 1 : 0;
        A.hist[t] = 0;
        A.deg[t] = 0;
        for (int r = r0; r < r1; r++) {
            A.read_txn[r] = t;
            A.read_snap[r] = too ? INT64_MAX : sn;  // the read check skips too-old transactions
        }
        for (int w = A.wo[t], w1 = A.wo[t + 1]; w < w1; w++) A.write_txn[w] = t;
        return;
    }
    if ((int)blockIdx.x < A.prep_blocks + A.bmax2_blocks) {  // bmax2: one word per block
        bmax2_block(A.hd, A.sc->D, (int)blockIdx.x - A.prep_blocks);
        return;
    }
    const int64_t i0 = (int64_t)(blockIdx.x - A.prep_blocks - A.bmax2_blocks) * blockDim.x;
    const int64_t i = i0 + threadIdx.x;
    [[maybe_unused]] __shared__ uint64_t sp[2][SCATTER ? SS_MAXB : 1];
    if constexpr (SCATTER) {
        if (i0 < A.R) splitter_fill(J, 0, sp[0]);
        if (i0 + blockDim.x > A.R) splitter_fill(J, 1, sp[1]);
        __syncthreads();
    }
    if (i >= (int64_t)A.R + A.W) return;
    const Key b = encode_key(A.bytes + A.koff[2 * i], A.klen[2 * i], A.btail, A.btail_cap, A.sc);
    const Key e = encode_key(A.bytes + A.koff[2 * i + 1], A.klen[2 * i + 1], A.btail, A.btail_cap, A.sc);
    A.keys.put(2 * i, b);
    A.keys.put(2 * i + 1, e);
    if (kcmp(b, e) >= 0) atomicCAS(&A.sc->err, 0, FDBCS_E_RANGE);  // every range must be non-empty
    if constexpr (SCATTER) {
        const uint8_t* const* tails = A.keys.tail;
        if (i < A.R) {
            if (J.nb[0]) scatter_rec(J, 0, (int)i, SRec{b.hi, b.lo, b.meta, (uint32_t)(2 * i), rec_pad(b)}, tails, sp[0]);
        } else {
            const int w = (int)(i - A.R);
            scatter_rec(J, 1, 2 * w, SRec{b.hi, b.lo, b.meta, (uint32_t)(2 * i), rec_pad(b)}, tails, sp[1]);
            scatter_rec(J, 1, 2 * w + 1, SRec{e.hi, e.lo, e.meta, (uint32_t)(2 * i + 1), rec_pad(e)}, tails, sp[1]);
        }
    }
}

// The per-transaction path (stage.h): k_unpack's work and the ingest's in one
// launch, straight from the record stream.  A wavefront takes STG_TPW
// consecutive transactions: lanes < STG_TPW read their record headers (into
// LDS), then the wavefront's ranges go one per lane -- range k belongs to the
// transaction whose range prefix covers it, and its StageRange entry (written
// by the host's add) gives both keys' places with no prefix sum over the
// record.  Each lane writes the batch view's entries of its range (later
// readers: load metrics), the prep arrays (tooOld, range -> txn) and encodes,
// validates and scatters the range as k_ingest's encode lanes do.
#ifndef FDBCS_STG_TPW
#define FDBCS_STG_TPW 8
#endif
#ifndef FDBCS_STG_BLOCK
#define FDBCS_STG_BLOCK 256
#endif
constexpr int STG_TPW = FDBCS_STG_TPW;
constexpr int STG_BLOCK = FDBCS_STG_BLOCK;
static_assert(STG_TPW >= 1 && STG_TPW <= 64 && STG_BLOCK % 64 == 0, "staged ingest shape");

// a wavefront's transactions in LDS (k_ingest_staged, k_live_ingest)
struct StgShared {
    uint64_t base[STG_BLOCK / 64][STG_TPW];
    int64_t snap[STG_BLOCK / 64][STG_TPW];
    int32_t ro[STG_BLOCK / 64][STG_TPW], wo[STG_BLOCK / 64][STG_TPW], nr[STG_BLOCK / 64][STG_TPW],
        pre[STG_BLOCK / 64][STG_TPW];
};

// LIVE's capacities and stream bounds
struct LiveOut {
    int32_t capT, capR, capW;
    // the window copy stays below this: the stream allocation's size, and in
    // the live kernel the bytes the host has written whole, rounded up to 16
    // (reading lines the host is still appending to made its adds stall)
    uint64_t stream_cap;
    uint64_t valid;  // live kernel: the stream bytes the host had written whole (the published transactions' records)
    bool spec;  // read the window [stream_cap - LIVE_WIN, stream_cap) together with the offsets
};

// LIVE: a wavefront's records come over PCIe into an LDS window first -- its
// transactions' record bytes from the first one on, 16 bytes a lane, one
// round trip for the group instead of dependent header / entry / key reads
// per lane (measured: ~36 transactions per us with the per-lane reads, slower
// than the Resolver's adds arrive at the end of a batch); a key or record
// past the window is read from the host-mapped stream directly.
constexpr int LIVE_WIN = 4096;  // bytes per wavefront (config 2: 8 records of ~300 bytes)
// A host-mapped word as the host wrote it last: relaxed system-scope loads
// (sc0 sc1) bypass the GPU's caches -- the progress words and the record
// offsets (a 128-byte line of offsets also holds later groups' entries).
// Plain or non-temporal loads of a line the host was still appending to left
// it in a cache, and a later group reading that line saw its old bytes
// (measured: wrong keys whenever groups ran before the final word); the
// record windows avoid such lines instead (TxnStage::publish pads).
__device__ inline uint64_t host_load(const uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct LiveWin {
    const uint8_t* win;  // LDS
    uint64_t lo, hi;     // the stream bytes [lo, hi) it holds
    uint64_t valid;      // ... of which those below `valid` were written whole when copied
    const uint8_t* host;
    __device__ const uint8_t* at(uint64_t off, uint64_t len) const {
        // (+8: encode_key reads the aligned words around a key -- bytes past
        // the key, which it masks, may be ones the host had not written yet)
        if (off >= lo && off + len <= valid && off + len + 8 <= hi) return win + (off - lo);
        // past the window: plain loads of the stream itself, which the caches
        // may hold from before the host wrote it -- a system-scope acquire
        // drops them first (rare: a group larger than the window)
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
        return host + off;
    }
};

// One wavefront's group of transactions [t0, t0 + nt) (nt <= STG_TPW) of a
// per-transaction record stream.  LIVE (k_live_ingest): the stream is
// host-mapped and the batch's read count is not known yet, so the writes sit
// at A.wbase = 2 caps.R (BatchBufs::lv_wbase); a transaction past the live
// capacities marks lv_err and fails the batch (the host cancels first).
template <bool SCATTER, bool LIVE>
__device__ inline void staged_group(const IngestArgs& A, const SortJobs& J, const StagedBatch& S, const LiveOut& O,
                                    int t0, int nt, StgShared& L, const uint64_t* sp0, const uint64_t* sp1,
                                    uint8_t* win = nullptr) {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    // ---- headers: lane q < nt reads transaction t0 + q
    const int t = t0 + lane;
    const bool ht = lane < nt;
    int n = 0;
    const uint64_t to = ht ? (LIVE ? host_load(S.toff + t) : S.toff[t]) : STAGE_EMPTY;
    LiveWin X{win, 0, 0, O.valid, S.stream};
    if constexpr (LIVE) {  // the group's records into the LDS window (16-byte aligned, coalesced)
        // each lane's 16-byte pieces are loaded before any is stored, so the
        // window is one round trip; speculative: the stream's last LIVE_WIN
        // bytes, loaded while the offsets are still in flight (a group among
        // the last published ones lies there)
        constexpr int WPL = LIVE_WIN / 16 / 64;
        const uint64_t shi = O.stream_cap & ~uint64_t(15);
        const uint64_t slo = shi > (uint64_t)LIVE_WIN ? shi - LIVE_WIN : 0;
        // (16-byte non-temporal loads: the window never reaches past the bytes
        // the host published, which end on a 128-byte line the host does not
        // write again -- TxnStage::publish -- so no cache can hold an older
        // copy of a line read here)
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        u32x4 v[WPL];
        auto load_win = [&](uint64_t lo, uint64_t hi) {
            const u32x4* src = reinterpret_cast<const u32x4*>(S.stream + lo);
            const int n16 = (int)((hi - lo) >> 4);
#pragma unroll
            for (int u = 0; u < WPL; u++)
                if (lane + 64 * u < n16) v[u] = __builtin_nontemporal_load(src + lane + 64 * u);
        };
        auto store_win = [&](uint64_t lo, uint64_t hi) {
            u32x4* dst = reinterpret_cast<u32x4*>(win);
            const int n16 = (int)((hi - lo) >> 4);
#pragma unroll
            for (int u = 0; u < WPL; u++)
                if (lane + 64 * u < n16) dst[lane + 64 * u] = v[u];
        };
        if (O.spec) load_win(slo, shi);
        uint64_t first = ~0ull;
        for (int q = 0; q < nt; q++) {
            const uint64_t o = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)to, q) |
                               ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(to >> 32), q) << 32);
            if (!(o & STAGE_EMPTY)) {
                first = o;
                break;
            }
        }
        if (first != ~0ull) {
            if (O.spec && first >= slo) {  // (the speculative window holds the group)
                X.lo = slo;
                X.hi = shi;
            } else {
                X.lo = first & ~uint64_t(15);
                X.hi = min(X.lo + (uint64_t)LIVE_WIN, shi);
                load_win(X.lo, X.hi);
            }
            store_win(X.lo, X.hi);
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_wave_barrier();
        }
        if (lane == 0) PMAX(A.sc, 22);
    }
    if (ht) {
        const StageTxn h = (!LIVE || (to & STAGE_EMPTY)) ? stage_txn(S.stream, to)
                                                        : stage_txn(X.at(to, sizeof(StageHdr)) - to, to);
        n = h.nr + h.nw;
        if (LIVE && (t >= O.capT || h.ro + h.nr > O.capR || h.wo + h.nw > O.capW)) {
            atomicOr(&A.sc->lv_err, 1);
            atomicCAS(&A.sc->err, 0, FDBCS_E_STATE);
            n = 0;
        }
        L.base[wv][lane] = h.base;
        L.snap[wv][lane] = h.snap < A.oldest && h.nr > 0 ? INT64_MAX : h.snap;  // (tooOld: nothing to check)
        L.ro[wv][lane] = h.ro;
        L.wo[wv][lane] = h.wo;
        L.nr[wv][lane] = h.nr;
        if (!LIVE || t < O.capT) {
            S.view.snap[t] = h.snap;
            S.view.ro[t] = h.ro;
            S.view.wo[t] = h.wo;
            A.too_old[t] = h.snap < A.oldest && h.nr > 0 ? 1 : 0;  // addTransaction's rule (SkipList.cpp:985)
            A.hist[t] = 0;
            A.deg[t] = 0;
        }
    }
    const int incl = wave_incl_scan(n);
    if (lane < STG_TPW) L.pre[wv][lane] = lane < nt ? incl : 1 << 30;
    const int ntot = __builtin_amdgcn_readlane(incl, STG_TPW - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // (this wavefront's LDS writes, read below)
    __builtin_amdgcn_wave_barrier();
    if (LIVE && lane == 0) PMAX(A.sc, 14);
    const uint8_t* const* tails = A.keys.tail;
    // ---- the wavefront's ranges, one per lane
    for (int k = lane; k < ntot; k += 64) {
        int j = 0;  // owner: the transactions whose range prefix ends at or before k
#pragma unroll
        for (int q = 0; q < STG_TPW - 1; q++) j += L.pre[wv][q] <= k;
        const int q = k - (j ? L.pre[wv][j - 1] : 0);
        const uint64_t base = L.base[wv][j];
        const uint64_t eo = base + sizeof(StageHdr) + sizeof(StageRange) * (uint64_t)q;
        const StageRange e = *reinterpret_cast<const StageRange*>(LIVE ? X.at(eo, sizeof(StageRange)) : S.stream + eo);
        const int nrj = L.nr[wv][j];
        int64_t i;  // the range's begin slot: read r at 2r, write w at wbase + 2w (fdbcs_batch_view's layout)
        int r = -1, w = -1;
        if (q < nrj) {
            r = L.ro[wv][j] + q;
            i = 2 * (int64_t)r;
            A.read_txn[r] = t0 + j;
            A.read_snap[r] = L.snap[wv][j];
        } else {
            w = L.wo[wv][j] + q - nrj;
            i = A.wbase + 2 * (int64_t)w;
            A.write_txn[w] = t0 + j;
        }
        const uint64_t ob = base + e.kofs, oe = base + stage_end_ofs(e);
        const uint32_t el = stage_end_len(e);
        const Key b = encode_key(LIVE ? X.at(ob, e.blen) : S.stream + ob, e.blen, A.btail, A.btail_cap, A.sc);
        const Key en = encode_key(LIVE ? X.at(oe, el) : S.stream + oe, el, A.btail, A.btail_cap, A.sc);
        if (A.lm.on) {  // iopsSample.addAndExpire of the range's begin, in the Resolver's add order (writes first)
            const int nwj = L.pre[wv][j] - (j ? L.pre[wv][j - 1] : 0) - nrj;
            const uint64_t pos = (uint64_t)L.ro[wv][j] + (uint64_t)L.wo[wv][j] + (uint64_t)(q < nrj ? nwj + q : q - nrj);
            const int64_t amt = roll_amount(roll_hash(A.lm.seed, A.lm.seq, pos), A.lm.offset_per_key + e.blen,
                                            A.lm.units);
            if (amt) lm_append(A.lm, A.sc, amt, b, pos);
        }
        if (kcmp(b, en) >= 0) atomicCAS(&A.sc->err, 0, FDBCS_E_RANGE);  // every range must be non-empty
        S.view.koff[i] = ob;
        S.view.klen[i] = e.blen;
        S.view.koff[i + 1] = oe;
        S.view.klen[i + 1] = el;
        A.keys.put(i, b);
        A.keys.put(i + 1, en);
        if constexpr (SCATTER) {
            if (w < 0) {
                if (J.nb[0]) scatter_rec(J, 0, r, SRec{b.hi, b.lo, b.meta, (uint32_t)i, rec_pad(b)}, tails, sp0);
            } else {
                scatter_rec(J, 1, 2 * w, SRec{b.hi, b.lo, b.meta, (uint32_t)i, rec_pad(b)}, tails, sp1);
                scatter_rec(J, 1, 2 * w + 1, SRec{en.hi, en.lo, en.meta, (uint32_t)(i + 1), rec_pad(en)}, tails, sp1);
            }
        }
    }
    if (LIVE && lane == 0) PMAX(A.sc, 15);  // (the ranges issued; their stores drain before ph[23])
}

template <bool SCATTER>
__global__ __launch_bounds__(STG_BLOCK) void k_ingest_staged(IngestArgs A, SortJobs J, StagedBatch S, int stg_blocks) {
    __shared__ StgShared L;
    [[maybe_unused]] __shared__ uint64_t sp[2][SCATTER ? SS_MAXB : 1];
    if ((int)blockIdx.x >= stg_blocks) {  // bmax2: one word per block
        bmax2_block(A.hd, A.sc->D, (int)blockIdx.x - stg_blocks);
        return;
    }
    if constexpr (SCATTER) {
        splitter_fill(J, 0, sp[0]);
        splitter_fill(J, 1, sp[1]);
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        A.sc->n_comb = 0;  // stays 0 if the batch has no transactions
        A.sc->n_comb_own = 0;
        A.sc->ss_resample = 0;
        A.sc->ss_maxc = 0;
        S.view.ro[A.T] = A.R;
        S.view.wo[A.T] = A.W;
    }
    const int wv = threadIdx.x >> 6;
    const int t0 = ((int)blockIdx.x * (STG_BLOCK / 64) + wv) * STG_TPW;
    if (t0 >= A.T) return;  // (the whole wavefront)
    staged_group<SCATTER, false>(A, J, S, LiveOut{}, t0, min(STG_TPW, A.T - t0), L, sp[0], sp[SCATTER ? 1 : 0]);
}

// ---- live ingest ------------------------------------------------------------
// The Resolver adds T transactions one by one before detectConflicts
// (Resolver.actor.cpp:140-153).  At fdbcs_batch_begin this persistent kernel
// is queued on the engine's stream (behind the previous batch's history
// update); it encodes each group of STG_TPW transactions as soon as the host
// has published it, reading the records straight from the host-mapped
// stream, so that by detectConflicts only the last groups remain.
//   block 0, wave 0: the poller -- reads the host's progress words (one PCIe
//                    read per ~1 us) and mirrors them to Scalars::lv_pub (one
//                    word, common.h lv_word), which the other waves poll in
//                    device memory;
//   other waves:     group g = wave, wave + waves, ... once published.
// Every wave leaves when the host's final word says its groups are past the
// batch, when the host cancels, or after LIVE_TIMEOUT (the poller fails the
// batch).  Nothing is left for detectConflicts to place: the writes and their
// sort records went to the gapped slots from A.wbase, and the per-batch resets
// ran in the prologue.
struct LiveArgs {
    IngestArgs A;      // T, R: the live capacities (the real counts come with the final word)
    SortJobs J;        // job 1's splitters (rounds mode: the read begins are not sorted)
    StagedBatch S;     // stream, toff: host-mapped; view: the batch view's arrays (capacity layout)
    LiveOut O;
    // host-mapped: [0] published T, [2] state, [3..5] final T, R, W (stage.h);
    // [6] the poller's timeout mark (written here, read by TxnStage::finish)
    uint64_t* prog;
    uint64_t timeout;      // wall_clock64 ticks (100 MHz)
    uint32_t gen;          // this live batch's generation (tags lv_pub)
    bool spec;             // the speculative window of the last groups (LiveTune)
};
// (LiveTune::blocks: 128 = 511 worker waves; 64: 1-2 us slower per window, 32: 12 us)

// Polling (MI355X_MICROARCH.md, inter-workgroup visibility): relaxed
// agent-scope loads and stores (sc1: past this CU's L1) for the mirrored
// word, relaxed system-scope loads of the host's words, the group's offsets
// and its records (host_load above), and a system-scope acquire only before a
// plain load of the stream past the window.  Acquire loads in the poll loops
// (an L1 invalidate per poll in up to 511 waves) held the kernel ~45 us
// behind the adds at config 2; an acquire per group cost 0.8-2.4 us on the
// last group.
template <class T>
__device__ inline T lv_load(const T* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ inline void lv_store(T* p, T v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(STG_BLOCK) void k_live_ingest(LiveArgs V) {
    __shared__ StgShared L;
    __shared__ uint64_t sp1[SS_MAXB];  // job 1's (live batches are in rounds mode: J.nb[0] = 0, no job 0)
    __shared__ __attribute__((aligned(16))) uint8_t win[STG_BLOCK / 64][LIVE_WIN];
    Scalars* sc = V.A.sc;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int wid = (int)blockIdx.x * (STG_BLOCK / 64) + wv;
    splitter_fill(V.J, 1, sp1);  // (every wave, the poller's too, before the barrier)
    if (blockIdx.x == 0 && threadIdx.x == 0) {  // the per-batch resets (k_ingest_staged's)
        sc->n_comb = 0;
        sc->n_comb_own = 0;
        sc->ss_resample = 0;
        sc->ss_maxc = 0;
    }
    __syncthreads();
    {  // bmax2 of the directory this batch's read check uses (the previous
       // batch's update ran before this kernel): off the path after the adds
        const int D = sc->D;
        for (int k = (int)blockIdx.x; k * BMAX2_SPAN < D; k += (int)gridDim.x) {
            bmax2_block(V.A.hd, D, k);
            __syncthreads();  // (bmax2_block's LDS is reused by the next word)
        }
    }
    const uint32_t gen = V.gen & 0x3FF;
    if (wid == 0) {  // the poller
        if (lane == 0) {
            const uint64_t t_start = wall_clock64();
            PSET(sc, 13);
            int64_t last = -1;
            for (;;) {
                // (the three words in one round trip: independent loads)
                const uint64_t st = host_load(V.prog + 2);
                const uint64_t pw = host_load(V.prog);  // (one word: the count and the bytes stay consistent)
                const int64_t pub = (int64_t)(pw & 0xFFFFF);
                const uint64_t used = (pw & ~LV_FINAL_BIT) >> 20;
                if (pw & LV_FINAL_BIT) {  // the batch is whole: its last T and bytes are this word's
                    PSET(sc, 10);
                    lv_store(&sc->lv_pub, lv_word(gen, LV_FINAL, (uint64_t)pub, used));
                    // (then the read and write counts, a round trip later, off the workers' path)
                    const int32_t R = (int32_t)host_load(V.prog + 4), W = (int32_t)host_load(V.prog + 5);
                    lv_store(&sc->lv_R, R);
                    lv_store(&sc->lv_W, W);
                    if (pub <= (int64_t)V.O.capT) {
                        V.S.view.ro[pub] = R;
                        V.S.view.wo[pub] = W;
                    } else {
                        atomicCAS(&sc->err, 0, FDBCS_E_STATE);
                    }
                    break;
                }
                if (st != LV_RUNNING) {
                    PSET(sc, 10);
                    uint64_t w = lv_word(gen, LV_CANCEL, 0, 0);
                    if (st == LV_FINAL) {
                        // (the final counts and bytes: written before the state word)
                        const uint64_t T = host_load(V.prog + 3);
                        const int32_t R = (int32_t)host_load(V.prog + 4), W = (int32_t)host_load(V.prog + 5);
                        lv_store(&sc->lv_R, R);
                        lv_store(&sc->lv_W, W);
                        w = lv_word(gen, LV_FINAL, T, host_load(V.prog + 1));
                        if (T <= (uint64_t)V.O.capT) {
                            V.S.view.ro[T] = R;
                            V.S.view.wo[T] = W;
                        } else {
                            atomicCAS(&sc->err, 0, FDBCS_E_STATE);
                        }
                    }
                    lv_store(&sc->lv_pub, w);
                    break;
                }
                if (pub != last) {
                    lv_store(&sc->lv_pub, lv_word(gen, LV_RUNNING, (uint64_t)pub, used));
                    last = pub;
                }
                if (wall_clock64() - t_start > V.timeout) {
                    // Give up, unless the batch became whole meanwhile.  Dekker
                    // with TxnStage::finish (which stores its final word, fences,
                    // then loads this mark): mark, fence, look again.  Either
                    // this look sees the final word (finish the batch as usual;
                    // should the host have seen the mark too, it falls back to
                    // the whole-stream ingest, which resets this kernel's work
                    // after it) or the host sees the mark and falls back.
                    __hip_atomic_store(V.prog + 6, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "");
                    if ((host_load(V.prog) & LV_FINAL_BIT) || host_load(V.prog + 2) != LV_RUNNING) continue;
                    atomicCAS(&sc->err, 0, FDBCS_E_STATE);
                    lv_store(&sc->lv_pub, lv_word(gen, LV_TIMEOUT, 0, 0));
                    break;
                }
                __builtin_amdgcn_s_sleep(4);
            }
        }
        return;
    }
    const int nwk = (int)gridDim.x * (STG_BLOCK / 64) - 1;
    for (int g = wid - 1;; g += nwk) {
        const int t0 = g * STG_TPW;
        int tav;
        uint64_t used;
        for (;;) {  // (wave-uniform: one word; another batch's word reads as "nothing yet")
            const uint64_t w0 = lv_load(&sc->lv_pub);
            const uint64_t w = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)w0) |
                               ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(w0 >> 32)) << 32);
            const int st = lv_gen(w) == gen ? lv_state(w) : LV_RUNNING;
            if (st == LV_CANCEL || st == LV_TIMEOUT) return;
            const int pub = lv_gen(w) == gen ? lv_txns(w) : 0;
            if (st == LV_FINAL || pub >= t0 + STG_TPW) {
                tav = pub;
                used = lv_used(w);
                break;
            }
            __builtin_amdgcn_s_sleep(8);
        }
        if (t0 >= tav) {
            if (lane == 0) PMAX(sc, 11);
            return;
        }
        LiveOut O = V.O;
        // (the published bytes end on a 128-byte line, at least 16 bytes past
        // the last record: encode_key's aligned reads around its last key
        // stay inside)
        O.stream_cap = min(O.stream_cap, used);
        O.valid = used;
        if (lane == 0) PMAX(sc, 20);
        if (lane == 0) PMAX(sc, 21);
        // a group among the last published ones: its records end at most
        // `used`, so the window's last LIVE_WIN bytes are read together with
        // the offsets (one round trip instead of two)
        O.spec = V.spec && tav - t0 <= 2 * STG_TPW;
        staged_group<true, true>(V.A, V.J, V.S, O, t0, min(STG_TPW, tav - t0), L, sp1, sp1, win[wv]);
        if (lane == 0) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            PMAX(sc, 23);
        }
    }
}

// a failed live batch: its sort counters (this parity), load-metrics entries,
// tails and flags back to a batch's start
__global__ void k_live_reset(int32_t* cnt, Scalars* sc) {
    for (int k = threadIdx.x; k < SS_CNT; k += blockDim.x) cnt[k] = 0;
    if (threadIdx.x == 0) {
        sc->ss_over[0] = sc->ss_over[1] = 0;
        sc->lm_count = 0;
        sc->lm_bytes = 0;
        sc->btail_used = 0;
        sc->lv_err = 0;
        sc->err = 0;
    }
}

// quantile q of the sorted output sits at position floor(q * n / SS_Q)
__device__ inline void emit_quantiles(const SortJobs& J, int job, int64_t pos, const SRec& x,
                                      const uint8_t* const* tails) {
    const int64_t n = J.n[job];
    for (int64_t q = (pos * SS_Q + n - 1) / n; q < SS_Q && (q * n) / SS_Q == pos; q++)
        put_quantile(J, job, (int)q, x, tails);
}

// One bucket of the sample sort by one 64-lane workgroup (bid < nb[0] + nb[1]).
__device__ void ss_bucket_wave(const SortJobs& J, const KeyArrays& keys, int bid, uint64_t* s_buf) {
    uint64_t *s_hi = s_buf, *s_lo = s_buf + SS_ROW, *s_mi = s_buf + 2 * SS_ROW;  // LDS path
    uint4* s_r4 = reinterpret_cast<uint4*>(s_buf);  // rank path: 32-byte records
    static_assert(3 * SS_ROW * 8 >= 2 * (SS_WAVE + 8) * 16, "rank path staging");
    const int nbk = J.nb[0] + J.nb[1];
    const int job = bid < J.nb[0] ? 0 : 1;
    const int b = job ? bid - J.nb[0] : bid;
    const int lane = threadIdx.x;
    const int32_t* cnt = J.cnt + job * SS_MAXB;
    const uint8_t* const* tails = keys.tail;
    const int64_t c0 = PCLK();
    for (int k = bid * 64 + lane; k < SS_CNT; k += nbk * 64) J.cnt_next[k] = 0;
    // offset = counts of the earlier buckets: lane L sums counts [16L, 16L+16)
    // below b with four independent 16-byte loads (one round trip)
    int part = 0;
    {
        const int4* c4 = reinterpret_cast<const int4*>(cnt) + 4 * lane;
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int4 x = c4[v];
            const int k0 = 16 * lane + 4 * v;
            part += (k0 < b ? x.x : 0) + (k0 + 1 < b ? x.y : 0) + (k0 + 2 < b ? x.z : 0) + (k0 + 3 < b ? x.w : 0);
        }
    }
    const int offset = wave_reduce_sum(part);
    const int c = cnt[b];
    const int64_t c1 = PCLK();
    if (c == 0) return;
    // the write cover before this bucket: the cover deltas of the earlier buckets
    const bool cover = job && J.wcov;
    int doff = 0;
    if (cover) {
        const int4* d4 = reinterpret_cast<const int4*>(J.dcnt) + 4 * lane;
        int dp = 0;
#pragma unroll
        for (int v = 0; v < 4; v++) {
            const int4 x = d4[v];
            const int k0 = 16 * lane + 4 * v;
            dp += (k0 < b ? x.x : 0) + (k0 + 1 < b ? x.y : 0) + (k0 + 2 < b ? x.z : 0) + (k0 + 3 < b ? x.w : 0);
        }
        doff = wave_reduce_sum(dp);
    }
    auto delta = [](uint32_t idx) { return (idx & 1) ? -1 : 1; };  // (a write begin opens, an end closes)
    SRec* out = J.out[job] + offset;
    const SRec* row = J.tmp + ((int64_t)job * SS_MAXB + b) * SS_ROW;
    if (c <= SS_WAVE) {
        // rank sort: the bucket's records go to LDS, every lane ranks its
        // (up to two) records against all c of them -- the order is total, so
        // ranks are distinct.  Broadcast LDS reads, no exchange network.
        SRec x[2];
#pragma unroll
        for (int q = 0; q < 2; q++) {
            const int e = lane + 64 * q;
            if (e < c) {
                x[q] = row[e];
                s_r4[2 * e] = make_uint4((uint32_t)x[q].hi, (uint32_t)(x[q].hi >> 32), (uint32_t)x[q].lo,
                                         (uint32_t)(x[q].lo >> 32));
                s_r4[2 * e + 1] = make_uint4(x[q].meta, x[q].idx, (uint32_t)x[q].pad, (uint32_t)(x[q].pad >> 32));
            }
        }
        // Long-key buckets (config 4: a 64-byte tenant prefix): when every
        // record ties on its first 17 bytes, each compare below would read two
        // tails from global memory.  Instead the tail words all records share
        // are skipped once -- W: the first tail word where some record differs
        // from record 0 -- and the 16 bytes from there rank the records from
        // LDS (zero past a key's end; equal words and both keys ending inside
        // them: length, then the tie rule; a key longer than that: the full
        // compare).
        const uint64_t h0 = __shfl(x[0].hi, 0), l0 = __shfl(x[0].lo, 0);
        const uint32_t m0 = (uint32_t)__shfl((int)x[0].meta, 0), i0 = (uint32_t)__shfl((int)x[0].idx, 0);
        bool same = true;
#pragma unroll
        for (int q = 0; q < 2; q++)
            if (lane + 64 * q < c)
                same &= (x[q].hi == h0) & (x[q].lo == l0) & ((x[q].meta >> 24) == (m0 >> 24)) &
                        (key_len(x[q].meta) > 17);
        const bool longb = c > 1 && key_len(m0) > 17 && __ballot(!same) == 0;  // (wave-uniform)
        // (LW ranked words: 32 bytes past the shared ones, so that a point
        // write's k and k\x00 -- equal words, zero-padded -- are told apart by
        // their lengths for keys up to 32 bytes past W, not by a full compare)
        constexpr int LW = 4;
        uint64_t* s_t = s_buf + 4 * (SS_WAVE + 8);  // (after the records' 2 uint4 each, read 8 past c)
        static_assert(4 * (SS_WAVE + 8) + LW * (SS_WAVE + 8) <= 3 * SS_ROW, "long-key staging");
        uint64_t xt[2][LW] = {};
        uint32_t lim = 0;  // keys up to this long end inside the ranked words
        if (longb) {
            auto tail_words = [](uint32_t meta) { return (key_len(meta) - 17 + 7) >> 3; };
            const uint64_t pd0 = __shfl(x[0].pad, 0);  // (record 0's tail: its scatter's pointer, or the key arrays')
            const uint64_t* t0 = reinterpret_cast<const uint64_t*>(pd0 ? reinterpret_cast<const uint8_t*>(pd0)
                                                                         : tails[i0]);
            const uint32_t n0 = tail_words(m0);
            uint32_t wmin = 0xFFFFFFFFu;
#pragma unroll
            for (int q = 0; q < 2; q++) {
                if (lane + 64 * q >= c) continue;
                const uint64_t* t = reinterpret_cast<const uint64_t*>(rec_tail(x[q], tails));
                const uint32_t nm = min(tail_words(x[q].meta), n0);
                uint32_t w = 0;
                while (w < nm) {  // (four independent loads a step)
                    uint64_t a[4], z[4];
#pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const bool ok = w + k < nm;
                        a[k] = ok ? t[w + k] : 0;
                        z[k] = ok ? t0[w + k] : 0;
                    }
                    int d = 4;
#pragma unroll
                    for (int k = 3; k >= 0; k--)
                        if (a[k] != z[k]) d = k;
                    if (d < 4) {
                        w += d;
                        break;
                    }
                    w += 4;
                }
                wmin = min(wmin, min(w, nm));
            }
            const uint32_t W = wave_reduce_min(wmin);
            lim = 17 + 8 * (W + LW);
#pragma unroll
            for (int q = 0; q < 2; q++) {
                const int e = lane + 64 * q;
                if (e >= c) continue;
                const uint64_t* t = reinterpret_cast<const uint64_t*>(rec_tail(x[q], tails));
                const uint32_t n = tail_words(x[q].meta);
#pragma unroll
                for (int k = 0; k < LW; k++) {
                    xt[q][k] = W + k < n ? __builtin_bswap64(t[W + k]) : 0;
                    s_t[LW * e + k] = xt[q][k];
                }
            }
        }
        const int64_t c2 = PCLK();
        const int64_t c2b = c2;
        __syncthreads();
        // (a long-key bucket's order from the ranked words: -1 / 1, or 0 when
        // they tie and a key runs past them -- resolved after the loop, every
        // lane's ties at once, instead of a wave-wide stall on each record a
        // lane ties with: a point write's begin k and end k\x00 always do)
        auto long_cmp = [&](const uint64_t* aw, const SRec& a, const uint64_t* bw, const SRec& bb) {
#pragma unroll
            for (int k = 0; k < LW; k++)
                if (aw[k] != bw[k]) return aw[k] < bw[k] ? -1 : 1;
            const uint32_t la = key_len(a.meta), lb = key_len(bb.meta);
            if (la > lim || lb > lim) return 0;
            if (la != lb) return la < lb ? -1 : 1;
            const uint32_t pa = a.idx & 1, pb = bb.idx & 1;
            return (pa != pb ? pa > pb : a.idx < bb.idx) ? -1 : 1;
        };
        int rank[2] = {0, 0}, dsum[2] = {0, 0};
        auto rec_at = [&](int j) {
            const uint4 a = s_r4[2 * j], m = s_r4[2 * j + 1];
            return SRec{(uint64_t)a.x | ((uint64_t)a.y << 32), (uint64_t)a.z | ((uint64_t)a.w << 32), m.x, m.y,
                        (uint64_t)m.z | ((uint64_t)m.w << 32)};  // (with the tail pointer: rec_tail)
        };
        if (!longb) {
            for (int j0 = 0; j0 < c; j0 += 8) {  // eight records per round: their LDS reads overlap
                SRec y[8];
#pragma unroll
                for (int u = 0; u < 8; u++) y[u] = rec_at(j0 + u);
#pragma unroll
                for (int u = 0; u < 8; u++)
                    if (j0 + u < c)
#pragma unroll
                        for (int q = 0; q < 2; q++) {
                            const bool lt = (lane + 64 * q < c) && rec_lt(y[u], x[q], tails);
                            rank[q] += lt;
                            dsum[q] += lt ? delta(y[u].idx) : 0;
                        }
            }
        } else {
            constexpr int NPEND = 4;
            int pend[2][NPEND], np[2] = {0, 0};
            constexpr int YU = 16 / LW;  // records per round (8 of 4 words each: 193 VGPRs)
            for (int j0 = 0; j0 < c; j0 += YU) {
                SRec y[YU];
                uint64_t yt[YU][LW];
#pragma unroll
                for (int u = 0; u < YU; u++) {
                    y[u] = rec_at(j0 + u);
#pragma unroll
                    for (int k = 0; k < LW; k++) yt[u][k] = s_t[LW * (j0 + u) + k];
                }
#pragma unroll
                for (int u = 0; u < YU; u++)
                    if (j0 + u < c)
#pragma unroll
                        for (int q = 0; q < 2; q++) {
                            bool lt = false;
                            if (lane + 64 * q < c) {
                                const int r = long_cmp(yt[u], y[u], xt[q], x[q]);
                                if (r == 0 && np[q] < NPEND) pend[q][np[q]++] = j0 + u;
                                else lt = r == 0 ? rec_lt(y[u], x[q], tails) : r < 0;
                            }
                            rank[q] += lt;
                            dsum[q] += lt ? delta(y[u].idx) : 0;
                        }
            }
            for (int k = 0; k < NPEND; k++)  // (the ties: full compares, all lanes together)
#pragma unroll
                for (int q = 0; q < 2; q++)
                    if (k < np[q]) {
                        const SRec y = rec_at(pend[q][k]);
                        const bool lt = rec_lt(y, x[q], tails);
                        rank[q] += lt;
                        dsum[q] += lt ? delta(y.idx) : 0;
                    }
        }
        const int64_t c3 = PCLK();
#pragma unroll
        for (int q = 0; q < 2; q++) {
            if (lane + 64 * q < c) {
                out[rank[q]] = x[q];
                if (job) J.out_slot[offset + rank[q]] = x[q].idx;
                if (cover) J.wcov[offset + rank[q]] = doff + dsum[q] + delta(x[q].idx);
                emit_quantiles(J, job, (int64_t)offset + rank[q], x[q], tails);
            }
        }
        if (lane == 0) {
            PACC(J.sc, 24, c1 - c0);
            PACC(J.sc, 25, c2b - c1);
            PACC(J.sc, 26, c3 - c2b);
            PACC(J.sc, 27, PCLK() - c3);
            PACC(J.sc, 28, 1);
        }
        return;
    }
    if (lane == 0) atomicMax(&J.sc->ss_maxc, c);  // (stats: the largest bucket above the register path)
    if (c <= SS_ROW) {
        int P = 1;
        while (P < c) P <<= 1;
        const LdsRecs L{s_hi, s_lo, s_mi};
        for (int k = lane; k < P; k += 64) L.put(k, k < c ? row[k] : rec_inf());
        __syncthreads();
        lds_bitonic(L, P, tails);
        int run = doff;
        for (int k0 = 0; k0 < c; k0 += 64) {
            const int k = k0 + lane;
            SRec x{};
            if (k < c) x = L.get(k);
            if (cover) {  // (every lane: the scan)
                const int inc = wave_incl_scan(k < c ? delta(x.idx) : 0);
                if (k < c) J.wcov[offset + k] = run + inc;
                run += __builtin_amdgcn_readlane(inc, 63);
            }
            if (k >= c) continue;
            out[k] = x;
            if (job) J.out_slot[offset + k] = x.idx;
            emit_quantiles(J, job, (int64_t)offset + k, x, tails);
        }
        return;
    }
    // overflow: members are found through the per-record bucket ids
    const int n = J.n[job];
    const int32_t* bkt = J.bkt + (job ? J.n[0] : 0);
    for (int i = lane; i < n; i += 64) {
        if (bkt[i] != b) continue;
        const SRec x = load_rec(keys, J.sbase[job] + (int64_t)i * J.sstride[job]);
        int rank = 0, dsum = 0;
        for (int j = 0; j < n; j++) {
            if (bkt[j] != b) continue;
            const SRec y = load_rec(keys, J.sbase[job] + (int64_t)j * J.sstride[job]);
            const bool lt = rec_lt(y, x, tails);
            rank += lt;
            dsum += lt ? delta(y.idx) : 0;
        }
        out[rank] = x;
        if (job) J.out_slot[offset + rank] = x.idx;
        if (cover) J.wcov[offset + rank] = doff + dsum + delta(x.idx);
        emit_quantiles(J, job, (int64_t)offset + rank, x, tails);
    }
}

__global__ __launch_bounds__(64) void k_ss_bucket(SortJobs J, KeyArrays keys) {
    __shared__ __attribute__((aligned(16))) uint64_t s_buf[3 * SS_ROW];
    ss_bucket_wave(J, keys, (int)blockIdx.x, s_buf);
}

// The sort's buckets and the history read check of every read in one launch
// of 64-lane workgroups: the read check needs only the encoded keys and the
// history, not the sorted records, so its dependent searches fill the CUs
// while the buckets sort -- one dependent launch fewer on the way to the
// verdicts (the edge lanes, which need the sorted records, follow).
template <bool WIDE>
__global__ __launch_bounds__(64) void k_ss_bucket_rc(SortJobs J, KeyArrays keys, ReadCheckArgs RA, int nbk) {
    __shared__ __attribute__((aligned(16))) uint64_t s_buf[3 * SS_ROW];
    if ((int)blockIdx.x < nbk) {
        ss_bucket_wave(J, keys, (int)blockIdx.x, s_buf);
        return;
    }
    const Group<RC_G> g;
    read_check_group<WIDE>(RA, g, (int)(((blockIdx.x - nbk) * 64 + threadIdx.x) / RC_G));
}

// ---- large batches: merge sort ------------------------------------------
// Past LARGE_T transactions one batch holds millions of endpoints (config 5:
// 5 M read begins, 4 M write endpoints), far beyond what 1,024 buckets of
// <= 512 records can take.  The large-batch sort is a plain merge sort over
// the same total order (rec_lt), so its output is identical:
//   k_ms_tile  : a workgroup bitonic-sorts MS_TILE records in LDS;
//   k_ms_merge : one pass merges sorted runs pairwise -- each workgroup takes
//                MS_CHUNK outputs, finds where its two merge-path diagonals
//                cut the runs (binary searches in global memory), stages the
//                two input pieces in LDS and every lane merges MS_ITEMS
//                outputs from its own diagonal;
//   k_ms_finish: compact slot copy of the write endpoints, the quantiles the
//                next (small) batch splits by, zeroed bucket counters.
// Jobs ping-pong between their output array and a scratch array; the tile
// sort starts in whichever makes the last pass land in the output.
static constexpr int MS_TILE = 2048;
static constexpr int MS_THREADS = 256;
static constexpr int MS_ITEMS = 8;
static constexpr int MS_CHUNK = MS_THREADS * MS_ITEMS;

struct MergeSortArgs {
    int32_t n[2];
    int64_t sbase[2];
    int32_t sstride[2];
    int32_t passes[2];
    SRec* buf[2][2];      // [job][0]: output, [job][1]: scratch
    int32_t blocks0;      // blocks of job 0 in this launch
};

static int ms_passes(int n) {
    int p = 0;
    for (int64_t w = MS_TILE; w < n; w <<= 1) p++;
    return p;
}

// Sort of one MS_TILE tile by its workgroup: every lane sorts its MS_ITEMS
// records in registers (Batcher's 19-comparator network), then log2(MS_THREADS)
// merge rounds through LDS, each lane producing its MS_ITEMS outputs of a pair
// of runs from its merge-path cut.  About 6x fewer LDS operations and 16
// barriers instead of an LDS bitonic network's 66.  On entry r holds the
// lane's records (rec_inf padding), on exit the tile's sorted positions
// [MS_ITEMS * lane, MS_ITEMS * lane + MS_ITEMS).
static_assert(MS_ITEMS == 8 && MS_TILE == MS_THREADS * MS_ITEMS, "tile sort layout");
__device__ inline void cas_rec(SRec& a, SRec& b, const uint8_t* const* tails) {
    if (rec_lt_inf(b, a, tails)) {
        const SRec t = a;
        a = b;
        b = t;
    }
}

__device__ void tile_sort_regs(const LdsRecs& L, SRec (&r)[MS_ITEMS], const uint8_t* const* tails) {
    constexpr int NET[19][2] = {{0, 1}, {2, 3}, {4, 5}, {6, 7}, {0, 2}, {1, 3}, {4, 6}, {5, 7}, {1, 2}, {5, 6},
                                {0, 4}, {1, 5}, {2, 6}, {3, 7}, {2, 4}, {3, 5}, {1, 2}, {3, 4}, {5, 6}};
#pragma unroll
    for (int c = 0; c < 19; c++) cas_rec(r[NET[c][0]], r[NET[c][1]], tails);
    const int t = threadIdx.x;
    for (int w = MS_ITEMS; w < MS_TILE; w <<= 1) {
#pragma unroll
        for (int q = 0; q < MS_ITEMS; q++) L.put(t * MS_ITEMS + q, r[q]);
        __syncthreads();
        const int o = t * MS_ITEMS;
        const int base = o / (2 * w) * (2 * w), d = o - base;
        const int A = base, B = base + w;
        int lo = max(0, d - w), hi = min(d, w);
        while (lo < hi) {  // (take from A only when strictly below: ties -- padding -- from B)
            const int mid = (lo + hi) >> 1;
            if (rec_lt_inf(L.get(A + mid), L.get(B + d - 1 - mid), tails)) lo = mid + 1;
            else hi = mid;
        }
        int ia = lo, ib = d - lo;
        SRec xa = ia < w ? L.get(A + ia) : rec_inf(), xb = ib < w ? L.get(B + ib) : rec_inf();
#pragma unroll
        for (int q = 0; q < MS_ITEMS; q++) {
            const bool ta = ib >= w || (ia < w && rec_lt_inf(xa, xb, tails));
            if (ta) {
                r[q] = xa;
                ia++;
                xa = ia < w ? L.get(A + ia) : rec_inf();
            } else {
                r[q] = xb;
                ib++;
                xb = ib < w ? L.get(B + ib) : rec_inf();
            }
        }
        __syncthreads();
    }
}

__global__ __launch_bounds__(MS_THREADS) void k_ms_tile(MergeSortArgs M, KeyArrays keys) {
    __shared__ uint64_t s_hi[MS_TILE], s_lo[MS_TILE], s_mi[MS_TILE];
    const int job = (int)blockIdx.x < M.blocks0 ? 0 : 1;
    const int tile = job ? blockIdx.x - M.blocks0 : blockIdx.x;
    const int n = M.n[job];
    const int64_t i0 = (int64_t)tile * MS_TILE;
    const LdsRecs L{s_hi, s_lo, s_mi};
    SRec r[MS_ITEMS];
#pragma unroll
    for (int q = 0; q < MS_ITEMS; q++) {
        const int64_t i = i0 + threadIdx.x * MS_ITEMS + q;
        r[q] = i < n ? load_rec(keys, M.sbase[job] + i * M.sstride[job]) : rec_inf();
    }
    tile_sort_regs(L, r, keys.tail);
    SRec* dst = M.buf[job][M.passes[job] & 1];
#pragma unroll
    for (int q = 0; q < MS_ITEMS; q++) {
        const int64_t i = i0 + threadIdx.x * MS_ITEMS + q;
        if (i < n) dst[i] = r[q];
    }
}

// number of records taken from a (the rest from b) among the first d of the
// merge of sorted a[0, la) and b[0, lb); records are distinct
template <typename GetA, typename GetB>
__device__ inline int merge_path(GetA ga, int la, GetB gb, int lb, int d, const uint8_t* const* tails) {
    int lo = max(0, d - lb), hi = min(d, la);
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (rec_lt(ga(mid), gb(d - 1 - mid), tails)) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// One merge-sort chunk: MS_CHUNK outputs [o0, o0 + MS_CHUNK) of the pass that
// merges runs of width w of src[0, n) into dst[0, n).
__device__ void merge_chunk(const SRec* src, SRec* dst, int n, int64_t w, int64_t o0, const uint8_t* const* tails,
                            const LdsRecs& L, int* s_cut) {
    const int64_t base = o0 / (2 * w) * (2 * w);
    const int la = (int)min<int64_t>(w, n - base);
    const int lb = (int)max<int64_t>(0, min<int64_t>(w, n - base - w));
    const SRec* A = src + base;
    const SRec* B = src + base + la;
    const int d0 = (int)(o0 - base), d1 = min(d0 + MS_CHUNK, la + lb);
    if (threadIdx.x < 2) {
        const int d = threadIdx.x ? d1 : d0;
        s_cut[threadIdx.x] = merge_path([&](int i) { return A[i]; }, la, [&](int i) { return B[i]; }, lb, d, tails);
    }
    __syncthreads();
    const int a0 = s_cut[0], a1 = s_cut[1];
    const int b0 = d0 - a0, b1 = d1 - a1;
    const int na = a1 - a0, nb = b1 - b0;
    for (int k = threadIdx.x; k < na + nb; k += MS_THREADS) L.put(k, k < na ? A[a0 + k] : B[b0 + k - na]);
    __syncthreads();
    const int dl = threadIdx.x * MS_ITEMS;
    if (dl >= na + nb) return;
    int ia = merge_path([&](int i) { return L.get(i); }, na, [&](int i) { return L.get(na + i); }, nb, dl, tails);
    int ib = dl - ia;
    SRec* out = dst + base + d0 + dl;
    const int cnt = min(MS_ITEMS, na + nb - dl);
    for (int k = 0; k < cnt; k++) {
        bool takeA;
        if (ia >= na) takeA = false;
        else if (ib >= nb) takeA = true;
        else takeA = rec_lt(L.get(ia), L.get(na + ib), tails);
        out[k] = takeA ? L.get(ia++) : L.get(na + ib++);
    }
}

__global__ __launch_bounds__(MS_THREADS) void k_ms_merge(MergeSortArgs M, int pass, KeyArrays keys) {
    __shared__ uint64_t s_hi[MS_CHUNK], s_lo[MS_CHUNK], s_mi[MS_CHUNK];
    __shared__ int s_cut[2];
    const int job = (int)blockIdx.x < M.blocks0 ? 0 : 1;
    const int chunk = job ? blockIdx.x - M.blocks0 : blockIdx.x;
    const int P = M.passes[job];
    merge_chunk(M.buf[job][(P - pass) & 1], M.buf[job][(P - pass - 1) & 1], M.n[job], (int64_t)MS_TILE << pass,
                (int64_t)chunk * MS_CHUNK, keys.tail, LdsRecs{s_hi, s_lo, s_mi}, s_cut);
}

__global__ __launch_bounds__(256) void k_ms_finish(MergeSortArgs M, SortJobs J, KeyArrays keys) {
    const int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (g < M.n[1]) J.out_slot[g] = M.buf[1][0][g].idx;
    if (g < 2 * SS_Q) {
        const int job = (int)(g / SS_Q), q = (int)(g % SS_Q);
        const int64_t n = M.n[job];
        if (n > 0) put_quantile(J, job, q, M.buf[job][0][q * n / SS_Q], keys.tail);
    }
    if (g < SS_CNT) J.cnt_next[g] = 0;  // (this path leaves the current parity's counters zero)
}

// Bucketed large-batch sort (steady state: splitters from the previous batch's
// quantiles exist).  The records of each job are first distributed over
// SS_MAXB buckets by the splitters (count, scan, scatter), then every bucket
// is merge-sorted on its own: bucket b needs only ceil(log2(size_b / MS_TILE))
// merge passes instead of the whole job's.  Buckets ping-pong between the
// job's output array and scratch like the jobs of the plain merge sort; a
// bucket's scatter target is the array its tile sort must start in.
static constexpr int LB_MAXP = 16;  // merge passes a bucket may need (2^16 tiles)

static constexpr int LB_RPB = 4096;  // records per count / scatter block (16 per thread)

struct BucketSortArgs {
    SortJobs J;
    SRec* buf[2][2];
    int32_t* hist;  // per-block bucket counts, bucket-major per job: [job base + b * nblk + blk]
    int32_t* hoff;  // their exclusive scan (global positions; job 1's start at n0)
    int32_t* off;   // [2][SS_MAXB + 1] bucket starts
    int32_t* pb;    // [2][SS_MAXB] merge passes per bucket
    int32_t* toff;  // [2][SS_MAXB + 1] tile prefix
    int32_t* coff;  // [LB_MAXP][2][SS_MAXB + 1] merge-chunk prefix of the buckets still merging in pass p
    int32_t* maxp;  // [1]
    int32_t* bkt;   // [n0 + n1]
    int32_t nblk[2];
    int64_t hbase[2];
    int32_t tiles0, chunks0;  // grid split between the jobs (tile, merge launches)
};

__device__ inline int lb_find(const int32_t* pre, int nb, int x) {  // bucket with pre[b] <= x < pre[b + 1]
    int lo = 0, hi = nb;
    while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (pre[mid] <= x) lo = mid;
        else hi = mid;
    }
    return lo;
}

// per-block histograms in LDS (no global atomics: 1,024 hot counters would
// serialize millions of atomics in L2)
__global__ __launch_bounds__(256) void k_lb_count(BucketSortArgs A, KeyArrays keys) {
    __shared__ uint64_t sp[SS_MAXB];
    __shared__ int32_t h[SS_MAXB];
    const SortJobs& J = A.J;
    const int job = (int)blockIdx.x < A.nblk[0] ? 0 : 1;
    const int blk = job ? blockIdx.x - A.nblk[0] : blockIdx.x;
    const int nb = J.nb[job];
    splitter_fill(J, job, sp);
    for (int b = threadIdx.x; b < nb; b += blockDim.x) h[b] = 0;
    __syncthreads();
    const int i1 = min(J.n[job], (blk + 1) * LB_RPB);
    int32_t* bkt = A.bkt + (job ? J.n[0] : 0);
    for (int i = blk * LB_RPB + threadIdx.x; i < i1; i += blockDim.x) {
        const SRec x = load_rec(keys, J.sbase[job] + (int64_t)i * J.sstride[job]);
        const int b = bucket_of(J, job, sp, x, keys.tail);
        bkt[i] = b;
        atomicAdd(&h[b], 1);
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nb; b += blockDim.x) A.hist[A.hbase[job] + (int64_t)b * A.nblk[job] + blk] = h[b];
}

__global__ __launch_bounds__(SS_MAXB) void k_lb_scan(BucketSortArgs A) {
    __shared__ int64_t red[SS_MAXB / 64 + 1];
    const int job = blockIdx.x, b = threadIdx.x;
    const int nb = A.J.nb[job];
    const int n = A.J.n[job];
    const int adj = job ? A.J.n[0] : 0;
    const int o = b < nb ? A.hoff[A.hbase[job] + (int64_t)b * A.nblk[job]] - adj : n;
    const int o1 = b + 1 < nb ? A.hoff[A.hbase[job] + (int64_t)(b + 1) * A.nblk[job]] - adj : n;
    const int c = b < nb ? o1 - o : 0;
    int p = 0;
    for (int64_t w = MS_TILE; w < c; w <<= 1) p++;
    int64_t tot;
    const int64_t to = block_excl_scan((int64_t)cdiv(c, MS_TILE), red, tot);
    if (b < nb) {
        A.off[job * (SS_MAXB + 1) + b] = o;
        A.pb[job * SS_MAXB + b] = p;
        A.toff[job * (SS_MAXB + 1) + b] = (int32_t)to;
        if (p) atomicMax(A.maxp, p);
    }
    if (b == 0) {
        A.off[job * (SS_MAXB + 1) + nb] = n;
        A.toff[job * (SS_MAXB + 1) + nb] = (int32_t)tot;
    }
    for (int q = 0; q < LB_MAXP; q++) {
        const int64_t co = block_excl_scan((int64_t)(p > q ? cdiv(c, MS_CHUNK) : 0), red, tot);
        int32_t* pre = A.coff + ((int64_t)q * 2 + job) * (SS_MAXB + 1);
        if (b < nb) pre[b] = (int32_t)co;
        if (b == 0) pre[nb] = (int32_t)tot;
    }
}

// the same record partition as k_lb_count: each block's slice of a bucket
// starts at its scanned offset; ranks inside the slice by LDS atomics
__global__ __launch_bounds__(256) void k_lb_scatter(BucketSortArgs A, KeyArrays keys) {
    __shared__ int32_t cur[SS_MAXB];
    __shared__ uint8_t par[SS_MAXB];
    const SortJobs& J = A.J;
    const int job = (int)blockIdx.x < A.nblk[0] ? 0 : 1;
    const int blk = job ? blockIdx.x - A.nblk[0] : blockIdx.x;
    const int nb = J.nb[job];
    const int adj = job ? J.n[0] : 0;
    for (int b = threadIdx.x; b < nb; b += blockDim.x) {
        cur[b] = A.hoff[A.hbase[job] + (int64_t)b * A.nblk[job] + blk] - adj;
        par[b] = (uint8_t)(A.pb[job * SS_MAXB + b] & 1);
    }
    __syncthreads();
    const int i1 = min(J.n[job], (blk + 1) * LB_RPB);
    const int32_t* bkt = A.bkt + adj;
    for (int i = blk * LB_RPB + threadIdx.x; i < i1; i += blockDim.x) {
        const int b = bkt[i];
        const int pos = atomicAdd(&cur[b], 1);
        A.buf[job][par[b]][pos] = load_rec(keys, J.sbase[job] + (int64_t)i * J.sstride[job]);
    }
}

__global__ __launch_bounds__(MS_THREADS) void k_lb_tile(BucketSortArgs A, KeyArrays keys) {
    __shared__ uint64_t s_hi[MS_TILE], s_lo[MS_TILE], s_mi[MS_TILE];
    const int job = (int)blockIdx.x < A.tiles0 ? 0 : 1;
    const int tile = job ? blockIdx.x - A.tiles0 : blockIdx.x;
    const int nb = A.J.nb[job];
    const int32_t* toff = A.toff + job * (SS_MAXB + 1);
    if (nb == 0 || tile >= toff[nb]) return;
    const int b = lb_find(toff, nb, tile);
    const int64_t o = A.off[job * (SS_MAXB + 1) + b];
    const int c = A.off[job * (SS_MAXB + 1) + b + 1] - (int)o;
    const int64_t i0 = (int64_t)(tile - toff[b]) * MS_TILE;
    SRec* a = A.buf[job][A.pb[job * SS_MAXB + b] & 1] + o;  // sorted in place
    const LdsRecs L{s_hi, s_lo, s_mi};
    SRec r[MS_ITEMS];
#pragma unroll
    for (int q = 0; q < MS_ITEMS; q++) {
        const int64_t i = i0 + threadIdx.x * MS_ITEMS + q;
        r[q] = i < c ? a[i] : rec_inf();
    }
    tile_sort_regs(L, r, keys.tail);
#pragma unroll
    for (int q = 0; q < MS_ITEMS; q++) {
        const int64_t i = i0 + threadIdx.x * MS_ITEMS + q;
        if (i < c) a[i] = r[q];
    }
}

__global__ __launch_bounds__(MS_THREADS) void k_lb_merge(BucketSortArgs A, int pass, KeyArrays keys) {
    __shared__ uint64_t s_hi[MS_CHUNK], s_lo[MS_CHUNK], s_mi[MS_CHUNK];
    __shared__ int s_cut[2];
    const int job = (int)blockIdx.x < A.chunks0 ? 0 : 1;
    const int chunk = job ? blockIdx.x - A.chunks0 : blockIdx.x;
    const int nb = A.J.nb[job];
    const int32_t* pre = A.coff + ((int64_t)pass * 2 + job) * (SS_MAXB + 1);
    if (nb == 0 || chunk >= pre[nb]) return;
    const int b = lb_find(pre, nb, chunk);
    const int64_t o = A.off[job * (SS_MAXB + 1) + b];
    const int c = A.off[job * (SS_MAXB + 1) + b + 1] - (int)o;
    const int P = A.pb[job * SS_MAXB + b];
    merge_chunk(A.buf[job][(P - pass) & 1] + o, A.buf[job][(P - pass - 1) & 1] + o, c, (int64_t)MS_TILE << pass,
                (int64_t)(chunk - pre[b]) * MS_CHUNK, keys.tail, LdsRecs{s_hi, s_lo, s_mi}, s_cut);
}

int64_t lb_hist_words(int R, int W) {
    return (int64_t)SS_MAXB * (cdiv(R, LB_RPB) + cdiv(2 * (int64_t)W, LB_RPB)) + 1;
}

// returns false when a bucket would need more than LB_MAXP passes (the
// caller falls back to the plain merge sort)
static bool launch_bucket_sort(const SortJobs& J, BatchBufs& b, hipStream_t s) {
    BucketSortArgs A;
    A.J = J;
    for (int j = 0; j < 2; j++) A.buf[j][0] = J.out[j];
    A.buf[0][1] = b.ss_tmp;
    A.buf[1][1] = b.ss_tmp + J.n[0];
    int32_t* m = b.lb_meta;
    A.pb = m;
    A.maxp = m + 2 * SS_MAXB;
    A.off = m + 2 * SS_MAXB + 8;
    A.toff = A.off + 2 * (SS_MAXB + 1);
    A.coff = A.toff + 2 * (SS_MAXB + 1);
    A.bkt = b.ss_bkt;
    A.hist = b.lb_hist;
    A.hoff = b.lb_hist + b.lb_hist_cap;
    for (int j = 0; j < 2; j++) A.nblk[j] = cdiv(J.n[j], LB_RPB);
    A.hbase[0] = 0;
    A.hbase[1] = (int64_t)J.nb[0] * A.nblk[0];
    const int64_t hn = A.hbase[1] + (int64_t)J.nb[1] * A.nblk[1];
    A.tiles0 = J.n[0] ? cdiv(J.n[0], MS_TILE) + J.nb[0] : 0;
    A.chunks0 = J.n[0] ? cdiv(J.n[0], MS_CHUNK) + J.nb[0] : 0;
    hipMemsetAsync(A.maxp, 0, sizeof(int32_t), s);
    const int cblocks = A.nblk[0] + A.nblk[1];
    hipLaunchKernelGGL(k_lb_count, dim3(cblocks), dim3(256), 0, s, A, b.keys);
    scan_i32(A.hist, A.hoff, nullptr, (int32_t)hn, nullptr, b.scan_tmp, s);
    hipLaunchKernelGGL(k_lb_scan, dim3(2), dim3(SS_MAXB), 0, s, A);
    int32_t maxp = 0;
    hipMemcpyAsync(&maxp, A.maxp, sizeof(maxp), hipMemcpyDeviceToHost, s);
    hipStreamSynchronize(s);
    if (maxp > LB_MAXP) return false;
    hipLaunchKernelGGL(k_lb_scatter, dim3(cblocks), dim3(256), 0, s, A, b.keys);
    const int tiles = A.tiles0 + (J.n[1] ? cdiv(J.n[1], MS_TILE) + J.nb[1] : 0);
    hipLaunchKernelGGL(k_lb_tile, dim3(tiles), dim3(MS_THREADS), 0, s, A, b.keys);
    const int chunks = A.chunks0 + (J.n[1] ? cdiv(J.n[1], MS_CHUNK) + J.nb[1] : 0);
    for (int p = 0; p < maxp; p++) hipLaunchKernelGGL(k_lb_merge, dim3(chunks), dim3(MS_THREADS), 0, s, A, p, b.keys);
    MergeSortArgs M;  // (only n and the output arrays matter to the finish)
    for (int j = 0; j < 2; j++) {
        M.n[j] = J.n[j];
        M.buf[j][0] = J.out[j];
    }
    const int64_t fin = std::max<int64_t>(std::max<int64_t>(M.n[1], SS_CNT), 2 * SS_Q);
    hipLaunchKernelGGL(k_ms_finish, dim3(cdiv(fin, 256)), dim3(256), 0, s, M, J, b.keys);
    return true;
}

int64_t lb_meta_words() { return 2 * SS_MAXB + 8 + 4 * (SS_MAXB + 1) + (int64_t)LB_MAXP * 2 * (SS_MAXB + 1); }

static void launch_merge_sort(const SortJobs& J, BatchBufs& b, hipStream_t s) {
    MergeSortArgs M;
    for (int j = 0; j < 2; j++) {
        M.n[j] = J.n[j];
        M.sbase[j] = J.sbase[j];
        M.sstride[j] = J.sstride[j];
        M.passes[j] = ms_passes(J.n[j]);
        M.buf[j][0] = J.out[j];
    }
    M.buf[0][1] = b.ss_tmp;
    M.buf[1][1] = b.ss_tmp + J.n[0];
    M.blocks0 = cdiv(M.n[0], MS_TILE);
    const int tiles = M.blocks0 + cdiv(M.n[1], MS_TILE);
    if (tiles > 0) hipLaunchKernelGGL(k_ms_tile, dim3(tiles), dim3(MS_THREADS), 0, s, M, b.keys);
    const int P = std::max(M.passes[0], M.passes[1]);
    for (int p = 0; p < P; p++) {
        MergeSortArgs Mp = M;
        for (int j = 0; j < 2; j++)
            if (p >= M.passes[j]) Mp.n[j] = 0;  // this job is already sorted (no blocks)
        // (n is kept for the jobs that take part: block counts from their sizes)
        Mp.blocks0 = cdiv(Mp.n[0], MS_CHUNK);
        const int blocks = Mp.blocks0 + cdiv(Mp.n[1], MS_CHUNK);
        hipLaunchKernelGGL(k_ms_merge, dim3(blocks), dim3(MS_THREADS), 0, s, Mp, p, b.keys);
    }
    const int64_t fin = std::max<int64_t>(std::max<int64_t>(M.n[1], SS_CNT), 2 * SS_Q);
    hipLaunchKernelGGL(k_ms_finish, dim3(cdiv(fin, 256)), dim3(256), 0, s, M, J, b.keys);
}

static int ss_buckets(int n) {
    // FDBCS_TEST_SORT_BUCKETS forces few buckets so tests reach the LDS and
    // global-memory bucket paths
    const char* force = getenv("FDBCS_TEST_SORT_BUCKETS");
    if (n <= 0) return 0;
    if (force && atoi(force) > 0) return std::min(atoi(force), SS_MAXB);
    int want = (n + 23) / 24, nb = 1;
    while (nb < want && nb < SS_MAXB) nb <<= 1;
    return nb;
}

// Staging records the sort needs (engine sizes b.ss_tmp).
int64_t sort_staging_records(int R, int W, bool large) {
    const int64_t small = 2 * (int64_t)SS_MAXB * SS_ROW;
    return large ? std::max<int64_t>(small, (int64_t)R + 2 * (int64_t)W) : small;
}

bool large_batch_mode(int64_t T) {
    return T > LARGE_T || getenv("FDBCS_TEST_LARGE_BATCH") != nullptr;  // (tests: the large path at small T)
}

static SortJobs make_sort_jobs(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, int parity) {
    const int R = v.read_count, W = v.write_count;
    SortJobs J;
    J.n[0] = R;
    J.n[1] = 2 * W;
    J.sbase[0] = 0;
    J.sstride[0] = 2;
    J.sbase[1] = write_base(b, v);
    J.sstride[1] = 1;
    J.out[0] = b.rec_r0;
    J.out[1] = b.rec_w0;
    J.out_slot = b.sw_slot;
    J.quant = b.ss_q;
    J.qtail = b.ss_qt;
    J.cnt = b.ss_cnt + parity * SS_CNT;
    J.cnt_next = b.ss_cnt + (parity ^ 1) * SS_CNT;
    J.dcnt = J.cnt + 2 * SS_MAXB;
    J.wcov = nullptr;
    J.bkt = b.ss_bkt;
    J.tmp = b.ss_tmp;
    J.sc = sc;
    if (b.rounds && !b.large) {
        // rounds mode: the read begins are not sorted -- the decision needs per
        // read only its place among the sorted write endpoints, and whether
        // some write covers its begin (the write cover, wcov), not the reads'
        // own order (DESIGN.md §4 "Write cover")
        J.n[0] = 0;
        J.wcov = b.wcov;
    }
    for (int j = 0; j < 2; j++) J.nb[j] = ss_buckets(J.n[j]);
    if (b.lv_wbase && b.lv_nb1) J.nb[1] = b.lv_nb1;  // (a live batch: the buckets k_live_ingest scattered into)
    J.blocks0 = cdiv(J.n[0], 256);
    return J;
}

// Per-transaction staging stream -> batch view (kernels.h StageHdr).  Lane t
// places its reads at slots 2(ro + k) and its writes at 2R + 2(wo + k): the
// slot layout every later stage addresses (include/fdbcs.h fdbcs_batch_view).
__global__ __launch_bounds__(256) void k_unpack(const uint8_t* __restrict__ stream,
                                                const uint64_t* __restrict__ toff, int T, int R, int W,
                                                UnpackOut o) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t > T) return;
    if (t == T) {
        o.ro[T] = R;
        o.wo[T] = W;
        return;
    }
    const StageTxn h = stage_txn(stream, toff[t]);
    const uint64_t base = h.base;
    o.snap[t] = h.snap;
    o.ro[t] = h.ro;
    o.wo[t] = h.wo;
    const StageRange* ent = reinterpret_cast<const StageRange*>(stream + base + sizeof(StageHdr));
    for (int k = 0; k < h.nr + h.nw; k++) {
        const StageRange e = ent[k];
        const int64_t slot = k < h.nr ? 2ll * (h.ro + k) : 2ll * R + 2ll * (h.wo + k - h.nr);
        o.koff[slot] = base + e.kofs;
        o.klen[slot] = e.blen;
        o.koff[slot + 1] = base + stage_end_ofs(e);
        o.klen[slot + 1] = stage_end_len(e);
    }
}

// The stream's rest (after the last chunk copy) read by the engine's own
// queue from the host-mapped pinned buffer: 8-byte words, one per lane
// (FDBCS_PULL_REST; stage.hip)
__global__ __launch_bounds__(256) void k_pull(const uint64_t* __restrict__ src, uint64_t* __restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

void launch_pull(const uint8_t* host_src, uint8_t* dst, uint64_t bytes, hipStream_t s) {
    const int64_t n = (int64_t)((bytes + 7) / 8);
    if (n <= 0) return;
    const int nb = (int)std::min<int64_t>(256, (n + 255) / 256);
    hipLaunchKernelGGL(k_pull, dim3(nb), dim3(256), 0, s, reinterpret_cast<const uint64_t*>(host_src),
                       reinterpret_cast<uint64_t*>(dst), n);
}

void launch_unpack(const uint8_t* stream, const uint64_t* toff, int T, int R, int W, UnpackOut o, hipStream_t s) {
    hipLaunchKernelGGL(k_unpack, dim3(cdiv((int64_t)T + 1, 256)), dim3(256), 0, s, stream, toff, T, R, W, o);
}

void launch_ingest(const fdbcs_batch_view& v, int64_t oldest, BatchBufs& b, Scalars* sc, bool scatter, int parity,
                   const Dir& hd, hipStream_t s, bool sharded, const LmArgs* lm) {
    constexpr int IB = FDBCS_INGEST_BLOCK;  // (A/B: scripts/build_variants.sh)
    IngestArgs A;
    A.lm = lm && b.staged.stream ? *lm : LmArgs{};  // (k_ingest, the view path, does not roll)
    A.T = v.txn_count; A.R = v.read_count; A.W = v.write_count;
    A.wbase = write_base(b, v);
    A.prep_blocks = std::max(1, cdiv(v.txn_count, IB));
    A.snap = v.snapshot; A.ro = v.read_off; A.wo = v.write_off;
    A.koff = v.key_off; A.klen = v.key_len; A.bytes = v.key_bytes;
    A.oldest = oldest; A.too_old = b.too_old; A.hist = b.hist; A.read_txn = b.read_txn; A.read_snap = b.read_snap;
    A.write_txn = b.write_txn;
    A.keys = b.keys; A.btail = b.btail; A.btail_cap = b.btail_cap; A.sc = sc; A.deg = b.deg;
    A.hd = hd;
    A.bmax2_blocks = v.read_count > 0 ? cdiv(hd.cap, BMAX2_SPAN) : 0;  // (D <= cap; idle blocks exit)
    (void)sharded;
    const int blocks = A.prep_blocks + A.bmax2_blocks + cdiv((int64_t)v.read_count + v.write_count, IB);
    const SortJobs J = make_sort_jobs(v, b, sc, parity);
    if (b.staged.stream) {  // the per-transaction path: straight from the record stream
        const int sb = std::max(1, cdiv(cdiv((int64_t)v.txn_count, STG_TPW), STG_BLOCK / 64));
        if (scatter)
            hipLaunchKernelGGL(k_ingest_staged<true>, dim3(sb + A.bmax2_blocks), dim3(STG_BLOCK), 0, s, A, J, b.staged, sb);
        else
            hipLaunchKernelGGL(k_ingest_staged<false>, dim3(sb + A.bmax2_blocks), dim3(STG_BLOCK), 0, s, A, J, b.staged, sb);
        return;
    }
    if (scatter)
        hipLaunchKernelGGL(k_ingest<true>, dim3(blocks), dim3(IB), 0, s, A, J);
    else
        hipLaunchKernelGGL(k_ingest<false>, dim3(blocks), dim3(IB), 0, s, A, J);
}

void launch_live_ingest(BatchBufs& b, Scalars* sc, const LiveCaps& caps, int64_t oldest, int parity,
                        const uint8_t* stream, uint64_t stream_cap, const uint64_t* toff, const uint64_t* prog,
                        UnpackOut view, const LmArgs* lm, uint32_t gen, const Dir& hd, const LiveTune& tune,
                        hipStream_t s) {
    IngestArgs A{};
    A.hd = hd;
    A.T = caps.T; A.R = caps.R; A.W = caps.W;
    A.oldest = oldest; A.too_old = b.too_old; A.hist = b.hist; A.read_txn = b.read_txn; A.read_snap = b.read_snap;
    A.write_txn = b.write_txn;
    A.keys = b.keys; A.btail = b.btail; A.btail_cap = b.btail_cap; A.sc = sc; A.deg = b.deg;
    A.lm = lm ? *lm : LmArgs{};
    fdbcs_batch_view vc{};
    vc.read_count = caps.R;
    vc.write_count = caps.W;
    b.lv_wbase = 2 * (int64_t)caps.R;  // (the writes' slots and job 1's buckets hold until the batch's detect)
    b.lv_nb1 = 0;
    A.wbase = b.lv_wbase;
    const SortJobs J = make_sort_jobs(vc, b, sc, parity);
    b.lv_nb1 = J.nb[1];
    StagedBatch S;
    S.stream = stream;
    S.toff = toff;
    S.view = view;
    S.live = true;
    const LiveOut O{caps.T, caps.R, caps.W, stream_cap};
    const LiveArgs V{A, J, S, O, const_cast<uint64_t*>(prog), tune.timeout_ticks, gen, tune.spec};
    hipLaunchKernelGGL(k_live_ingest, dim3(std::max(2, tune.blocks)), dim3(STG_BLOCK), 0, s, V);
}

void launch_live_reset(BatchBufs& b, Scalars* sc, int parity, hipStream_t s) {
    hipLaunchKernelGGL(k_live_reset, dim3(1), dim3(256), 0, s, b.ss_cnt + parity * SS_CNT, sc);
}

bool launch_sort_ranges(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, bool sample, int parity,
                        bool scattered, hipStream_t s, HistBufs* h, int cur, int64_t v0, bool guard) {
    const SortJobs J = make_sort_jobs(v, b, sc, parity);
    b.sr = b.rec_r0;
    b.sw = b.rec_w0;
    b.rc_fused = false;
    if (J.n[0] + J.n[1] == 0) return false;
    if (b.large) {  // bucketed merge sort once splitters exist; the plain merge sort on the first batch
        static const bool plain = getenv("FDBCS_LARGE_SORT_PLAIN") != nullptr;  // (A/B measurements)
        if (sample || plain || !launch_bucket_sort(J, b, s)) launch_merge_sort(J, b, s);
        return true;
    }
    if (!scattered) {  // (otherwise the ingest already put every record into its bucket)
        if (sample) hipLaunchKernelGGL(k_ss_sample, dim3(2), dim3(1024), 0, s, J, b.keys, 0);
        hipLaunchKernelGGL(k_ss_scatter, dim3(J.blocks0 + cdiv(J.n[1], 256)), dim3(256), 0, s, J, b.keys);
    }
    if (guard || !scattered)
        hipLaunchKernelGGL(k_ss_guard, dim3(2), dim3(1024), 0, s, J, b.keys, b.ss_gsamp);  // overflow guard
    const int nbk = J.nb[0] + J.nb[1];
    static const bool separate = getenv("FDBCS_SEPARATE_READ_CHECK") != nullptr;  // (A/B measurements)
    const int R = v.read_count;
    if (h && R > 0 && !b.dir_join && !separate) {  // the history read check rides in the buckets' launch
        const ReadCheckArgs RA{R, b.keys, b.read_txn, b.read_snap, b.hist, h->pool, h->dir[cur], sc, v0, h->shard,
                               nullptr};
        const int rc_blocks = cdiv((int64_t)R * RC_G, 64);
        if (FDBCS_RC_WIDE)
            hipLaunchKernelGGL(k_ss_bucket_rc<true>, dim3(nbk + rc_blocks), dim3(64), 0, s, J, b.keys, RA, nbk);
        else
            hipLaunchKernelGGL(k_ss_bucket_rc<false>, dim3(nbk + rc_blocks), dim3(64), 0, s, J, b.keys, RA, nbk);
        b.rc_fused = true;
        return true;
    }
    hipLaunchKernelGGL(k_ss_bucket, dim3(nbk), dim3(64), 0, s, J, b.keys);
    return true;  // the counters of the other parity are zero now
}

// --------------------------------------------------------------- edges ----
// Large and sparse (sharded protocol B) batches list the overlap pairs.
// A read r of t and a write w of u overlap iff r.b < w.e && w.b < r.e.
// Split on which begin comes first (keys only, no ranks):
//   w.b >= r.b : the write begins among the sorted write endpoints with key in
//                [r.b, r.e)                                       (by reader)
//   w.b <  r.b : the read begins with key in (w.b, w.e)           (by writer)
// Only pairs u < t where both are still undecided (not tooOld, no history
// conflict) matter; each is appended to (et, eu) through one global counter
// (duplicates kept).  Other batches only search each read's position among
// the sorted write endpoints (rounds_lane) for k_decide_rounds.
__device__ inline int lb_key(const SRec* a, int n, const Key& k, const uint8_t* const* tails) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (rec_vs_key(a[mid], k, tails) < 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}
__device__ inline int ub_key(const SRec* a, int n, const Key& k, const uint8_t* const* tails) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (rec_vs_key(a[mid], k, tails) <= 0) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// an overlap pair (reader t, earlier writer u); duplicates are kept (they
// only repeat a source in the decision's CSR)
__device__ inline void edge_pair(int t, int u, int32_t* et, int32_t* eu, int64_t cap, Scalars* sc, int32_t* deg) {
    atomicAdd(&deg[t], 1);  // (sources per reader, for the grid decision; zeroed by the ingest)
    const int idx = atomicAdd(&sc->edges_total, 1);
    if (idx < cap) {
        et[idx] = t;
        eu[idx] = u;
    }
}

// Where write w's begin and end fall in the pre-batch history, searched
// speculatively for every write (the merge plan later picks the writes that
// open and close each combined range, k_plan_ranges).
struct WriteSearchArgs {
    int R, W;
    KeyArrays keys;
    Pool pool;
    Dir dir;
    const Scalars* sc;
    int64_t v0;
    WriteHits wh;
    const int32_t* qx;  // large batches: directory entry of every write endpoint (k_dir_join; index R + slot - 2R)
    int64_t wbase;      // slot of write 0's begin (write_base)
};

__device__ inline void write_search_group(const WriteSearchArgs& A, const Group<RC_G>& g, int w) {
    if (w >= A.W) return;
    const int64_t s = A.wbase + 2 * (int64_t)w;
    const Key b = A.keys.get(s), e = A.keys.get(s + 1);
    const int D = A.sc->D;
    DirHit hb, he;
    if (A.qx) {
        const int xb = A.qx[A.R + 2 * w], xe = A.qx[A.R + 2 * w + 1];
        hb = DirHit{xb, A.dir.page[xb], A.dir.cnt[xb]};
        he = DirHit{xe, A.dir.page[xe], A.dir.cnt[xe]};
    }
    const bool px = FDBCS_DIR_PX && A.sc->px_on;  // (long keys: the searches' prefix skips)
    if (!A.qx) {
        if (px) grp_dir_find2<true>(g, A.dir, D, b, e, hb, he);
        else grp_dir_find2<false>(g, A.dir, D, b, e, hb, he);
    }
    int ib, ie;
    bool eqb, eqe;
    if (px) grp_page_find2<true>(g, A.pool, A.dir, hb.x, hb.page, hb.cnt, b, he.x, he.page, he.cnt, e, ib, eqb, ie, eqe);
    else grp_page_find2<false>(g, A.pool, A.dir, hb.x, hb.page, hb.cnt, b, he.x, he.page, he.cnt, e, ib, eqb, ie, eqe);
    if (g.lane != 0) return;
    uint64_t hmb[HM_WORDS], hme[HM_WORDS];  // real positions for the merge plan's counts (holes, common.h)
    load_hmask(A.pool, hb.page, hmb);
    load_hmask(A.pool, he.page, hme);
    const int nrb = A.dir.nr[hb.x];
    int64_t vb;
    bool from_v0 = false;  // no boundary below e: the header version (sharded: the carry-in)
    if (ie > 0) vb = A.pool.ver[(int64_t)he.page * PAGE + ie - 1];
    else if (he.x > 0 && A.dir.cnt[he.x - 1] > 0)
        vb = A.pool.ver[(int64_t)A.dir.page[he.x - 1] * PAGE + A.dir.cnt[he.x - 1] - 1];
    else vb = A.v0, from_v0 = true;  // (only entry 0 can be an empty page)
    A.wh.b[w] = WHitB{hb.x, ib, nrb, real_before(hmb, ib)};
    // (feq bit 1: the merge substitutes its own v0)
    A.wh.e[w] = WHitE{vb, he.x, ie, real_before(hme, ie), (int32_t)(eqe | from_v0 << 1), 0};
}

// Edges need not skip transactions that already conflict with the history:
// a conflicting reader is aborted whatever its sources, and a conflicting
// writer never commits, so its edges never fire (k_decide_combine).  That
// keeps the edges independent of the read check, so both run in one launch.
struct EdgesArgs {
    int R, W;
    KeyArrays keys;
    const SRec* sr;
    const SRec* sw;
    const int32_t* read_txn;
    const int32_t* write_txn;
    const uint8_t* too_old;
    int32_t* et;
    int32_t* eu;
    int64_t cap;
    Scalars* sc;
    int32_t* deg;
    // rounds mode (k_decide_rounds): no pairs; per read the sorted write
    // endpoints at or below its begin / below its end, per sorted write
    // endpoint whether its key differs from the previous one's
    int32_t* rq;     // [2R] or null (edges mode)
    uint8_t* wnew;   // [2W]
    int32_t* plist;  // candidate reads (appended at sc->n_pot; duplicates allowed)
    int64_t plist_cap;
    int32_t* winv;   // [2W] sorted position of each write endpoint
    const int32_t* wcov;  // [2W] write cover at each sorted write endpoint (rounds mode)
    uint32_t* rstamp;  // [R] batch stamp of reads already on plist
    uint32_t rseq;     // this batch's stamp
    int64_t wbase;     // slot of write 0's begin (write_base)
};

// The two searches of an edge lane: an LDS sample of the sorted array's first
// key words (EQ evenly spaced records, loaded by the block) narrows each key
// to ~n/EQ records, then both keys are binary-searched in lockstep so their
// loads overlap.
constexpr int EQ = 1024;

__device__ inline void sample_fill(uint64_t* smp, const SRec* a, int n) {
    const int m = min(n, EQ);
    for (int q = threadIdx.x; q < m; q += blockDim.x) smp[q] = a[(int64_t)q * n / m].hi;
}

// [lo, hi) of a[0, n) that holds every record whose key word equals k.hi
// (records before lo are < k, records from hi on are > k)
__device__ inline void sample_narrow(const uint64_t* smp, int n, uint64_t h, int& lo, int& hi) {
    const int m = min(n, EQ);
    int a = 0, len = m;  // c_lt = #samples < h
    while (len > 0) {
        const int half = len >> 1;
        if (smp[a + half] < h) { a += half + 1; len -= half + 1; }
        else len = half;
    }
    int b = a;  // c_le = #samples <= h
    if (b < m && smp[b] == h) {
        len = m - b;
        while (len > 0) {
            const int half = len >> 1;
            if (smp[b + half] <= h) { b += half + 1; len -= half + 1; }
            else len = half;
        }
    }
    lo = a > 0 ? (int)((int64_t)(a - 1) * n / m) + 1 : 0;
    hi = b < m ? (int)((int64_t)b * n / m) : n;
}

// first i in [lo, hi) with a[i] >= k (strict1: > k1) for two keys at once
__device__ inline void bsearch2(const SRec* a, const Key& k1, bool strict1, int lo1, int hi1, const Key& k2, int lo2,
                                int hi2, const uint8_t* const* tails, int& r1, int& r2) {
    while (lo1 < hi1 || lo2 < hi2) {
        const int m1 = (lo1 + hi1) >> 1, m2 = (lo2 + hi2) >> 1;
        const bool a1 = lo1 < hi1, a2 = lo2 < hi2;
        SRec x1, x2;
        if (a1) x1 = a[m1];
        if (a2) x2 = a[m2];
        if (a1) {
            const int c = rec_vs_key(x1, k1, tails);
            if (strict1 ? c <= 0 : c < 0) lo1 = m1 + 1;
            else hi1 = m1;
        }
        if (a2) {
            if (rec_vs_key(x2, k2, tails) < 0) lo2 = m2 + 1;
            else hi2 = m2;
        }
    }
    r1 = lo1;
    r2 = lo2;
}

__device__ inline bool rec_key_eq(const SRec& a, const SRec& b, const uint8_t* const* tails) {
    if (a.hi != b.hi || a.lo != b.lo || a.meta != b.meta) return false;
    return key_len(a.meta) <= 17 || tail_cmp(rec_tail(a, tails), key_len(a.meta), rec_tail(b, tails), key_len(b.meta)) == 0;
}

// rounds mode, two kinds of lanes:
//   i < R        read i: pb = sorted write endpoints with key <= its begin (at
//                an equal key both write endpoint types sort before a read
//                begin, SkipList.cpp:169-172), pe = those with key < its end
//                (a read end sorts first); a candidate if some write endpoint
//                has a key in [begin, end) -- every overlap where the write
//                begins at or after the read does -- or if some write covers
//                its begin: the write cover (begins minus ends among the
//                first pb endpoints) counts exactly the writes [wb, we) with
//                wb <= begin < we -- the overlaps where the read begins inside
//                the write.  (The reads need no order of their own: before the
//                cover, a lane per write searched the sorted read begins.)
//   R + p        sorted write endpoint p starts a new distinct key

__device__ inline void candidate(const EdgesArgs& A, int r) {
    // once per read and batch (a read inside many writes is marked by each;
    // a race between two markers only lets a duplicate through)
    if (A.rstamp[r] == A.rseq) return;
    A.rstamp[r] = A.rseq;
    const int j = atomicAdd(&A.sc->n_pot, 1);
    if (j < A.plist_cap) A.plist[j] = r;
    else A.sc->dec_wide = 1;  // (overflow: every read is a candidate)
}

__device__ inline void rounds_lane(const EdgesArgs& A, int i, const uint64_t* smp_w) {
    const int R = A.R, P = 2 * A.W;
    const uint8_t* const* tails = A.keys.tail;
    if (i < R) {
        if (A.too_old[A.read_txn[i]]) return;  // (not decided by the rounds)
        const Key b = A.keys.get(2 * (int64_t)i), e = A.keys.get(2 * (int64_t)i + 1);
        int lb, hb, le, he, pb, pe;
        sample_narrow(smp_w, P, b.hi, lb, hb);
        sample_narrow(smp_w, P, e.hi, le, he);
        bsearch2(A.sw, b, true, lb, hb, e, le, he, tails, pb, pe);
        A.rq[2 * i] = pb;
        A.rq[2 * i + 1] = pe;
        if (pe > pb || (pb > 0 && (A.wcov[pb - 1] > 0 || rec_vs_key(A.sw[pb - 1], b, tails) == 0))) candidate(A, i);
    } else if (i < R + P) {
        const int p = i - R;
        const SRec x = A.sw[p];
        A.wnew[p] = p == 0 || !rec_key_eq(A.sw[p - 1], x, tails);
        A.winv[x.idx - A.wbase] = p;
    }
}

__device__ inline void edges_lane(const EdgesArgs& A, int i, const uint64_t* smp_r, const uint64_t* smp_w) {
    const int R = A.R, W = A.W;
    const int64_t wbase = A.wbase;
    const uint8_t* const* tails = A.keys.tail;
    if (A.rq) {
        rounds_lane(A, i, smp_w);
        return;
    }
    if (i < R) {
        const int t = A.read_txn[i];
        if (A.too_old[t]) return;
        const Key b = A.keys.get(2 * (int64_t)i), e = A.keys.get(2 * (int64_t)i + 1);
        int lb, hb, le, he, lo, hi;
        sample_narrow(smp_w, 2 * W, b.hi, lb, hb);
        sample_narrow(smp_w, 2 * W, e.hi, le, he);
        bsearch2(A.sw, b, false, lb, hb, e, le, he, tails, lo, hi);
        for (int k = lo; k < hi; k++) {
            const uint32_t slot = A.sw[k].idx;
            if (slot & 1) continue;  // a write end
            const int u = A.write_txn[(slot - wbase) >> 1];
            if (u < t && !A.too_old[u]) edge_pair(t, u, A.et, A.eu, A.cap, A.sc, A.deg);
        }
    } else if (i < R + W) {
        const int w = i - R;
        const int u = A.write_txn[w];
        if (A.too_old[u]) return;
        const Key b = A.keys.get(wbase + 2 * (int64_t)w), e = A.keys.get(wbase + 2 * (int64_t)w + 1);
        int lb, hb, le, he, lo, hi;
        sample_narrow(smp_r, R, b.hi, lb, hb);
        sample_narrow(smp_r, R, e.hi, le, he);
        bsearch2(A.sr, b, true, lb, hb, e, le, he, tails, lo, hi);
        for (int k = lo; k < hi; k++) {
            const int t = A.read_txn[A.sr[k].idx >> 1];
            if (t > u && !A.too_old[t]) edge_pair(t, u, A.et, A.eu, A.cap, A.sc, A.deg);
        }
    }
}

// ---- rounds-mode edge lanes as blocks of the decision's launch ----------
// (launch_decide with b.edges_fused).  Block 0 of k_decide_rounds, the
// decision, waits for these blocks inside the launch instead of a kernel
// boundary: every handed-off value (rq, plist, n_pot, dec_wide, wnew, winv)
// is stored write-through (sc1) and drained (s_waitcnt vmcnt(0)) by every
// storing wave, then one lane per block adds to Scalars::e_done; block 0
// polls that counter and reads the values with sc1 loads
// (MI355X_MICROARCH.md, inter-workgroup visibility: the write-through form,
// no L2 writeback or invalidate).  No deadlock: only block 0 waits, on one
// CU, and the blocks it waits for wait on nothing.
// read i (as rounds_lane), its outputs write-through
__device__ inline void fused_read_lane(const EdgesArgs& A, int i, const uint64_t* smp_w) {
    const int P = 2 * A.W;
    const uint8_t* const* tails = A.keys.tail;
    if (A.too_old[A.read_txn[i]]) return;
    const Key b = A.keys.get(2 * (int64_t)i), e = A.keys.get(2 * (int64_t)i + 1);
    int lb, hb, le, he, pb, pe;
    sample_narrow(smp_w, P, b.hi, lb, hb);
    sample_narrow(smp_w, P, e.hi, le, he);
    bsearch2(A.sw, b, true, lb, hb, e, le, he, tails, pb, pe);
    st1(reinterpret_cast<uint64_t*>(A.rq) + i, (uint64_t)(uint32_t)pb | (uint64_t)(uint32_t)pe << 32);
    if (pe > pb || (pb > 0 && (A.wcov[pb - 1] > 0 || rec_vs_key(A.sw[pb - 1], b, tails) == 0))) {
        const int j = atomicAdd(&A.sc->n_pot, 1);  // (one lane per read: no stamp needed)
        if (j < A.plist_cap) st1(A.plist + j, i);
        else st1(&A.sc->dec_wide, 1);  // (overflow: every read is a candidate)
    }
}

// sorted write endpoints 4q .. 4q + 3: new-key flags (one 4-byte word) and
// their sorted positions
__device__ inline void fused_quad_lane(const EdgesArgs& A, int q) {
    const int P = 2 * A.W, p0 = 4 * q;
    const uint8_t* const* tails = A.keys.tail;
    SRec x[5];
#pragma unroll
    for (int k = 0; k < 5; k++) {  // (sw[p0 - 1 .. p0 + 3], loads issued together)
        const int p = p0 - 1 + k;
        if (p >= 0 && p < P) x[k] = A.sw[p];
    }
    uint32_t word = 0;
#pragma unroll
    for (int k = 1; k < 5; k++) {
        const int p = p0 - 1 + k;
        if (p >= P) break;
        const bool nw = p == 0 || !rec_key_eq(x[k - 1], x[k], tails);
        word |= (uint32_t)nw << (8 * (k - 1));
        st1(A.winv + (x[k].idx - A.wbase), p);
    }
    st1(reinterpret_cast<uint32_t*>(A.wnew) + q, word);
}

__host__ __device__ inline int fused_edge_quads(int W) { return (2 * W + 3) / 4; }

// one edge block of the decision's launch: lanes [0, R) reads, then quads
__device__ void fused_edge_block(const EdgesArgs& A, int eb, uint64_t* smp_w) {
    const int i0 = eb * (int)blockDim.x;
    if (i0 < A.R) sample_fill(smp_w, A.sw, 2 * A.W);
    __syncthreads();
    const int i = i0 + (int)threadIdx.x;
    if (i < A.R) fused_read_lane(A, i, smp_w);
    else if (i < A.R + fused_edge_quads(A.W)) fused_quad_lane(A, i - A.R);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // (every wave drains its sc1 stores)
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(&A.sc->e_done, 1);
}

// One launch, three kinds of blocks: read-check groups and write-search
// groups (history), then edge lanes (intra-batch) -- all latency-bound
// searches, so they overlap.
template <bool WIDE>
__global__ __launch_bounds__(256) void k_edges_read_check(ReadCheckArgs RA, int rc_blocks, WriteSearchArgs WA,
                                                          int ws_blocks, EdgesArgs EA) {
    __shared__ uint64_t smp_r[EQ], smp_w[EQ];
    if ((int)blockIdx.x < rc_blocks) {
        const Group<RC_G> g;
        read_check_group<WIDE>(RA, g, (int)((blockIdx.x * blockDim.x + threadIdx.x) / RC_G));
    } else if ((int)blockIdx.x < rc_blocks + ws_blocks) {
        const Group<RC_G> g;
        write_search_group(WA, g, (int)(((blockIdx.x - rc_blocks) * blockDim.x + threadIdx.x) / RC_G));
    } else {
        const int i0 = (blockIdx.x - rc_blocks - ws_blocks) * blockDim.x;
        if (i0 < EA.R) sample_fill(smp_w, EA.sw, 2 * EA.W);          // readers search the writes
        if (!EA.rq && i0 + (int)blockDim.x > EA.R) sample_fill(smp_r, EA.sr, EA.R);  // writers search the reads
        __syncthreads();
        edges_lane(EA, i0 + threadIdx.x, smp_r, smp_w);
    }
}

// Large batches: the directory entry of every sorted read begin and write
// endpoint by one merge-join with the directory's first keys instead of a
// search-index descent per key (dir_search: entry x = the number of entries
// j >= 1 with first(j) <= k).  In the merged order (first keys before queries
// of equal key) a query at merged position m with index i has x = m - i.
// Job 0: sorted read begins -> qx[read index]; job 1: sorted write endpoints
// -> qx[R + endpoint index].
struct DirJoinArgs {
    const SRec* q[2];
    int32_t nq[2];
    int32_t blocks0;
    Dir dir;
    const Scalars* sc;
    KeyArrays keys;
    int R;
    int32_t* qx;
    // by_pos: qx by sorted position instead -- [0, R) job 0, [R, R + 2W) job 1
    // (k_page_join's runs)
    int by_pos;
};

__global__ __launch_bounds__(MS_THREADS) void k_dir_join(DirJoinArgs A) {
    __shared__ uint64_t s_hi[MS_CHUNK], s_lo[MS_CHUNK], s_mi[MS_CHUNK];
    __shared__ int s_cut[2];
    const int job = (int)blockIdx.x < A.blocks0 ? 0 : 1;
    const int chunk = job ? blockIdx.x - A.blocks0 : blockIdx.x;
    const Dir& d = A.dir;
    const int nf = A.sc->D - 1;  // first keys of entries 1 .. D-1
    const int nq = A.nq[job];
    const SRec* Q = A.q[job];
    const int d0 = chunk * MS_CHUNK;
    if (d0 >= nf + nq) return;
    const int d1 = min(d0 + MS_CHUNK, nf + nq);
    const uint8_t* const* qt = A.keys.tail;
    auto fkey = [&](int j) { return dir_first(d, j + 1); };
    auto f_le_q = [&](const Key& f, const SRec& x) {
        return kcmp(f, Key{x.hi, x.lo, x.meta, qt[x.idx]}) <= 0;
    };
    if (threadIdx.x < 2) {  // first keys among the first dd merged positions
        const int dd = threadIdx.x ? d1 : d0;
        int lo = max(0, dd - nq), hi = min(dd, nf);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (f_le_q(fkey(mid), Q[dd - 1 - mid])) lo = mid + 1;
            else hi = mid;
        }
        s_cut[threadIdx.x] = lo;
    }
    __syncthreads();
    const int a0 = s_cut[0], a1 = s_cut[1], b0 = d0 - a0, b1 = d1 - a1;
    const int na = a1 - a0, nb = b1 - b0;
    const LdsRecs L{s_hi, s_lo, s_mi};  // [0, na): first keys (idx = entry - 1), [na, na + nb): queries
    for (int k = threadIdx.x; k < na + nb; k += MS_THREADS) {
        if (k < na) {
            const int j = a0 + k;
            L.put(k, SRec{d.fhi[j + 1], d.flo[j + 1], d.fmeta[j + 1], (uint32_t)j, 0});
        } else {
            L.put(k, Q[b0 + k - na]);
        }
    }
    __syncthreads();
    auto lds_f_le_q = [&](int fa, int qb) {
        const SRec f = L.get(fa);
        return f_le_q(Key{f.hi, f.lo, f.meta, d.ftail[f.idx + 1]}, L.get(qb));
    };
    const int dl = threadIdx.x * MS_ITEMS;
    if (dl >= na + nb) return;
    int ia, ib;
    {
        int lo = max(0, dl - nb), hi = min(dl, na);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (lds_f_le_q(mid, na + dl - 1 - mid)) lo = mid + 1;
            else hi = mid;
        }
        ia = lo;
        ib = dl - lo;
    }
    const int cnt = min(MS_ITEMS, na + nb - dl);
    for (int q = 0; q < cnt; q++) {
        const int m = d0 + dl + q;
        if (ia < na && (ib >= nb || lds_f_le_q(ia, na + ib))) {
            ia++;
        } else {
            const int i = b0 + ib;
            const uint32_t slot = L.get(na + ib).idx;
            ib++;
            const int x = m - i;
            if (A.by_pos) A.qx[(job ? A.R : 0) + i] = x;
            else if (job == 0) A.qx[slot >> 1] = x;
            else A.qx[A.R + (int)(slot - 2 * (uint32_t)A.R)] = x;
        }
    }
}

// ---- large batches: read checks and write searches, a lane per query ------
// (config 5: 5 M reads and 4 M write endpoints over a 10^8-boundary history.)
// The queries are sorted and k_dir_join gave each its directory entry (by
// sorted position), so one lane answers one query with wide loads instead of
// a 16-lane group probing 8 bytes a lane: the page's index line (hi of slots
// 0, 16, ..., 240: 128 bytes), then the 16 slots of its window (128 bytes),
// compared in registers; the full key only on a tie of the first 8 bytes.
// A read whose end lies in the same page (the reads are short) searches the
// same index line again and covers the versions between; one whose end lies
// past the page goes to a list the 16-lane search then checks.  A write
// endpoint gets its WriteHits record (slot, real boundaries before it,
// valueBefore).  Measured first as a wavefront per page run, the page's keys
// staged in LDS: slower (4.35 ms against 2.12 ms for the read-check stage at
// config 5: ~10 queries per page left most lanes idle and every page was
// read whole).
struct PageJoinArgs {
    int R, P;             // sorted read begins (job 0), sorted write endpoints (job 1)
    const int32_t* xs;    // [R + P] directory entry of each sorted query (k_dir_join, by_pos)
    int32_t* fall;        // reads whose end lies past their begin's page; Scalars::n_fall
    const SRec* sr;
    const SRec* sw;
    KeyArrays keys;
    const int32_t* read_txn;
    const int64_t* read_snap;
    uint8_t* hist;
    Pool pool;
    Dir dir;
    Scalars* sc;
    int64_t v0;
    WriteHits wh;
    int64_t wbase;
};

// slot s of a page (base) against k: the 8-byte word v already loaded
__device__ inline int slot_vs(const Pool& p, int64_t base, int s, uint64_t v, const Key& k) {
    if (v != k.hi) return v < k.hi ? -1 : 1;
    return kcmp(pool_key(p, base + s), k);
}

// lower bound of k among the cnt slots of a page by one lane: idx = the
// page's 16 index words (Pool::pidx), then one 16-slot window
__device__ inline int lane_page_lb(const Pool& p, int64_t base, int cnt, const uint64_t (&idx)[16], const Key& k,
                                   bool& eq) {
    int n = 0;
    bool eq_n = false;  // slot 16n holds k (when 16n < cnt)
#pragma unroll
    for (int j = 0; j < 16; j++) {
        if (16 * j < cnt) {
            const int c = slot_vs(p, base, 16 * j, idx[j], k);
            n += c < 0;
            if (j == n && c == 0) eq_n = true;  // (the first slot not below k, when it equals k)
        }
    }
    if (n == 0) {
        eq = cnt > 0 && eq_n;
        return 0;
    }
    const int w = 16 * (n - 1), e = min(cnt, 16 * n);
    uint64_t v[16];
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(p.hi + base + w);
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const ulonglong2 x = src[j];  // (a page's slots are 16-aligned: 128 bytes, whole line)
        v[2 * j] = x.x;
        v[2 * j + 1] = x.y;
    }
    int m = 0;  // slots of the window below k (slot w is)
    bool eq_m = false;
#pragma unroll
    for (int j = 0; j < 16; j++) {
        if (w + j < e) {
            const int c = slot_vs(p, base, w + j, v[j], k);
            m += c < 0;
            if (j == m && c == 0) eq_m = true;
        }
    }
    const int i = w + m;
    eq = i < e ? eq_m : (e < cnt && eq_n);
    return i;
}

__device__ inline void lane_index(const Pool& p, int pg, uint64_t (&idx)[16]) {
    const ulonglong2* src = reinterpret_cast<const ulonglong2*>(p.pidx + (int64_t)pg * (PAGE / PIDX_STRIDE));
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const ulonglong2 x = src[j];
        idx[2 * j] = x.x;
        idx[2 * j + 1] = x.y;
    }
}

__global__ __launch_bounds__(256) void k_page_join(PageJoinArgs A) {
    const int k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= A.R + A.P) return;
    const Dir& d = A.dir;
    const int x = A.xs[k];
    const int pg = d.page[x], cnt = d.cnt[x];
    const int64_t base = (int64_t)pg * PAGE;
    uint64_t idx[16];
    if (k < A.R) {  // the history check of read r
        const SRec rec = A.sr[k];
        const int r = (int)(rec.idx >> 1);
        const int64_t s = A.read_snap[r];
        if (s == INT64_MAX) return;
        const Key b{rec.hi, rec.lo, rec.meta, key_len(rec.meta) > 17 ? A.keys.tail[2 * (int64_t)r] : nullptr};
        const Key e = A.keys.get_short(2 * (int64_t)r + 1);  // (config 5: 64 of ~610 bytes a read fetched)
        bool past = false;  // e > the next page's first key: e lies past this page
        if (x + 1 < A.sc->D) {
            const uint64_t fh = d.fhi[x + 1];
            past = fh != e.hi ? fh < e.hi : kcmp(dir_first(d, x + 1), e) < 0;
        }
        if (past) {
            A.fall[atomicAdd(&A.sc->n_fall, 1)] = r;  // (past this page: the 16-lane search)
            return;
        }
        lane_index(A.pool, pg, idx);
        bool eqb, eqe;
        const int ib = lane_page_lb(A.pool, base, cnt, idx, b, eqb);
        const int ie = lane_page_lb(A.pool, base, cnt, idx, e, eqe);
        const int i0 = eqb ? ib : ib - 1;  // the slot whose version covers b
        bool c = i0 < 0 && A.v0 > s;
        for (int i = max(i0, 0); i < ie; i++) c |= A.pool.ver[base + i] > s;
        if (c) A.hist[A.read_txn[r]] = 1;
        return;
    }
    // where write endpoint (slot) falls (write_search_group)
    const SRec rec = A.sw[k - A.R];
    const uint32_t slot = rec.idx;
    const int w = (int)(((int64_t)slot - A.wbase) >> 1);
    const Key key{rec.hi, rec.lo, rec.meta, key_len(rec.meta) > 17 ? A.keys.tail[slot] : nullptr};
    uint64_t hm[HM_WORDS];
    load_hmask(A.pool, pg, hm);
    lane_index(A.pool, pg, idx);
    bool eq;
    const int i = lane_page_lb(A.pool, base, cnt, idx, key, eq);
    const int rb = real_before(hm, i);
    if (!(slot & 1)) {
        A.wh.b[w] = WHitB{x, i, d.nr[x], rb};
        return;
    }
    int64_t vb;
    bool from_v0 = false;  // no boundary below e: the header version
    if (i > 0) vb = A.pool.ver[base + i - 1];
    else if (x > 0 && d.cnt[x - 1] > 0) vb = A.pool.ver[(int64_t)d.page[x - 1] * PAGE + d.cnt[x - 1] - 1];
    else vb = A.v0, from_v0 = true;  // (only entry 0 can be an empty page)
    A.wh.e[w] = WHitE{vb, x, i, rb, (int32_t)((int)eq | (int)from_v0 << 1), 0};
}

// the reads k_page_join listed (their end lies past their begin's page): the
// 16-lane history check with the directory search
template <bool WIDE>
__global__ __launch_bounds__(256) void k_read_check_list(ReadCheckArgs RA, const int32_t* list) {
    const Group<RC_G> g;
    const int n = RA.sc->n_fall;
    const int ng = gridDim.x * blockDim.x / RC_G;
    for (int q = (int)((blockIdx.x * blockDim.x + threadIdx.x) / RC_G); q < n; q += ng)
        read_check_group<WIDE>(RA, g, list[q]);
}

// Large batches: the overlap edges by one merge-join of the sorted read
// begins with the sorted write endpoints instead of two binary searches per
// range.  In the merged order (key; a read before a write endpoint of equal
// key) a read at merged position m with sorted index k has m - k write
// endpoints below its begin -- lb_key(sw, r.b) -- and a write begin at m with
// sorted index j has m - j reads at or below it -- ub_key(sr, w.b).  From
// there each range scans forward to its end exactly as edges_lane loops
// between its two search results.  Workgroups take MS_CHUNK merged positions
// (merge-path cuts, the two pieces staged in LDS), lanes MS_ITEMS each.
__device__ inline bool rd_before_wr(const SRec& r, const SRec& w, const uint8_t* const* tails) {
    return rec_vs_key(r, Key{w.hi, w.lo, w.meta, rec_tail(w, tails)}, tails) <= 0;  // key(r) <= key(w)
}

__global__ __launch_bounds__(MS_THREADS) void k_edges_merge(EdgesArgs A) {
    __shared__ uint64_t s_hi[MS_CHUNK], s_lo[MS_CHUNK], s_mi[MS_CHUNK];
    __shared__ int s_cut[2];
    const int R = A.R, nw = 2 * A.W;
    const int64_t wbase = A.wbase;
    const uint8_t* const* tails = A.keys.tail;
    const SRec* sr = A.sr;
    const SRec* sw = A.sw;
    const int d0 = blockIdx.x * MS_CHUNK, d1 = min(d0 + MS_CHUNK, R + nw);
    auto before = [&](const SRec& r, const SRec& w) { return rd_before_wr(r, w, tails); };
    if (threadIdx.x < 2) {  // reads among the first d merged positions
        const int d = threadIdx.x ? d1 : d0;
        int lo = max(0, d - nw), hi = min(d, R);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (before(sr[mid], sw[d - 1 - mid])) lo = mid + 1;
            else hi = mid;
        }
        s_cut[threadIdx.x] = lo;
    }
    __syncthreads();
    const int a0 = s_cut[0], a1 = s_cut[1], b0 = d0 - a0, b1 = d1 - a1;
    const int na = a1 - a0, nb = b1 - b0;
    const LdsRecs L{s_hi, s_lo, s_mi};
    for (int k = threadIdx.x; k < na + nb; k += MS_THREADS) L.put(k, k < na ? sr[a0 + k] : sw[b0 + k - na]);
    __syncthreads();
    const int dl = threadIdx.x * MS_ITEMS;
    if (dl >= na + nb) return;
    int ia, ib;
    {
        int lo = max(0, dl - nb), hi = min(dl, na);
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (before(L.get(mid), L.get(na + dl - 1 - mid))) lo = mid + 1;
            else hi = mid;
        }
        ia = lo;
        ib = dl - lo;
    }
    const int cnt = min(MS_ITEMS, na + nb - dl);
    for (int q = 0; q < cnt; q++) {
        const int m = d0 + dl + q;
        const bool take_r = ia < na && (ib >= nb || before(L.get(ia), L.get(na + ib)));
        // (the common case -- nothing overlaps -- costs the next record and the
        // end key's first word: a strictly greater first word decides)
        if (take_r) {
            const int k = a0 + ia++;
            const uint32_t slot = L.get(k - a0).idx;
            int j = m - k;
            if (j >= nw || sw[j].hi > A.keys.hi[slot + 1]) continue;
            const Key e = A.keys.get((int64_t)slot + 1);
            if (rec_vs_key(sw[j], e, tails) >= 0) continue;
            const int t = A.read_txn[slot >> 1];
            if (A.too_old[t]) continue;
            for (; j < nw; j++) {  // write endpoints with key in [r.b, r.e)
                const SRec x = sw[j];
                if (rec_vs_key(x, e, tails) >= 0) break;
                if (x.idx & 1) continue;  // a write end
                const int u = A.write_txn[(x.idx - wbase) >> 1];
                if (u < t && !A.too_old[u]) edge_pair(t, u, A.et, A.eu, A.cap, A.sc, A.deg);
            }
        } else {
            const int j = b0 + ib++;
            const uint32_t slot = L.get(na + j - b0).idx;
            if (slot & 1) continue;  // only write begins search the reads
            int k = m - j;
            if (k >= R || sr[k].hi > A.keys.hi[slot + 1]) continue;
            const Key e = A.keys.get((int64_t)slot + 1);
            if (rec_vs_key(sr[k], e, tails) >= 0) continue;
            const int u = A.write_txn[(slot - wbase) >> 1];
            if (A.too_old[u]) continue;
            for (; k < R; k++) {  // reads beginning in (w.b, w.e)
                const SRec x = sr[k];
                if (rec_vs_key(x, e, tails) >= 0) break;
                const int t = A.read_txn[x.idx >> 1];
                if (t > u && !A.too_old[t]) edge_pair(t, u, A.et, A.eu, A.cap, A.sc, A.deg);
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_write_search(WriteSearchArgs WA) {
    const Group<RC_G> g;
    write_search_group(WA, g, (int)((blockIdx.x * blockDim.x + threadIdx.x) / RC_G));
}

// the write searches held back by launch_edges_read_check(defer_ws): only
// the merge needs them, so they run after the verdicts
void launch_write_search(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t v0,
                         hipStream_t s) {
    if (!b.ws_deferred) return;
    b.ws_deferred = false;
    const int R = v.read_count, W = v.write_count;
    if (W == 0) return;
    WriteSearchArgs WA{R, W, b.keys, h.pool, h.dir[cur], sc, v0, b.wh, nullptr, write_base(b, v)};
    hipLaunchKernelGGL(k_write_search, dim3(cdiv((int64_t)W * RC_G, 256)), dim3(256), 0, s, WA);
}

static EdgesArgs make_edges_args(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc) {
    return EdgesArgs{v.read_count, v.write_count, b.keys, (const SRec*)b.sr, (const SRec*)b.sw, b.read_txn,
                     b.write_txn, b.too_old, b.et, b.eu, b.edge_cap, sc, b.deg, b.rounds ? b.rq : nullptr, b.wnew,
                     b.plist, b.list_cap, b.winv, b.wcov, b.rstamp, b.rseq, write_base(b, v)};
}

void launch_edges_read_check(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t v0,
                             hipStream_t s, bool defer_ws) {
    const int R = v.read_count, W = v.write_count;
    // unsharded batches with b.dir_join: directory entries by merge-join (ss_bkt is free once the sort is done)
    static const bool dir_search = getenv("FDBCS_LARGE_DIR_SEARCH") != nullptr;  // (A/B measurements)
    const bool dj = b.dir_join && !(h.shard.has_lo | h.shard.has_hi) && !dir_search && R + W > 0;
    // ... and then the read checks and write searches by page runs
    // (k_page_join; FDBCS_LARGE_PAGE_JOIN=0: the 16-lane searches from the
    // join's entries, A/B)
    static const bool no_pj = getenv("FDBCS_LARGE_PAGE_JOIN") && !atoi(getenv("FDBCS_LARGE_PAGE_JOIN"));
    const bool pj = dj && !no_pj && b.pj_fall && R + 2 * (int64_t)W + 64 <= b.pj_cap;
    if (dj) {
        DirJoinArgs J{{b.sr, b.sw}, {R, 2 * W}, 0, h.dir[cur], sc, b.keys, R, b.ss_bkt, pj ? 1 : 0};
        const int64_t cap_f = h.cap_dir;  // (an upper bound on D: blocks past the merged length exit)
        J.blocks0 = cdiv(cap_f + R, MS_CHUNK);
        const int blocks = J.blocks0 + cdiv(cap_f + 2 * (int64_t)W, MS_CHUNK);
        hipLaunchKernelGGL(k_dir_join, dim3(blocks), dim3(MS_THREADS), 0, s, J);
    }
    const int32_t* qx = dj && !pj ? b.ss_bkt : nullptr;
    ReadCheckArgs RA{R, b.keys, b.read_txn, b.read_snap, b.hist, h.pool, h.dir[cur], sc, v0, h.shard, qx};
    if (pj && R + W > 0) {
        (void)hipMemsetAsync(&sc->n_fall, 0, sizeof(int32_t), s);
        const PageJoinArgs PJ{R, 2 * W, b.ss_bkt, b.pj_fall, (const SRec*)b.sr, (const SRec*)b.sw, b.keys,
                              b.read_txn, b.read_snap, b.hist, h.pool, h.dir[cur], sc, v0, b.wh, write_base(b, v)};
        const int64_t nq = R + 2 * (int64_t)W;
        hipLaunchKernelGGL(k_page_join, dim3(cdiv(nq, 256)), dim3(256), 0, s, PJ);
        if (R > 0) {
            if (FDBCS_RC_WIDE) hipLaunchKernelGGL(k_read_check_list<true>, dim3(1024), dim3(256), 0, s, RA, b.pj_fall);
            else hipLaunchKernelGGL(k_read_check_list<false>, dim3(1024), dim3(256), 0, s, RA, b.pj_fall);
        }
    }
    const EdgesArgs EA = make_edges_args(v, b, sc);
    WriteSearchArgs WA{R, W, b.keys, h.pool, h.dir[cur], sc, v0, b.wh, qx, write_base(b, v)};
    // (rc_fused: the history read check already ran in the sort's bucket launch)
    const int rc_blocks = b.rc_fused || pj ? 0 : cdiv((int64_t)R * RC_G, 256);
    b.rc_fused = false;
    b.ws_deferred = defer_ws && !dj;
    const int ws_blocks = b.ws_deferred || pj ? 0 : cdiv((int64_t)W * RC_G, 256);
    static const bool search_edges = getenv("FDBCS_LARGE_EDGES_SEARCH") != nullptr;  // (A/B measurements)
    const bool join = b.large && !search_edges;
    const int e_blocks = R > 0 && W > 0 && !join ? cdiv(R + (b.rounds ? 2 * W : W), 256) : 0;
    const bool wide = FDBCS_RC_WIDE;  // (WIDE = false: the two-level range maximum, kept for A/B)
    // rounds mode with nothing else in this launch (the read check fused into
    // the sort's buckets, the write searches deferred): the edge lanes become
    // blocks of the decision's launch instead, one dependent launch fewer
    // before the verdicts (k_decide_rounds, "fused edge lanes")
    // Measured and off by default (FDBCS_FUSE_EDGES=1 turns it on): config 2,
    // alternating runs on one box, HBM-resident batch 0.1996 / 0.1979 ms fused
    // against 0.1957 / 0.1962 separate -- the decision launch's blocks carry
    // its ~150 KB of LDS, so its edge blocks run one per CU (44 CUs of 16
    // waves instead of 176 of 4) and the searches lose more than the launch
    // boundary saves
    static const bool fuse = getenv("FDBCS_FUSE_EDGES") && atoi(getenv("FDBCS_FUSE_EDGES"));
    b.edges_fused = b.rounds && defer_ws && fuse && rc_blocks == 0 && ws_blocks == 0 && e_blocks > 0 && !join;
    if (!b.edges_fused && rc_blocks + ws_blocks + e_blocks > 0) {
        if (wide)
            hipLaunchKernelGGL(k_edges_read_check<true>, dim3(rc_blocks + ws_blocks + e_blocks), dim3(256), 0, s, RA,
                               rc_blocks, WA, ws_blocks, EA);
        else
            hipLaunchKernelGGL(k_edges_read_check<false>, dim3(rc_blocks + ws_blocks + e_blocks), dim3(256), 0, s, RA,
                               rc_blocks, WA, ws_blocks, EA);
    }
    if (join && R > 0 && W > 0)
        hipLaunchKernelGGL(k_edges_merge, dim3(cdiv((int64_t)R + 2 * (int64_t)W, MS_CHUNK)), dim3(MS_THREADS), 0, s,
                           EA);
}

// ------------------------------------------ decide by rounds + combine ----
// checkIntraBatchConflicts (SkipList.cpp:1133-1153) without enumerating
// (reader, earlier writer) pairs, then combineWriteConflictRanges
// (:1320-1337); one workgroup, its state in LDS.
//
// The decision: U = transactions neither tooOld nor conflicting with the
// history.  t in U commits iff no read of t overlaps a write of a committed
// u < t.  Write C(t) for that predicate given a candidate committed set C;
// the committed set is the unique fixed point C* = {t in U : C*(t)} (unique
// by induction on the index).  Jacobi from C_0 = U: C_{k+1} = {t in U :
// C_k(t)} -- even iterates contain C*, odd ones are contained in it, and
// transaction t is final after at most t + 1 rounds -- stops at C_{k+1} =
// C_k, which is C*.  Config 3 (Zipf) converges in ~8 rounds.  Only candidate
// reads (k_edges_read_check marked those a write of the batch may overlap)
// are evaluated; with none (config 2, uniform keys) there is no round.
//
// A round without pairs.  Key positions are ranks among the DISTINCT keys of
// the sorted write endpoints: write w = [B, E), B < E its begin / end ranks;
// read r = (Gb, Ge), Gb = distinct keys <= its begin, Ge = distinct keys <
// its end.  [rb, re) overlaps [wb, we) (rb < we and wb < re, the half-open
// overlap the reference's tie order encodes) iff B < Ge and Gb <= E: (a) Gb
// <= B < Ge, the write begins inside the read, or (b) B < Gb <= E, the read
// begins inside the write.  Per round each write of a candidate u takes the
// min at val[B] and paints stab over (B, E] (min); a read of t conflicts iff
// min(val[Gb, Ge)) < t or stab[Gb] < t.  A hot key is one rank, so a round
// costs O(candidate reads + writes of U) LDS operations whatever the fan-in
// (the pair list it replaces held ~10^6 pairs per Zipf batch).  val and stab
// are 16-bit (transaction indices and ranks < 65535, rounds_fit); long
// paints and range queries go through block minima of RB1 and RB2 ranks.
//
// Combine: over the sorted write endpoints (END before BEGIN at equal keys),
// a counter of open committed writes; a combined range starts at a committed
// BEGIN seen with the counter at 0 and ends at the committed END that brings
// it back to 0.
struct RoundArgs {
    int T, R, W;
    EarlyOut eo;              // eo.flag: verdicts go to host-mapped memory, then the flag
    int combine;              // 0: the multi-block combine kernels follow
    int lcap;                 // items that fit in LDS (else A.items)
    const uint8_t* too_old;
    const uint8_t* hist;
    const int32_t* read_txn;
    const int32_t* write_txn;
    const int32_t* rq;        // [2R] (k_edges_read_check, rounds mode)
    const int32_t* plist;     // candidate reads, sc->n_pot of them
    const uint8_t* wnew;      // [2W]
    const int32_t* winv;      // [2W]
    const uint32_t* sw_slot;  // [2W] slots of the sorted write endpoints
    int64_t lcap_list;        // plist entries (past it: dec_wide)
    uint2* items;             // [2 * lcap_list] global fallback of the item list
    uint8_t* committed;
    uint8_t* verdict;
    int32_t* cb_pos;          // combined range begins / ends, as positions among the sorted write endpoints
    int32_t* ce_pos;
    Scalars* sc;
    // blocks 1.. of the launch: the merge's write searches (deferred by the
    // read check), beside the decision in block 0, which holds one CU
    WriteSearchArgs ws;
    int64_t wbase;  // slot of write 0's begin (write_base)
    // blocks 1 .. eblocks: the fused edge lanes (b.edges_fused), before the
    // write-search blocks; 0: k_edges_read_check ran them
    EdgesArgs ea;
    int eblocks;
};

static constexpr int DC_THREADS = 1024;
static constexpr int CPMAX = 32;  // sorted endpoints per thread kept in registers (combine)
static constexpr int RB1 = 64, RB2 = 4096;
static constexpr uint16_t INF16 = 0xFFFF;
static constexpr size_t ROUNDS_LDS_MAX = 156 * 1024;
// Items are taken DG per lane at a time (item i + k * nthr), their loads
// issued together: one workgroup is latency-bound on its global inputs.
constexpr int DG = 8;

__device__ __host__ inline int64_t rank_words16(int64_t P) {  // val + stab + their block minima, in u16
    const int64_t n = P + 3;
    return 2 * (n + n / RB1 + 3 + n / RB2 + 3);
}

__host__ __device__ inline size_t rounds_lds_base(int64_t T, int64_t W) {
    const int64_t P = 2 * W;
    const int64_t bits = 4 * ((T + 31) / 32) + (W + 31) / 32;
    return (size_t)(4 * bits + 2 * rank_words16(P) + 64);
}

bool rounds_fit(int64_t T, int64_t W) {
    return T < INF16 && 2 * W + 2 < INF16 && 2 * W <= CPMAX * DC_THREADS &&
           rounds_lds_base(T, W) + 8 * 1024 <= ROUNDS_LDS_MAX;
}

// 16-bit min in LDS (no ds_min_u16 on gfx950): CAS on the containing word,
// skipped when the value there is already lower.  arr is 4-byte aligned.
__device__ inline void lds_min16(uint16_t* arr, int idx, uint16_t v) {
    uint32_t* w = reinterpret_cast<uint32_t*>(arr) + (idx >> 1);
    const int sh = (idx & 1) * 16;
    uint32_t old = *w;
    while (((old >> sh) & 0xFFFFu) > v) {
        const uint32_t nw = (old & ~(0xFFFFu << sh)) | ((uint32_t)v << sh);
        const uint32_t prev = atomicCAS(w, old, nw);
        if (prev == old) break;
        old = prev;
    }
}

// f over positions [a, b): per position below RB1 / RB2 boundaries, per
// block of RB1 / RB2 positions inside them
template <typename F1, typename F2, typename F3>
__device__ inline void blocks_of(int a, int b, F1 pos, F2 blk1, F3 blk2) {
    while (a < b && (a & (RB1 - 1))) pos(a++);
    while (a + RB1 <= b && (a & (RB2 - 1))) {
        blk1(a / RB1);
        a += RB1;
    }
    while (a + RB2 <= b) {
        blk2(a / RB2);
        a += RB2;
    }
    while (a + RB1 <= b) {
        blk1(a / RB1);
        a += RB1;
    }
    while (a < b) pos(a++);
}

__device__ inline bool bit_of(const uint32_t* bits, int t) { return (bits[t >> 5] >> (t & 31)) & 1; }

__global__ __launch_bounds__(DC_THREADS) void k_decide_rounds(RoundArgs A) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    if (blockIdx.x > 0) {
        if ((int)blockIdx.x <= A.eblocks) {  // a fused edge block (its sample of the sorted writes in LDS)
            fused_edge_block(A.ea, (int)blockIdx.x - 1, reinterpret_cast<uint64_t*>(lds));
            return;
        }
        // a write-search block: 64 groups of RC_G lanes
        const Group<RC_G> g;
        write_search_group(A.ws, g, (int)(((blockIdx.x - 1 - A.eblocks) * blockDim.x + threadIdx.x) / RC_G));
        return;
    }
    __shared__ int32_t red32[DC_THREADS / 64 + 1];
    __shared__ int32_t s_nw, s_nr;
    const int T = A.T, R = A.R, W = A.W, P = 2 * A.W;
    const int tid = threadIdx.x, nthr = blockDim.x;
    const int nwords = (T + 31) >> 5, wwords = (W + 31) >> 5;
    uint32_t* ubits = lds;              // U
    uint32_t* cbits = lds + nwords;     // the candidate committed set; C* at the end
    uint32_t* nbits = cbits + nwords;   // conflicts found this round
    uint32_t* tbits = nbits + nwords;   // too old (the verdicts read it here, not from global memory)
    uint32_t* cwb = tbits + nwords;     // committed, per write (combine)
    uint16_t* r16 = reinterpret_cast<uint16_t*>(cwb + wwords);  // ranks: P u16 first, then val / stab
    uint2* litems = reinterpret_cast<uint2*>(r16 + ((rank_words16(P) + 3) & ~3));  // lcap items
    Scalars* sc = A.sc;
    const int64_t wbase = A.wbase;
    int ncand = 0;
    PHASE(sc, 0);
    // (the flag's error words, final before this launch: loaded now, off the
    // way from the verdicts to the flag)
    uint32_t eo_err = 0, eo_last = 0, eo_lm = 0, eo_shmax = 0;
    if (A.eo.flag && tid == 0) {
        eo_err = (uint32_t)sc->err;
        eo_last = (uint32_t)sc->last_err;
        eo_lm = (uint32_t)sc->lm_count;  // (the ingest's load-metrics entries, if a sample is attached)
        eo_shmax = (uint32_t)sc->sh_max;  // (protocol B: the largest shard edge count, identical on every rank)
    }

    // ---- U: 4 transactions per lane from one 4-byte load of each flag array ----
    for (int i = tid; i < nwords; i += nthr) nbits[i] = tbits[i] = 0;
    if (tid == 0) s_nw = s_nr = 0;
    __syncthreads();
    for (int t4 = tid; 4 * t4 < T; t4 += nthr) {
        const uint32_t to = reinterpret_cast<const uint32_t*>(A.too_old)[t4];
        const uint32_t hs = reinterpret_cast<const uint32_t*>(A.hist)[t4];
        uint32_t m = 0, mt = 0;
#pragma unroll
        for (int k = 0; k < 4; k++) {
            m |= (uint32_t)(4 * t4 + k < T && !(((to | hs) >> (8 * k)) & 0xFF)) << k;
            mt |= (uint32_t)(4 * t4 + k < T && ((to >> (8 * k)) & 0xFF)) << k;
        }
        if (m) atomicOr(&nbits[t4 >> 3], m << (4 * (t4 & 7)));
        if (mt) atomicOr(&tbits[t4 >> 3], mt << (4 * (t4 & 7)));
    }
    __syncthreads();
    for (int i = tid; i < nwords; i += nthr) {
        ubits[i] = cbits[i] = nbits[i];
        nbits[i] = 0;
    }
    if (A.eblocks && tid == 0) {  // the fused edge blocks of this launch (U above overlapped them)
        while (ld1(&sc->e_done) < A.eblocks) __builtin_amdgcn_s_sleep(1);
        st1(&sc->e_done, 0);  // (every edge block has added: zero for the next batch)
    }
    __syncthreads();
    const bool wide = ld1(&sc->dec_wide) != 0;
    const int npot = wide ? R : (int)min((int64_t)ld1(&sc->n_pot), A.lcap_list);
    if (npot == 0) goto decided;  // no read can meet a write of the batch: C* = U
    PHASE(sc, 2);
    {
        // ---- distinct ranks of the sorted write endpoints (u16, LDS) ----
        const int CH = ((P + nthr - 1) / nthr + 3) & ~3;
        const int p0 = min(P, tid * CH), p1 = min(P, p0 + CH);
        uint32_t fl[CPMAX / 4 + 1];
        int nnew = 0;
#pragma unroll
        for (int k = 0; k < CPMAX / 4 + 1; k++) {
            fl[k] = p0 + 4 * k < p1 ? ld1(reinterpret_cast<const uint32_t*>(A.wnew) + (p0 >> 2) + k) : 0;
            nnew += __popc(fl[k] & 0x01010101u & (p0 + 4 * k + 4 <= p1 ? ~0u : (1u << (8 * (p1 - p0 - 4 * k))) - 1));
        }
        int tot;
        int d = block_excl_scan(nnew, red32, tot) - 1;  // (its barriers also publish U)
        for (int p = p0; p < p1; p++) {
            d += (fl[(p - p0) >> 2] >> (8 * ((p - p0) & 3))) & 1;
            r16[p] = (uint16_t)d;
        }
        __syncthreads();
        // the item list: writes of U (B | E << 16, u), then candidate reads of U (Gb | Ge << 16, t)
        for (int w0 = tid; w0 < W; w0 += DG * nthr) {
            int u[DG], pb[DG], pe[DG];
#pragma unroll
            for (int k = 0; k < DG; k++) u[k] = w0 + k * nthr < W ? A.write_txn[w0 + k * nthr] : -1;
#pragma unroll
            for (int k = 0; k < DG; k++) {
                const int w = w0 + k * nthr;
                if (u[k] >= 0 && bit_of(ubits, u[k])) {
                    pb[k] = ld1(A.winv + 2 * w);
                    pe[k] = ld1(A.winv + 2 * w + 1);
                } else {
                    u[k] = -1;
                }
            }
#pragma unroll
            for (int k = 0; k < DG; k++) {
                if (u[k] < 0) continue;
                const int j = atomicAdd(&s_nw, 1);
                const uint2 it{(uint32_t)r16[pb[k]] | ((uint32_t)r16[pe[k]] << 16), (uint32_t)u[k]};
                if (j < A.lcap) litems[j] = it;
                else A.items[j] = it;
            }
        }
        __syncthreads();
        const int nw = s_nw;
        for (int i0 = tid; i0 < npot; i0 += DG * nthr) {
            int r[DG], t[DG], pb[DG], pe[DG];
#pragma unroll
            for (int k = 0; k < DG; k++) r[k] = i0 + k * nthr < npot ? (wide ? i0 + k * nthr : ld1(A.plist + i0 + k * nthr)) : -1;
#pragma unroll
            for (int k = 0; k < DG; k++) r[k] = r[k] < R ? r[k] : -1;
#pragma unroll
            for (int k = 0; k < DG; k++) t[k] = r[k] >= 0 ? A.read_txn[r[k]] : -1;
#pragma unroll
            for (int k = 0; k < DG; k++) {
                if (t[k] >= 0 && bit_of(ubits, t[k]) && !A.too_old[t[k]]) {
                    const uint64_t q = ld1(reinterpret_cast<const uint64_t*>(A.rq) + r[k]);  // (pb, pe)
                    pb[k] = (int32_t)(uint32_t)q;
                    pe[k] = (int32_t)(uint32_t)(q >> 32);
                } else {
                    t[k] = -1;
                }
            }
#pragma unroll
            for (int k = 0; k < DG; k++) {
                if (t[k] < 0) continue;
                const int j = nw + atomicAdd(&s_nr, 1);
                const uint32_t gb = pb[k] > 0 ? r16[pb[k] - 1] + 1u : 0u, ge = pe[k] > 0 ? r16[pe[k] - 1] + 1u : 0u;
                const uint2 it{gb | (ge << 16), (uint32_t)t[k]};
                if (j < A.lcap) litems[j] = it;
                else A.items[j] = it;
            }
        }
        __syncthreads();
        ncand = s_nr;
        PHASE(sc, 3);
    }
    {
        // ---- rounds: val / stab over the distinct ranks, in LDS ----
        const int ND = P + 1;  // ranks a read can ask for: 0 .. (distinct keys) <= P
        const int n1 = ND / RB1 + 1, n2 = ND / RB2 + 1;
        auto ev = [](int n) { return (n + 1) & ~1; };  // (every array 4-byte aligned: lds_min16)
        uint16_t* val = r16;
        uint16_t* vb1 = val + ev(ND + 1);
        uint16_t* vb2 = vb1 + ev(n1 + 1);
        uint16_t* stab = vb2 + ev(n2 + 1);
        uint16_t* st1 = stab + ev(ND + 1);
        uint16_t* st2 = st1 + ev(n1 + 1);
        const int nwords16 = (int)(st2 + ev(n2 + 1) - val);
        const int nw = s_nw, ni = s_nw + s_nr;
        const int lcap = A.lcap;
        auto item = [&](int j) { return j < lcap ? litems[j] : A.items[j]; };  // (past lcap: global)
        int rounds = 0;
        for (;;) {
            rounds++;
            for (int i = tid; 2 * i < nwords16; i += nthr) reinterpret_cast<uint32_t*>(val)[i] = 0xFFFFFFFFu;
            __syncthreads();
            for (int j = tid; j < nw; j += nthr) {  // writes of the candidates
                const uint2 it = item(j);
                const int u = (int)it.y;
                if (!bit_of(cbits, u)) continue;
                const int B = it.x & 0xFFFF, E = it.x >> 16;
                lds_min16(val, B, (uint16_t)u);
                blocks_of(B + 1, E + 1, [&](int q) { lds_min16(stab, q, (uint16_t)u); },
                          [&](int q) { lds_min16(st1, q, (uint16_t)u); }, [&](int q) { lds_min16(st2, q, (uint16_t)u); });
            }
            __syncthreads();
            for (int j = tid; j < n1; j += nthr) {  // block minima of val
                uint16_t m = INF16;
                for (int q = j * RB1; q < min(ND, (j + 1) * RB1); q++) m = min(m, val[q]);
                vb1[j] = m;
            }
            __syncthreads();
            for (int j = tid; j < n2; j += nthr) {
                uint16_t m = INF16;
                for (int q = j * (RB2 / RB1); q < min(n1, (j + 1) * (RB2 / RB1)); q++) m = min(m, vb1[q]);
                vb2[j] = m;
            }
            __syncthreads();
            for (int j = nw + tid; j < ni; j += nthr) {  // candidate reads
                const uint2 it = item(j);
                const int t = (int)it.y;
                if (bit_of(nbits, t)) continue;
                const int gb = it.x & 0xFFFF, ge = it.x >> 16;
                uint16_t m = min(stab[gb], min(st1[gb / RB1], st2[gb / RB2]));
                blocks_of(gb, ge, [&](int q) { m = min(m, val[q]); }, [&](int q) { m = min(m, vb1[q]); },
                          [&](int q) { m = min(m, vb2[q]); });
                if (m < t) atomicOr(&nbits[t >> 5], 1u << (t & 31));  // a committed u < t
            }
            __syncthreads();
            bool changed = false;
            for (int i = tid; i < nwords; i += nthr) {
                const uint32_t c = ubits[i] & ~nbits[i];
                changed |= c != cbits[i];
                cbits[i] = c;
                nbits[i] = 0;
            }
            if (!__syncthreads_or(changed)) break;
            if (rounds == 1) PHASE(sc, 4);
        }
        if (tid == 0) sc->jac_iters = rounds;
    }
decided:
    PHASE(sc, 5);
    {
        // 16 transactions per lane, one 16-byte store each of verdicts and
        // committed flags: into host-mapped memory that is one PCIe write per
        // 16 verdicts instead of one per verdict (byte stores made the flag
        // ~20 us late at T = 5,000)
        const bool al16 = ((reinterpret_cast<uintptr_t>(A.verdict) | reinterpret_cast<uintptr_t>(A.committed)) & 15) == 0;
        for (int t0 = 16 * tid; t0 < T; t0 += 16 * nthr) {
            const uint32_t cw = cbits[t0 >> 5] >> (t0 & 31);  // (t0 % 32 is 0 or 16; bits past T are 0)
            const uint32_t tw = tbits[t0 >> 5] >> (t0 & 31);
            uint32_t vw[4] = {0, 0, 0, 0}, cm[4] = {0, 0, 0, 0};
#pragma unroll
            for (int k = 0; k < 16; k++) {
                const uint32_t c = (cw >> k) & 1;
                const uint32_t v = c ? FDBCS_COMMITTED : (((tw >> k) & 1) ? FDBCS_TOO_OLD : FDBCS_CONFLICT);
                vw[k >> 2] |= v << (8 * (k & 3));
                cm[k >> 2] |= c << (8 * (k & 3));
            }
            if (al16 && t0 + 16 <= T) {
                *reinterpret_cast<uint4*>(A.verdict + t0) = make_uint4(vw[0], vw[1], vw[2], vw[3]);
                *reinterpret_cast<uint4*>(A.committed + t0) = make_uint4(cm[0], cm[1], cm[2], cm[3]);
            } else {
                for (int k = 0; k < 16 && t0 + k < T; k++) {
                    A.verdict[t0 + k] = (uint8_t)(vw[k >> 2] >> (8 * (k & 3)));
                    A.committed[t0 + k] = (uint8_t)(cm[k >> 2] >> (8 * (k & 3)));
                }
            }
        }
    }
    if (A.eo.flag) {
        // host-mapped verdicts: every lane's stores and the error words, a
        // system-scope fence, then the flag (a plain store after the fence
        // stayed in L2 until the workgroup ended: the host saw the flag ~19 us
        // late, after the combine below)
        if (tid == 0) {
            A.eo.flag[1] = eo_err;
            A.eo.flag[2] = eo_last;
            A.eo.flag[3] = eo_lm;
            A.eo.flag[4] = eo_shmax;
        }
        __threadfence_system();
        __syncthreads();
        if (tid == 0) {
#ifndef FDBCS_FLAG_STORE
            // the flag as a system-scope exchange: an atomic is performed at
            // the host's memory, so nothing holds it back and no second fence
            // is needed (flag 1.7 us sooner by the decision's own clock)
            (void)__hip_atomic_exchange(A.eo.flag, A.eo.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
#else  // (A/B: the store and a second fence, round 4's first form)
            __hip_atomic_store(A.eo.flag, A.eo.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            __threadfence_system();
#endif
        }
    }
    PHASE(sc, 1);
    if (tid == 0) {
        sc->n_dep = ncand;  // candidate reads of U (stats)
        if (ncand == 0) sc->jac_iters = 0;
        sc->dec_wide = 0;
        sc->n_pot = 0;
        sc->edges_total = 0;
    }
    if (!A.combine) return;  // (committed[] is read by the multi-block combine)
    // ---- combine ----
    // committed flag per write, 32 writes per thread-word
    for (int i = tid; i < wwords; i += nthr) {
        // write_txn is padded to a multiple of 32 entries: eight 16-byte loads
        const int4* src = reinterpret_cast<const int4*>(A.write_txn + 32 * i);
        int4 v[8];
#pragma unroll
        for (int k = 0; k < 8; k++) v[k] = src[k];
        uint32_t m = 0;
        const int w0 = 32 * i;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const int us[4] = {v[k].x, v[k].y, v[k].z, v[k].w};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int u = us[q];
                if (w0 + 4 * k + q < W) m |= ((cbits[u >> 5] >> (u & 31)) & 1u) << (4 * k + q);
            }
        }
        cwb[i] = m;
    }
    __syncthreads();
    PHASE(sc, 6);
    const int CP = (P + nthr - 1) / nthr;
    const int q0 = min(P, tid * CP), q1 = min(P, q0 + CP);
    int gtot;
    // this thread's endpoints live in registers for all three passes (2W <= CPMAX * DC_THREADS)
    uint32_t slot[CPMAX];
    int8_t dd[CPMAX];
#pragma unroll
    for (int k = 0; k < CPMAX; k++) slot[k] = q0 + k < q1 ? A.sw_slot[q0 + k] : 0;
    int dsum = 0;
#pragma unroll
    for (int k = 0; k < CPMAX; k++) {
        const int w = (int)((slot[k] - wbase) >> 1);
        const bool com = q0 + k < q1 && ((cwb[w >> 5] >> (w & 31)) & 1);
        dd[k] = com ? ((slot[k] & 1) ? -1 : 1) : 0;
        dsum += dd[k];
    }
    PHASE(sc, 7);
    int dtot;
    const int cnt0 = block_excl_scan(dsum, red32, dtot);
    int ns = 0, c2 = cnt0;
#pragma unroll
    for (int k = 0; k < CPMAX; k++) {
        ns += dd[k] == 1 && c2 == 0;  // counter 0 -> 1: a combined range opens
        c2 += dd[k];
    }
    PHASE(sc, 8);
    int g = block_excl_scan(ns, red32, gtot);
    c2 = cnt0;
#pragma unroll
    for (int k = 0; k < CPMAX; k++) {
        if (dd[k] == 1 && c2 == 0) A.cb_pos[g++] = q0 + k;
        if (dd[k] == -1 && c2 == 1) A.ce_pos[g - 1] = q0 + k;  // counter 1 -> 0: it closes
        c2 += dd[k];
    }
    PHASE(sc, 9);
    if (tid == 0) sc->n_comb = gtot;
}

// ---------------------------------------------- multi-block combine ----
// For batches whose 2W sorted write endpoints exceed what one workgroup keeps
// in registers: the same sweep (combineWriteConflictRanges,
// SkipList.cpp:1320-1337) as three grid launches over blocks of CB_BLOCK
// consecutive endpoints.  d(p) = +1 / -1 at a committed BEGIN / END, else 0;
// the open-write counter before a block is the sum of d over its
// predecessors; a range opens where the counter goes 0 -> 1 and closes where
// it returns to 0.
//   k_comb_sum  : per-block sum of d
//   k_comb_open : counter at the block start (predecessor sums), opens per block
//   k_comb_emit : both prefixes, every range's begin / end slot; n_comb
static constexpr int CB_THREADS = 256, CB_ITEMS = 16, CB_BLOCK = CB_THREADS * CB_ITEMS;

struct CombArgs {
    int P;
    int64_t wbase;
    const uint32_t* sw_slot;
    const int32_t* write_txn;
    const uint8_t* committed;
    int32_t* bsum;   // [blocks]
    int32_t* bopen;  // [blocks]
    int32_t* cb_pos;
    int32_t* ce_pos;
    Scalars* sc;
};

// this thread's CB_ITEMS endpoints: d values (and slots)
__device__ inline int comb_load(const CombArgs& A, int8_t (&d)[CB_ITEMS], uint32_t (&slot)[CB_ITEMS]) {
    const int p0 = blockIdx.x * CB_BLOCK + threadIdx.x * CB_ITEMS;
    uint32_t w[CB_ITEMS];
#pragma unroll
    for (int k = 0; k < CB_ITEMS; k++) slot[k] = p0 + k < A.P ? A.sw_slot[p0 + k] : 0;
#pragma unroll
    for (int k = 0; k < CB_ITEMS; k++) w[k] = p0 + k < A.P ? A.write_txn[(slot[k] - A.wbase) >> 1] : 0;
    int sum = 0;
#pragma unroll
    for (int k = 0; k < CB_ITEMS; k++) {
        const bool com = p0 + k < A.P && A.committed[w[k]];
        d[k] = com ? ((slot[k] & 1) ? -1 : 1) : 0;
        sum += d[k];
    }
    return sum;
}

// sum of x[0 .. nblk) by wave 0, broadcast through LDS
__device__ inline int pred_sum(const int32_t* x, int nblk, int* s_out) {
    if (threadIdx.x < 64) {
        int acc = 0;
        for (int k = threadIdx.x; k < nblk; k += 64) acc += x[k];
        acc = wave_reduce_sum(acc);
        if (threadIdx.x == 0) *s_out = acc;
    }
    __syncthreads();
    return *s_out;
}

__global__ __launch_bounds__(CB_THREADS) void k_comb_sum(CombArgs A) {
    __shared__ int32_t red[CB_THREADS / 64 + 1];
    int8_t d[CB_ITEMS];
    uint32_t slot[CB_ITEMS];
    int tot;
    block_excl_scan(comb_load(A, d, slot), red, tot);
    if (threadIdx.x == 0) A.bsum[blockIdx.x] = tot;
}

__global__ __launch_bounds__(CB_THREADS) void k_comb_open(CombArgs A) {
    __shared__ int32_t red[CB_THREADS / 64 + 1];
    __shared__ int s0;
    int8_t d[CB_ITEMS];
    uint32_t slot[CB_ITEMS];
    const int sum = comb_load(A, d, slot);
    const int c0 = pred_sum(A.bsum, blockIdx.x, &s0);
    int tot;
    int c = c0 + block_excl_scan(sum, red, tot);
    int opens = 0;
#pragma unroll
    for (int k = 0; k < CB_ITEMS; k++) {
        opens += d[k] == 1 && c == 0;
        c += d[k];
    }
    block_excl_scan(opens, red, tot);
    if (threadIdx.x == 0) A.bopen[blockIdx.x] = tot;
}

__global__ __launch_bounds__(CB_THREADS) void k_comb_emit(CombArgs A) {
    __shared__ int32_t red[CB_THREADS / 64 + 1];
    __shared__ int s0, s1;
    int8_t d[CB_ITEMS];
    uint32_t slot[CB_ITEMS];
    const int sum = comb_load(A, d, slot);
    const int c0 = pred_sum(A.bsum, blockIdx.x, &s0);
    const int g0 = pred_sum(A.bopen, blockIdx.x, &s1);
    int tot;
    const int cs = c0 + block_excl_scan(sum, red, tot);
    int c = cs, opens = 0;
#pragma unroll
    for (int k = 0; k < CB_ITEMS; k++) {
        opens += d[k] == 1 && c == 0;
        c += d[k];
    }
    int gtot;
    int g = g0 + block_excl_scan(opens, red, gtot);
    c = cs;
#pragma unroll
    for (int k = 0; k < CB_ITEMS; k++) {
        if (d[k] == 1 && c == 0) A.cb_pos[g++] = blockIdx.x * CB_BLOCK + threadIdx.x * CB_ITEMS + k;
        if (d[k] == -1 && c == 1) A.ce_pos[g - 1] = blockIdx.x * CB_BLOCK + threadIdx.x * CB_ITEMS + k;  // (the open may lie in an earlier block)
        c += d[k];
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) A.sc->n_comb = g0 + gtot;
}

static void launch_combine_grid(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, hipStream_t s) {
    const int P = 2 * v.write_count;
    const int nblk = cdiv(P, CB_BLOCK);
    CombArgs C{P, write_base(b, v), b.sw_slot, b.write_txn, b.committed, b.comb_blk,
               b.comb_blk + nblk + 1, b.cb_pos, b.ce_pos, sc};
    hipLaunchKernelGGL(k_comb_sum, dim3(nblk), dim3(CB_THREADS), 0, s, C);
    hipLaunchKernelGGL(k_comb_open, dim3(nblk), dim3(CB_THREADS), 0, s, C);
    hipLaunchKernelGGL(k_comb_emit, dim3(nblk), dim3(CB_THREADS), 0, s, C);
}

// ------------------------------------------------------ grid decision ----
// For batches past one workgroup's LDS / register budget.  The same rule
// (checkIntraBatchConflicts, SkipList.cpp:1133-1153) in three launches:
//   k_dec_flags : a lane per txn: undecided = !tooOld && !history conflict;
//                 with no intra-batch source (deg from the edge kernel) it is
//                 final; per-block counts of dependents and their sources
//   k_dec_place : dependents' positions in index order and their CSR offsets
//                 (predecessor sums + a block scan)
//   k_dec_walk  : one workgroup: the CSR of the dependents' sources, the
//                 committed bits in LDS, and the ordered walk in chunks of 64
//                 (Jacobi on ballots, as in k_decide_combine)
static constexpr int DG_THREADS = 256;

struct DecGridArgs {
    int T;
    const uint8_t* too_old;
    const uint8_t* hist;
    const int32_t* deg;
    const int32_t* et;
    const int32_t* eu;
    int64_t edge_cap;
    int32_t* bd;        // [blocks] dependents per block
    int32_t* be;        // [blocks] their sources per block
    int32_t* didx;      // [T] dependent index or -1
    int32_t* dep_list;  // [T] dependents in index order
    int32_t* doff;      // [ndep + 1] CSR offsets per dependent
    int32_t* cur;       // [ndep] CSR fill cursors
    int32_t* csr;
    uint8_t* committed;
    uint64_t* cbits;    // [T / 64 + 1] committed as bits (k_dec_flags), for k_dec_walk's LDS copy
    uint8_t* verdict;
    Scalars* sc;
};

__device__ inline uint8_t verdict_of(bool committed, bool too_old) {
    return committed ? FDBCS_COMMITTED : (too_old ? FDBCS_TOO_OLD : FDBCS_CONFLICT);
}

__global__ __launch_bounds__(DG_THREADS) void k_dec_flags(DecGridArgs A) {
    __shared__ int64_t red[DG_THREADS / 64 + 1];
    const int t = blockIdx.x * DG_THREADS + threadIdx.x;
    bool dep = false;
    int d = 0;
    if (t < A.T) {
        const bool to = A.too_old[t];
        const bool und = !to && !A.hist[t];
        d = A.deg[t];
        dep = und && d > 0;
        A.committed[t] = und && !dep;  // (a dependent starts uncommitted)
        if (!dep) A.verdict[t] = verdict_of(und, to);
    }
    {  // the same as bits for k_dec_walk: a wavefront's 64 transactions are one aligned word
        const uint64_t m = __ballot(t < A.T && !dep && A.committed[t]);
        if ((threadIdx.x & 63) == 0 && t < A.T) A.cbits[t >> 6] = m;
    }
    int64_t tot;
    block_excl_scan(dep ? ((int64_t)1 << 32) | (uint32_t)d : (int64_t)0, red, tot);
    if (threadIdx.x == 0) {
        A.bd[blockIdx.x] = (int32_t)(tot >> 32);
        A.be[blockIdx.x] = (int32_t)(uint32_t)tot;
    }
}

__global__ __launch_bounds__(DG_THREADS) void k_dec_place(DecGridArgs A) {
    __shared__ int64_t red[DG_THREADS / 64 + 1];
    __shared__ int s0, s1;
    const int t = blockIdx.x * DG_THREADS + threadIdx.x;
    const int nd0 = pred_sum(A.bd, blockIdx.x, &s0);
    const int eo0 = pred_sum(A.be, blockIdx.x, &s1);
    bool dep = false;
    int d = 0;
    if (t < A.T) {
        d = A.deg[t];
        dep = !A.too_old[t] && !A.hist[t] && d > 0;
    }
    int64_t tot;
    const int64_t ex = block_excl_scan(dep ? ((int64_t)1 << 32) | (uint32_t)d : (int64_t)0, red, tot);
    if (t < A.T) {
        const int k = nd0 + (int)(ex >> 32);
        A.didx[t] = dep ? k : -1;
        if (dep) {
            A.dep_list[k] = t;
            A.doff[k] = eo0 + (int)(uint32_t)ex;
            A.cur[k] = 0;
        }
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) {
        const int nd = nd0 + (int)(tot >> 32);
        A.doff[nd] = eo0 + (int)(uint32_t)tot;
        A.sc->n_dep = nd;
    }
}

__global__ __launch_bounds__(1024) void k_dec_walk(DecGridArgs A) {
    extern __shared__ uint32_t cbits[];  // committed, a bit per txn
    const int T = A.T, tid = threadIdx.x, nthr = blockDim.x;
    Scalars* sc = A.sc;
    const int E = (int)min((int64_t)sc->edges_total, A.edge_cap);
    const int ndep = sc->n_dep;
    const uint32_t* cb32 = reinterpret_cast<const uint32_t*>(A.cbits);  // (little-endian halves of the words)
    for (int i = tid; i < (T + 31) / 32; i += nthr) cbits[i] = cb32[i];
    for (int e = tid; e < E; e += nthr) {
        const int t = A.et[e], u = A.eu[e];
        const int k = A.didx[t];
        if (k >= 0) A.csr[A.doff[k] + atomicAdd(&A.cur[k], 1)] = u;
    }
    __syncthreads();
    int iters = 0;
    if (tid < 64) {
        const int lane = tid;
        for (int c0 = 0; c0 < ndep; c0 += 64) {
            const int k = c0 + lane;
            const bool valid = k < ndep;
            const int t = valid ? A.dep_list[k] : 0;
            bool ext = false;
            uint64_t L = 0;
            if (valid) {
                for (int e = A.doff[k], e1 = A.doff[k + 1]; e < e1 && !ext; e++) {
                    const int u = A.csr[e];
                    const int di = A.didx[u];
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
            const bool c = valid && ((cm >> lane) & 1);
            if (c) atomicOr(&cbits[t >> 5], 1u << (t & 31));
            if (valid) {
                A.committed[t] = c;
                A.verdict[t] = verdict_of(c, false);  // (a dependent is not tooOld)
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
        }
    }
    if (tid == 0) {
        sc->jac_iters = iters;
        sc->edges_total = 0;  // next batch starts a new edge list
    }
}

bool launch_decide(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, uint8_t* verdict, hipStream_t s,
                   bool split, const EarlyOut* eo, HistBufs* h, int cur, int64_t v0) {
    const int T = v.txn_count;
    if (T == 0) return false;  // n_comb was zeroed by k_prep
    const int P = 2 * v.write_count;
    const int force_multi = getenv("FDBCS_TEST_MULTIBLOCK_COMBINE") ? 1 : 0;  // (tests)
    const bool multi = P > 0 && (P > CPMAX * DC_THREADS || force_multi || split);
    if (!b.rounds) {  // large or sparse batches: the overlap edges' grid decision, then the multi-block combine
        const int nb = cdiv(T, DG_THREADS);
        DecGridArgs G;
        G.T = T; G.too_old = b.too_old; G.hist = b.hist; G.deg = b.deg; G.et = b.et; G.eu = b.eu;
        G.edge_cap = b.edge_cap;
        G.bd = b.dec_blk; G.be = b.dec_blk + nb + 1; G.didx = b.dep_idx; G.dep_list = b.dep_list; G.doff = b.off;
        G.cur = b.cur; G.csr = b.csr; G.committed = b.committed; G.cbits = b.cbits; G.verdict = verdict; G.sc = sc;
        hipLaunchKernelGGL(k_dec_flags, dim3(nb), dim3(DG_THREADS), 0, s, G);
        hipLaunchKernelGGL(k_dec_place, dim3(nb), dim3(DG_THREADS), 0, s, G);
        hipLaunchKernelGGL(k_dec_walk, dim3(1), dim3(1024), (size_t)((T + 31) / 32) * 4, s, G);
        if (P > 0 && !split) launch_combine_grid(v, b, sc, s);
        return false;
    }
    RoundArgs A;
    A.T = T; A.R = v.read_count; A.W = v.write_count;
    A.wbase = write_base(b, v);
    A.combine = multi ? 0 : 1;
    const size_t base = rounds_lds_base(T, v.write_count);
    A.lcap = (int)std::min<int64_t>((int64_t)(ROUNDS_LDS_MAX - base) / 8, (int64_t)v.read_count + v.write_count);
    if (const char* c = getenv("FDBCS_TEST_ROUNDS_LCAP")) A.lcap = std::min(A.lcap, atoi(c));  // (tests: global items)
    A.too_old = b.too_old; A.hist = b.hist; A.read_txn = b.read_txn; A.write_txn = b.write_txn;
    A.rq = b.rq; A.plist = b.plist; A.wnew = b.wnew; A.winv = b.winv; A.sw_slot = b.sw_slot; A.items = b.items; A.lcap_list = b.list_cap;
    A.committed = b.committed; A.verdict = verdict; A.cb_pos = b.cb_pos; A.ce_pos = b.ce_pos; A.sc = sc;
    A.eo = EarlyOut{};
    if (eo) {
        A.eo = *eo;
        A.verdict = eo->verdict;
    }
    int wsb = 0;  // the deferred write searches ride in the same launch
    if (h && b.ws_deferred && v.write_count > 0) {
        b.ws_deferred = false;
        A.ws = WriteSearchArgs{v.read_count, v.write_count, b.keys, h->pool, h->dir[cur], sc, v0, b.wh, nullptr,
                               write_base(b, v)};
        wsb = cdiv((int64_t)v.write_count * RC_G, DC_THREADS);
    }
    A.eblocks = 0;  // the edge lanes too, when launch_edges_read_check left them (b.edges_fused)
    size_t shm = base + 8 * (size_t)A.lcap;
    if (b.edges_fused) {
        b.edges_fused = false;
        A.ea = make_edges_args(v, b, sc);
        A.eblocks = cdiv((int64_t)v.read_count + fused_edge_quads(v.write_count), DC_THREADS);
        shm = std::max<size_t>(shm, EQ * sizeof(uint64_t));  // (an edge block's sample of the sorted writes)
    }
    hipLaunchKernelGGL(k_decide_rounds, dim3(1 + A.eblocks + wsb), dim3(DC_THREADS), shm, s, A);
    if (multi && !split) launch_combine_grid(v, b, sc, s);
    return eo != nullptr;
}

// the combine of a split launch_decide (after the verdicts have been sent)
void launch_combine(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, hipStream_t s) {
    if (v.txn_count > 0 && v.write_count > 0) launch_combine_grid(v, b, sc, s);
}

// ---- exact sharded mode: exchange flags, foreign edges -------------------
__global__ __launch_bounds__(256) void k_flags_out(int T, const uint8_t* __restrict__ too_old,
                                                   const uint8_t* __restrict__ hist, uint8_t* __restrict__ flags) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < T) flags[t] = too_old[t] ? 2 : (hist[t] ? 1 : 0);
}

__global__ __launch_bounds__(256) void k_flags_in(int T, const uint8_t* __restrict__ flags,
                                                  uint8_t* __restrict__ too_old, uint8_t* __restrict__ hist) {
    const int t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t < T) {
        const uint8_t f = flags[t];
        too_old[t] = f == 2;
        hist[t] = f == 1;
    }
}

// the union of every shard's overlap edges replaces this shard's own; the
// per-reader source counts are recounted from it
__global__ __launch_bounds__(256) void k_set_edges(const int32_t* __restrict__ et, const int32_t* __restrict__ eu,
                                                   int64_t n, int32_t* __restrict__ det, int32_t* __restrict__ deu,
                                                   int32_t* __restrict__ deg, Scalars* sc) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) sc->edges_total = (int32_t)n;
    if (i >= n) return;
    const int32_t t = et[i];
    det[i] = t;
    deu[i] = eu[i];
    atomicAdd(&deg[t], 1);
}

void launch_flags_out(const BatchBufs& b, int T, uint8_t* flags, hipStream_t s) {
    if (T > 0) hipLaunchKernelGGL(k_flags_out, dim3(cdiv(T, 256)), dim3(256), 0, s, T, b.too_old, b.hist, flags);
}

void launch_flags_in(BatchBufs& b, int T, const uint8_t* flags, hipStream_t s) {
    if (T > 0) hipLaunchKernelGGL(k_flags_in, dim3(cdiv(T, 256)), dim3(256), 0, s, T, flags, b.too_old, b.hist);
}

// n < 0: the count is sc->edges_total (set on the device), at most -n
__global__ __launch_bounds__(256) void k_set_edges_dev(const int32_t* __restrict__ et, const int32_t* __restrict__ eu,
                                                       int32_t* __restrict__ det, int32_t* __restrict__ deu,
                                                       int32_t* __restrict__ deg, const Scalars* sc) {
    const int64_t n = sc->edges_total;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const int32_t t = et[i];
        det[i] = t;
        deu[i] = eu[i];
        atomicAdd(&deg[t], 1);
    }
}
void launch_set_edges(BatchBufs& b, Scalars* sc, int T, const int32_t* et, const int32_t* eu, int64_t n,
                      hipStream_t s) {
    if (n < 0) {  // (the device's count, sh_exchange_b)
        if (T > 0) hipMemsetAsync(b.deg, 0, (size_t)T * sizeof(int32_t), s);
        hipLaunchKernelGGL(k_set_edges_dev, dim3((unsigned)std::max<int64_t>(1, std::min<int64_t>(1024, cdiv(-n, 256)))),
                           dim3(256), 0, s, et, eu, b.et, b.eu, b.deg, (const Scalars*)sc);
        return;
    }
    if (T > 0) hipMemsetAsync(b.deg, 0, (size_t)T * sizeof(int32_t), s);
    hipLaunchKernelGGL(k_set_edges, dim3(std::max(1, cdiv(n, 256))), dim3(256), 0, s, et, eu, n, b.et, b.eu, b.deg,
                       sc);
}

}  // namespace fdbcs_dev

namespace fdbcs_dev {
// Kernels use up to 160 KiB of dynamic LDS, which gfx950 grants without an
// opt-in attribute; nothing to configure.  Clear any stale runtime error so it
// is not reported by an unrelated later call.
void configure_batch_kernels() { (void)hipGetLastError(); }
}  // namespace fdbcs_dev
