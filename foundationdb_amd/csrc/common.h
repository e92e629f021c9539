// common.h -- shared device-side definitions for the MI355X conflict-set engine.
//
// Key encoding.  A key of length L is held as
//   hi   = big-endian bytes [0, 8)   (zero padded)
//   lo   = big-endian bytes [8, 16)  (zero padded)
//   meta = (byte[16] << 24) | L      (byte[16] = 0 if L <= 16)
//   tail = device pointer to bytes [17, L), 8-byte aligned and zero padded to
//          a multiple of 8 -- only meaningful when L > 17.
// (hi, lo, meta) compared as unsigned integers order any two keys exactly as
// the reference's compare() (fdbserver/SkipList.cpp:113-120) unless both keys
// are longer than 17 bytes and share their first 17 bytes; only then are the
// tails consulted (8 bytes at a time, big-endian).  Point ranges [k, k\x00)
// (fdbclient/FDBTypes.h:288-291) of 16-byte keys therefore never touch a tail.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdbcs_dev {

constexpr int SS_QT = 64;          // tail bytes kept per sort splitter (longer ones are compared as prefixes)
constexpr int PAGE = 256;          // history page capacity (boundaries)
#ifndef FDBCS_FILL  // (page shape knobs: scripts/build_variants.sh A/B)
#define FDBCS_FILL 192
#endif
#ifndef FDBCS_SPLIT
#define FDBCS_SPLIT 224
#endif
#ifndef FDBCS_HOLE_EVERY
#define FDBCS_HOLE_EVERY 3
#endif
constexpr int FILL = FDBCS_FILL;   // target fill when a page is split / repacked
constexpr int SPLIT = FDBCS_SPLIT; // a merge splits a page whose boundaries would exceed this
constexpr int HOLE_EVERY = FDBCS_HOLE_EVERY;  // a rewritten page holds a hole after every 3rd boundary (at most)
static_assert(FILL <= SPLIT && SPLIT <= PAGE && HOLE_EVERY >= 1, "page shape");
constexpr uint32_t LEN_MASK = 0xFFFFFFu;

struct Key {
    uint64_t hi, lo;
    uint32_t meta;
    const uint8_t* tail;
};

__device__ __host__ inline int cdiv(int64_t a, int64_t b) { return (int)((a + b - 1) / b); }

__device__ __host__ inline uint32_t key_len(uint32_t meta) { return meta & LEN_MASK; }

__device__ inline uint64_t load_be64(const uint8_t* p) {
    uint64_t x = *reinterpret_cast<const uint64_t*>(p);
    return __builtin_bswap64(x);
}

// Compare the tails (bytes 17..) of two keys that both have length > 17 and
// identical first 17 bytes.  Tails are 8-byte aligned and zero padded.  Six
// words of each tail per step, their loads issued together (keys sharing a
// long prefix -- tenants, paths -- differ only words in; one dependent load
// per word made every such compare a chain of round trips).  Config 4 (keys
// sharing 64 bytes, so the first difference sits in tail word 5): read check
// 274 us with 4 words per step, 252 with 6, 256 with 8
// (profiles/r03_ab_tail_chunk.txt).
#ifndef FDBCS_TAIL_CHUNK
#define FDBCS_TAIL_CHUNK 6
#endif
__device__ inline int tail_cmp(const uint8_t* ta, uint32_t la, const uint8_t* tb, uint32_t lb) {
    constexpr uint32_t C = FDBCS_TAIL_CHUNK;
    const uint32_t m = (la < lb ? la : lb) - 17;
    const uint32_t words = (m + 7) >> 3;
    const uint64_t* a = reinterpret_cast<const uint64_t*>(ta);
    const uint64_t* b = reinterpret_cast<const uint64_t*>(tb);
    for (uint32_t w = 0; w < words; w += C) {
        uint64_t x[C], y[C];
#pragma unroll
        for (uint32_t k = 0; k < C; k++) {
            const bool ok = w + k < words;  // (never past a tail's last word)
            x[k] = ok ? a[w + k] : 0;
            y[k] = ok ? b[w + k] : 0;
        }
#pragma unroll
        for (uint32_t k = 0; k < C; k++) {
            if (x[k] != y[k]) return __builtin_bswap64(x[k]) < __builtin_bswap64(y[k]) ? -1 : 1;
        }
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}

__device__ inline int kcmp(uint64_t ahi, uint64_t alo, uint32_t am, const uint8_t* at,
                           uint64_t bhi, uint64_t blo, uint32_t bm, const uint8_t* bt) {
    if (ahi != bhi) return ahi < bhi ? -1 : 1;
    if (alo != blo) return alo < blo ? -1 : 1;
    if (am == bm) {
        if (key_len(am) <= 17) return 0;
        return tail_cmp(at, key_len(am), bt, key_len(bm));
    }
    uint32_t ab = am >> 24, bb = bm >> 24;
    if (ab != bb) return ab < bb ? -1 : 1;
    uint32_t la = key_len(am), lb = key_len(bm);
    if (la > 17 && lb > 17) return tail_cmp(at, la, bt, lb);
    return la < lb ? -1 : 1;
}

__device__ inline int kcmp(const Key& a, const Key& b) {
    return kcmp(a.hi, a.lo, a.meta, a.tail, b.hi, b.lo, b.meta, b.tail);
}

__device__ __noinline__ bool key_lt_tail(const Key& a, const Key& b) {
    return tail_cmp(a.tail, key_len(a.meta), b.tail, key_len(b.meta)) < 0;
}

// a < b, branch-free unless both keys are > 17 bytes and equal on 17 bytes
__device__ inline bool key_lt(const Key& a, const Key& b) {
    const bool heq = a.hi == b.hi, leq = a.lo == b.lo;
    const bool tail_case = heq & leq & ((a.meta >> 24) == (b.meta >> 24)) & (key_len(a.meta) > 17) &
                           (key_len(b.meta) > 17);
    if (__builtin_expect(tail_case, 0)) return key_lt_tail(a, b);
    return (a.hi < b.hi) | (heq & ((a.lo < b.lo) | (leq & (a.meta < b.meta))));
}

__device__ inline bool key_le(const Key& a, const Key& b) { return !key_lt(b, a); }

// Sort record: a key's fixed-width part plus its key slot (32 B so that LDS
// copies are two ds_read_b128).
struct __attribute__((aligned(16))) SRec {
    uint64_t hi, lo;
    uint32_t meta, idx;
    uint64_t pad;
};



// ---- Structure-of-arrays views -------------------------------------------------

struct KeyArrays {           // one key per slot
    uint64_t* hi;
    uint64_t* lo;
    uint32_t* meta;
    const uint8_t** tail;
    __device__ Key get(int64_t i) const { return Key{hi[i], lo[i], meta[i], tail[i]}; }
    // the tail pointer only for a key past 17 bytes (the only one that has
    // a tail): a random 8-byte load saved per short key, at the cost of a
    // dependent load for long ones
    __device__ Key get_short(int64_t i) const {
        const uint32_t m = meta[i];
        return Key{hi[i], lo[i], m, key_len(m) > 17 ? tail[i] : nullptr};
    }
    __device__ void put(int64_t i, const Key& k) const {
        hi[i] = k.hi; lo[i] = k.lo; meta[i] = k.meta; tail[i] = k.tail;
    }
};

// Key range [lo, hi) of a shard in the exact sharded mode (SURVEY.md §8e
// protocol A); has_lo / has_hi == 0: unbounded.  Keys live in device memory.
struct ShardBounds {
    Key lo, hi;
    int32_t has_lo, has_hi;
    __device__ bool below(const Key& k) const;   // k < lo
    __device__ bool at_or_above(const Key& k) const;  // k >= hi
};


// The history: a pool of pages (PAGE slots each) plus a directory that lists
// live pages in key order.  Page 0 of the directory may be empty only when it
// is the only page (empty history).
struct Pool {
    uint64_t* hi;
    uint64_t* lo;
    uint32_t* meta;
    int64_t* ver;
    const uint8_t** tail;
    // page index: pidx[s / 16] = hi[s] for every slot s that is a multiple of
    // 16 (16 per page = one 128-byte line), kept by every slot writer
    // (put_entry); the first step of a cooperative page search reads it.
    uint64_t* pidx;
    // holes: bit i of hmask[4 * page + i / 64] marks slot i of the page as a
    // hole (below).  Bits at or above the page's slot count are zero.
    uint64_t* hmask;
    // Long shared prefixes (config 4): px[s] = 8 bytes of slot s's key from
    // byte pskip[page] (common.h key_bytes_at), pxidx = px of slots 0, 16,
    // ..., 240 (one line per page, as pidx).  A search in a page uses them
    // when 0 < pskip <= the skip of the page's directory window (Dir::wsk):
    // then every key of the page and every query reaching it share their
    // first pskip bytes.  pskip < 0: the page was rewritten and k_page_px
    // sets it anew after the batch; 0: not used.
    uint64_t* px;
    uint64_t* pxidx;
    int32_t* pskip;
};
constexpr int PIDX_STRIDE = 16;
constexpr int HM_WORDS = PAGE / 64;

// Page slack ("holes").  Inserting into a dense sorted page moves every slot
// after the insertion point; instead a page keeps holes spread through it and
// an insertion moves only the slots up to the next hole (kernels_hist.hip
// k_page_merge).  A hole is an exact copy (key, version, tail pointer) of the
// real boundary before it, so lower bounds, range maxima and valueBefore read
// through holes unchanged; only global indices (start[], the compaction
// window, dumps) count real boundaries, and slot 0 of a page is always real.
// A page written with n real boundaries holds them at slot m + m / g
// (spread_slot) -- a hole after every g-th -- using spread_used(n) slots.
__host__ __device__ inline int spread_gap(int n) {
    if (n >= PAGE) return PAGE + 1;  // dense
    const int g = (n - 1) / (PAGE - n + 1) + 1;  // smallest g with (n-1)/g <= PAGE-n
    return g > HOLE_EVERY ? g : HOLE_EVERY;
}
__host__ __device__ inline int spread_slot(int m, int g) { return m + m / g; }
__host__ __device__ inline int spread_used(int n) { return n > 0 ? spread_slot(n - 1, spread_gap(n)) + 1 : 0; }
// a hole follows real boundary m (< n) of a spread page
__host__ __device__ inline bool spread_hole_after(int m, int n, int g) { return (m + 1) % g == 0 && m + 1 < n; }
// word w of the hole mask of a page spread with n boundaries: holes are the
// used slots s with s % (g + 1) == g
__host__ __device__ inline uint64_t spread_mask_word(int n, int w) {
    const int g = spread_gap(n), used = spread_used(n);
    uint64_t m = 0;
    if (g > PAGE) return 0;
    const int lo = 64 * w;
    int s = lo + ((g - lo % (g + 1)) + (g + 1)) % (g + 1);  // first s >= lo with s % (g+1) == g
    for (; s < lo + 64 && s < used; s += g + 1) m |= 1ull << (s - lo);
    return m;
}

struct Dir {
    int32_t* page;      // pool page id
    int32_t* cnt;       // slots in use in the page (boundaries and holes)
    int32_t* nr;        // boundaries in the page (real slots)
    int64_t* maxv;      // max version in the page
    int64_t* start;     // global index of the page's first boundary (prefix of nr); start[D] = H
    uint64_t* fhi;      // first key of the page (copy, for the search)
    uint64_t* flo;
    uint32_t* fmeta;
    const uint8_t** ftail;
    int64_t* bmax;      // max of maxv over groups of 64 directory entries
    int64_t* bmax2;     // max of maxv over groups of 4096 entries (built by each batch's ingest)
    // search index: level l >= 1 holds fhi[i * 16^l]; levels start at
    // 16-entry (128-byte) boundaries, so a 16-wide probe window is one cache
    // line (hist_search.h).  Rebuilt by k_bmax_commit with the directory.
    uint64_t* sidx;
    // Long shared prefixes (config 4: tenant + path, 64 bytes): a search
    // window of 16 entries at level l (aligned, as the searches take them) is
    // only ever searched by keys between the window's first key and the next
    // window's first key, so query and window share their common prefix
    // (wsk, when > 17 bytes); then 8 bytes of each key from there (fpx for
    // level 0, spx beside sidx for levels >= 1) order them without the tails.
    // Rebuilt with the directory (k_dir_px); wsk 0: not used.
    uint64_t* fpx;
    uint64_t* spx;
    int32_t* wsk;
    int32_t cap;        // entries allocated (levels are sized from it)
};

constexpr int BMAX2_SPAN = 4096;  // directory entries per bmax2 word

constexpr int SIDX_B = 16;      // fan-out
constexpr int SIDX_LOG = 4;
constexpr int SIDX_LEVELS = 7;  // 16^7 > any directory

// offset of level l (1-based) in sidx; level 0 is fhi itself
__host__ __device__ inline int64_t sidx_off(int64_t cap, int l) {
    int64_t o = 0;
    for (int q = 1; q < l; q++) {
        const int64_t n = (cap + (1ll << (SIDX_LOG * q)) - 1) >> (SIDX_LOG * q);
        o += (n + SIDX_B - 1) & ~(int64_t)(SIDX_B - 1);
    }
    return o;
}

#ifndef FDBCS_DIR_PX  // (A/B: 0 leaves Dir::wsk at 0 -- the tails decide every tie)
#define FDBCS_DIR_PX 1
#endif
constexpr int PX_MIN_SKIP = 18;           // (a shorter common prefix: the fixed 17 bytes order the keys)
constexpr int PX_MAX_SKIP = 17 + 8 * 14;  // (the searches hold 16 tail words of the query)

// offset of level l (0-based) in Dir::wsk: one skip per 16-entry window
__host__ __device__ inline int64_t wsk_off(int64_t cap, int l) {
    int64_t o = 0;
    for (int q = 0; q < l; q++) {
        const int64_t n = (cap + (1ll << (SIDX_LOG * q)) - 1) >> (SIDX_LOG * q);
        o += (n + SIDX_B - 1) / SIDX_B;
    }
    return o;
}

// Common prefix length of two keys in bytes (at most the shorter length).
__device__ inline int key_lcp(const Key& a, const Key& b) {
    const int la = (int)key_len(a.meta), lb = (int)key_len(b.meta);
    const int m = la < lb ? la : lb;
    uint64_t x = a.hi ^ b.hi;
    if (x) return min(m, __clzll((long long)x) >> 3);
    x = a.lo ^ b.lo;
    if (x) return min(m, 8 + (__clzll((long long)x) >> 3));
    if ((a.meta >> 24) != (b.meta >> 24) || m <= 17) return min(m, 16);
    const uint64_t* ta = reinterpret_cast<const uint64_t*>(a.tail);
    const uint64_t* tb = reinterpret_cast<const uint64_t*>(b.tail);
    const int words = (m - 17 + 7) >> 3;
    // (four independent loads a step: a shared 64-byte prefix is six words,
    // one round trip each when the loop exits word by word)
    for (int w = 0; w < words; w += 4) {
        uint64_t d[4];
#pragma unroll
        for (int k = 0; k < 4; k++) d[k] = w + k < words ? ta[w + k] ^ tb[w + k] : 0;
#pragma unroll
        for (int k = 0; k < 4; k++)  // (little-endian words: the first byte is the lowest)
            if (d[k]) return min(m, 17 + 8 * (w + k) + (__ffsll((unsigned long long)d[k]) - 1) / 8);
    }
    return m;
}

// The 8 bytes of a key at byte s >= 17 (big-endian, zero past its end).
__device__ inline uint64_t key_bytes_at(const Key& k, int s) {
    const int len = (int)key_len(k.meta);
    if (s >= len) return 0;
    const int t = s - 17, w = t >> 3, sh = t & 7;
    const int words = (len - 17 + 7) >> 3;
    const uint64_t* tw = reinterpret_cast<const uint64_t*>(k.tail);
    const uint64_t x0 = __builtin_bswap64(tw[w]);
    const uint64_t x1 = w + 1 < words ? __builtin_bswap64(tw[w + 1]) : 0;
    return sh ? (x0 << (8 * sh)) | (x1 >> (64 - 8 * sh)) : x0;
}

// Device-resident scalars shared between the kernels of one batch.
struct Scalars {
    int32_t D;              // directory entries (current buffer)
    int32_t D_next;         // directory entries being built
    int32_t free_top;       // free page stack size
    int32_t err;            // nonzero: abort history mutation
    int32_t n_comb;         // combined write ranges
    int32_t n_aff;          // affected pages
    int32_t n_full;         // of them, pages the merge rewrites (not in place)
    int32_t n_dep;          // dependent transactions (intra-batch)
    int32_t edges_total;
    int64_t H;              // boundaries
    uint64_t tail_used;     // bytes used in the history tail arena
    uint64_t btail_used;    // bytes used in the batch tail buffer
    int64_t win_g0, win_g1; // compaction window [g0, g1) (global indices)
    int64_t last_ver;       // version of the last boundary (INT64_MIN: empty), set at each commit
    int64_t win_r0;         // first removable index (g0 + 1: the first scanned node stays)
    int64_t win_prev;       // version of the node before index 0 (sharded mode: the previous shard's last)
    int32_t win_pA, win_pB; // first / last directory entry covering the window
    int32_t win_newpages;   // pages produced by the repack
    int32_t win_surv;       // survivors in the window pages
    int32_t jac_iters;      // stats: Jacobi iterations in the decision
    int32_t blocks_done;    // last-block-commits counter (k_win_dir); zero between launches
    int32_t free_next;      // free_top after the rebuild in flight
    int32_t win_np;         // directory entries covered by the compaction window
    int32_t last_err;       // err of the last batch (err is reset for the next one)
    int32_t ss_resample;    // stats: a sort bucket overflowed and the batch was bucketed again
    int32_t ss_over[2];     // a sort bucket of job j overflowed its staging row (the guard re-buckets)
    int32_t ss_maxc;        // stats: largest sort bucket above the register path (0: none)
    int32_t extra_total;    // free pages the merge takes (parts beyond each page's first)
    int32_t n_comb_own;     // combined ranges whose begin lies in this shard (all of them unsharded)
    int32_t dec_wide;       // rounds mode: the candidate list overflowed (every read is a candidate)
    int32_t n_pot;          // rounds mode: entries in the candidate read list
    // fdbcs_sharded (SURVEY.md §8e protocol A, exchanges on the device)
    int32_t carry_dev;      // nonzero: the read check / merge take valueBefore-of-shard from carry_check / carry_apply
    int32_t sh_rk_owner;    // shard holding removalKey (-1: "")
    int64_t carry_check;    // after the previous merge (step 7)
    int64_t carry_apply;    // after the previous compaction (from exchange 1)
    // tail arena GC (kernels_hist.hip): the arena's two halves; new tails go to
    // half tail_half (tail_used bytes of it), the compaction window copies the
    // survivors' tails out of the other half, and a sweep that covered the
    // whole history frees it
    int32_t tail_half;
    int32_t tail_flags;     // TF_* below
    int32_t free_base;      // free-stack slot where the merge's freed pages go (free_top - extra_total before
                            // k_bmax_commit moves free_top: its blocks read this, not free_top)
    // load-metrics roll inside the per-transaction ingest (LmArgs below):
    // entries / key bytes appended this batch; at the end of the batch they
    // move to lm_out_* (what a synchronized host reads) and restart at 0
    int32_t lm_count;
    int32_t lm_out_count;
    uint64_t lm_bytes;
    uint64_t lm_out_bytes;
    // live ingest (kernels_batch.hip k_live_ingest): the host's progress as
    // the kernel's poller mirrors it, and the batch's final shape
    // (tagged with the live batch's generation, so nothing needs resetting
    // between batches: a word of an earlier batch reads as "nothing yet")
    // the live kernel's mirror of the host's progress, one word the workers
    // read in one load: lv_word(gen, state, transactions, stream bytes written whole)
    uint64_t lv_pub;
    int32_t lv_R, lv_W;     // the final read / write counts (diagnostics)
    int32_t lv_err;         // a transaction past the live capacities (the host falls back)
    // rounds mode, edge lanes fused into the decision launch (k_decide_rounds):
    // edge blocks done; block 0 waits for all of them, then zeroes it
    int32_t e_done;
    // large batches (k_page_join): reads whose end lies past their begin's page
    int32_t n_fall;
    // protocol B's edge exchange at a fixed capacity (k_sh_edges_cat_fixed):
    // the largest shard count when some shard's did not fit (0: they did)
    int32_t sh_need;
    int32_t sh_max;         // every batch: the largest shard count (the host's capacity decay)
    int32_t sh_pad;
    int32_t px_on;          // some key longer than 17 bytes was ingested or loaded (sticky): k_dir_px runs
    int32_t n_pxd[2];       // rewritten pages listed for k_page_px (pskip < 0), by launch parity
    int64_t ph[32];         // phase timestamps (wall_clock64 ticks) in FDBCS_PHASES builds
};
constexpr int32_t LV_RUNNING = 0, LV_FINAL = 1, LV_CANCEL = 2, LV_TIMEOUT = 3;
constexpr uint64_t LV_FINAL_BIT = 1ull << 63;  // in the host's published word (stage.h prog_[0])
// gen: 10 bits (another batch's word reads as "nothing yet"), state: 2,
// transactions: 20 (live batches have T <= LARGE_T), bytes: 32 (the live
// stream stays below 4 GB)
__host__ __device__ inline uint64_t lv_word(uint32_t gen, int state, uint64_t T, uint64_t used) {
    return (uint64_t)(gen & 0x3FF) << 54 | (uint64_t)(state & 3) << 52 | (T & 0xFFFFF) << 32 | (used & 0xFFFFFFFFull);
}
__host__ __device__ inline uint32_t lv_gen(uint64_t w) { return (uint32_t)(w >> 54); }
__host__ __device__ inline int lv_state(uint64_t w) { return (int)((w >> 52) & 3); }
__host__ __device__ inline int32_t lv_txns(uint64_t w) { return (int32_t)((w >> 32) & 0xFFFFF); }
__host__ __device__ inline uint64_t lv_used(uint64_t w) { return w & 0xFFFFFFFFull; }

// ---- Resolver load metrics (load_metrics.hip; Resolver.actor.cpp:146-151) ----
// The draw of position `pos` of batch `seq` of a sample (counter-based, every
// thread computes its own: DESIGN.md §6.3) and TransientStorageMetricSample::
// add's decision (StorageMetrics.actor.h:167-181): the amount added, 0 if not
// sampled.  oracle/load_sample.py restates both.
__host__ __device__ inline uint64_t roll_hash(uint64_t seed, uint64_t seq, uint64_t pos) {
    uint64_t z = seed + seq * 0xD1B54A32D192ED03ull + pos * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__host__ __device__ inline int64_t roll_amount(uint64_t h, int64_t metric, int64_t units) {
    if (metric <= 0) return 0;
    if (metric >= units) return metric;
    return (int64_t)(h % (uint64_t)units) < metric ? units : 0;
}

// The roll of an attached sample (fdbcs_sample_attach) done by the
// per-transaction ingest as it encodes each range: a sampled range appends an
// entry (amount, add-order position, begin length, byte offset) and its begin
// key's bytes straight into pinned host memory -- entries at Scalars::
// lm_count, bytes at lm_bytes in 16-byte-aligned pieces, every store 16
// bytes wide (each store over PCIe is a transaction of its own); past the
// capacities only the counters move.
struct alignas(16) LmEntry {
    int64_t amount;
    uint32_t pos, len;
    uint64_t off;
    uint64_t pad;
};
static_assert(sizeof(LmEntry) == 32, "load-metrics entry");
struct LmArgs {
    int32_t on;
    uint64_t seed, seq;
    int64_t units, offset_per_key;
    LmEntry* ent;
    uint8_t* bytes;  // 16-byte aligned
    uint32_t cap_n;
    uint64_t cap_b;
};

// Internal status of a sharded batch whose fixed-capacity edge exchange was
// short (k_sh_edges_cat_fixed): every history stage after it leaves the
// history as it was, and the host runs the batch's exchange onward again
// with a larger capacity (engine.hip sh_run).  Never returned to a caller.
constexpr int32_t E_SH_RETRY = -100;

constexpr int32_t TF_NOGC = 1;        // a survivor's tail could not be moved this sweep: no swap
constexpr int32_t TF_FROM_START = 2;  // this sweep's first window started at boundary 0
constexpr int32_t TF_WRAP = 4;        // this batch's window reached the end (removalKey -> "")

// bytes of one half of a tail arena of `cap` bytes
__host__ __device__ inline uint64_t tail_half_bytes(uint64_t cap) { return (cap / 2) & ~7ull; }

// Intra-kernel phase timestamps for profiling builds (-DFDBCS_PHASES): block 0
// thread 0 records the 100 MHz wall clock into Scalars::ph[i].
#ifdef FDBCS_PHASES
#define PHASE(sc, i)                                                                           \
    do {                                                                                       \
        if (threadIdx.x == 0 && blockIdx.x == 0) (sc)->ph[(i)] = (int64_t)wall_clock64();     \
    } while (0)
// per-wave cycle accumulators in ph[16..31] (cumulative across batches)
#define PACC(sc, i, v) atomicAdd((unsigned long long*)&(sc)->ph[(i)], (unsigned long long)(v))
#define PCLK() ((int64_t)clock64())
// ph[i] = max(ph[i], the wall clock) from any lane
#define PMAX(sc, i) atomicMax((unsigned long long*)&(sc)->ph[(i)], (unsigned long long)wall_clock64())
#define PSET(sc, i) ((sc)->ph[(i)] = (int64_t)wall_clock64())
#else
#define PMAX(sc, i) \
    do {            \
    } while (0)
#define PSET(sc, i) \
    do {            \
    } while (0)
#define PHASE(sc, i) \
    do {             \
    } while (0)
#define PACC(sc, i, v) \
    do {               \
    } while (0)
#define PCLK() ((int64_t)0)
#endif

__device__ inline int64_t atomic_max_i64(int64_t* addr, int64_t v) {
    return (int64_t)atomicMax((long long*)addr, (long long)v);
}

__device__ inline bool ShardBounds::below(const Key& k) const { return has_lo && kcmp(k, lo) < 0; }
__device__ inline bool ShardBounds::at_or_above(const Key& k) const { return has_hi && kcmp(k, hi) >= 0; }

}  // namespace fdbcs_dev
