// kernels.h -- launcher prototypes shared by the kernel TUs and the engine.
#pragma once
#include <hip/hip_runtime.h>
#include "common.h"
#include "../../include/fdbcs.h"

namespace fdbcs_dev {

// Merge-plan accumulators, indexed by directory entry.
// where write w's ends fall in the pre-batch history (write_search_group),
// one record per end: the merge plan reads the opening write's begin record and
// the closing write's end record of every combined range (k_plan_ranges), two
// random lines per range instead of one per field
struct alignas(16) WHitB {
    int32_t pb;   // directory entry of b
    int32_t ib;   // lower bound of b in its page
    int32_t cb;   // boundaries (real) in b's page
    int32_t rb;   // real boundaries before slot ib (holes, common.h)
};
struct alignas(16) WHitE {
    int64_t vb;   // version of the boundary before e (valueBefore(e))
    int32_t pe;   // directory entry of e
    int32_t ie;   // lower bound of e in its page
    int32_t re;   // real boundaries before slot ie
    int32_t feq;  // bit 0: e is a boundary; bit 1: valueBefore(e) is the header version
    int64_t pad;
};
static_assert(sizeof(WHitB) == 16 && sizeof(WHitE) == 32, "write hit records");
struct WriteHits {
    WHitB* b;
    WHitE* e;
};

struct PageAcc {
    int32_t* er;    // old boundaries erased
    int32_t* nn;    // new boundaries landing
    int32_t* jlo;   // first combined range touching the page
    int32_t* jhi;   // last one
    int32_t* diff;  // +1 / -1 marks of pages wholly inside a range
};

// Per-batch device working set (sized by the engine before each batch).
// ---- per-transaction staging (ConflictBatch::addTransaction, SkipList.cpp:979-1008) ----
// fdbcs_batch_add appends one record per transaction to a pinned byte stream:
// a StageHdr, then (nr + nw) StageRange entries (reads first, in call order),
// then the key bytes (begin, end of each range), padded to 8 bytes.  ro / wo
// are the reads / writes added before this transaction.
struct StageHdr {
    int64_t snap;
    int32_t ro, wo, nr, nw;
};
static_assert(sizeof(StageHdr) == 24, "stage record header");
// a range's keys: the begin key at `kofs` bytes from the record's start, the
// end key right after it (key lengths <= FDBCS_MAX_KEY < 2^15).  A point range
// [k, k\x00) -- the Resolver's usual read and write -- is stored as k and one
// 0 byte: the end key is then the same bytes one longer, at the begin's
// offset, marked by STAGE_SHARED in elen (16 of a 16-byte key's 33 bytes not
// written by the add nor sent over PCIe).
struct StageRange {
    uint32_t kofs;
    uint16_t blen, elen;
};
static_assert(sizeof(StageRange) == 8, "stage range entry");
constexpr uint16_t STAGE_SHARED = 0x8000;
static_assert(FDBCS_MAX_KEY < STAGE_SHARED, "the shared-end flag sits above every key length");
// A transaction with no ranges (always committed: tooOld needs a read,
// SkipList.cpp:985) has no record: its offset entry is STAGE_EMPTY | wo << 32
// | ro, the reads and writes added before it -- one 8-byte store per add.
// Protocol B shards see many (the transactions with no range on the shard).
constexpr uint64_t STAGE_EMPTY = 1ull << 63;
struct StageTxn {
    int64_t snap;
    int32_t ro, wo, nr, nw;
    uint64_t base;  // record offset (nr + nw > 0)
};
__host__ __device__ inline StageTxn stage_txn(const uint8_t* stream, uint64_t toff) {
    if (toff & STAGE_EMPTY)
        return StageTxn{0, (int32_t)(uint32_t)toff, (int32_t)((toff >> 32) & 0x7fffffffu), 0, 0, 0};
    const StageHdr h = *reinterpret_cast<const StageHdr*>(stream + toff);  // (records are 8-byte aligned)
    return StageTxn{h.snap, h.ro, h.wo, h.nr, h.nw, toff};
}
// (end offset from the record, end length) of a StageRange
__host__ __device__ inline uint32_t stage_end_ofs(const StageRange& e) {
    return e.kofs + ((e.elen & STAGE_SHARED) ? 0u : (uint32_t)e.blen);
}
__host__ __device__ inline uint32_t stage_end_len(const StageRange& e) { return e.elen & (STAGE_SHARED - 1); }
// k_unpack: one lane per transaction turns the stream (device copy) into the
// arrays of a fdbcs_batch_view (layout below, key_bytes = the stream itself)
struct UnpackOut {
    int64_t* snap;     // [T]
    int32_t* ro;       // [T+1]
    int32_t* wo;       // [T+1]
    uint64_t* koff;    // [2R+2W]
    uint32_t* klen;    // [2R+2W]
};
void launch_unpack(const uint8_t* stream, const uint64_t* toff, int T, int R, int W, UnpackOut o, hipStream_t s);
// bytes from host-mapped memory (a device pointer to it) into dst, on s
void launch_pull(const uint8_t* host_src, uint8_t* dst, uint64_t bytes, hipStream_t s);
// the staged batch the next launch_ingest reads straight from the record
// stream (one launch for k_unpack's work and the ingest's; stream == null:
// the ingest reads a batch view)
struct StagedBatch {
    const uint8_t* stream = nullptr;  // device copy of the record stream
    const uint64_t* toff = nullptr;   // [T] record offsets (device)
    UnpackOut view{};                 // the batch view's arrays, written on the way
    // live ingest (stage.h): k_live_ingest already encoded the batch from the
    // host-mapped stream while the adds ran; run_batch launches no ingest
    bool live = false;
    // a live batch that outgrew its capacities: its partial work is undone
    // (launch_live_reset) before the ingest of the whole stream
    bool live_failed = false;
};

// Live ingest: the shape a live batch may reach, fixed
// when the batch begins (the buffers are sized for it; a batch past it falls
// back to the ingest at detectConflicts).
struct LiveCaps {
    int32_t T, R, W;
    uint64_t key_bytes;
};
// Live kernel shape, read from the environment when the conflict set is made
// (tests run every shape; the defaults are the measured best):
// FDBCS_LIVE_BLOCKS workgroups (128), FDBCS_LIVE_SPEC the speculative record
// window of the last groups (1), FDBCS_LIVE_TIMEOUT_US the poller's limit
// (8 s; the batch then falls back to the whole-stream ingest, stage.h).
struct LiveTune {
    int blocks = 128;
    bool spec = true;
    uint64_t timeout_ticks = 8ull * 100000000ull;  // (100 MHz wall clock)
};

struct BatchBufs {
    StagedBatch staged;  // per-transaction path: set for one run_batch (stage.h)
    // transaction level [T]
    uint8_t* too_old;
    uint8_t* hist;
    uint8_t* committed;
    int32_t* deg;        // unique intra-batch sources per reader
    int32_t* off;        // [T+1] exclusive scan of deg
    int32_t* cur;        // fill cursors
    int32_t* dep_list;   // dependents in index order
    int32_t* dep_idx;    // t -> index in dep_list or -1
    uint64_t* cbits;     // [T / 64 + 1] committed bits (grid decision)
    // range level
    int32_t* read_txn;   // [R]
    int64_t* read_snap;  // [R] snapshot of the read's transaction (INT64_MAX: too old)
    int32_t* write_txn;  // [W]
    // encoded keys [2R+2W]
    KeyArrays keys;
    uint8_t* btail;      // tail bytes of batch keys (8-aligned)
    uint64_t btail_cap;
    // sort records
    SRec* rec_r0;        // [R]   read begins, sorted
    SRec* rec_w0;        // [2W]  write endpoints, sorted
    SRec* sr;            // sorted read begins
    SRec* sw;            // sorted write endpoints
    uint32_t* sw_slot;   // [2W]  their slots (compact copy for the combine)
    // sample sort scratch
    int32_t* ss_cnt;     // [2 parities][3 * 1024] bucket counts of both jobs, then job 1's cover deltas;
                         // a batch zeroes the next batch's
    SRec* ss_q;          // [2 * 1024] quantiles of the previous batch's sorted output
    uint8_t* ss_qt;      // [2 * 1024 * SS_QT] their tail bytes (the batch keys they came from are gone)
    int32_t* ss_bkt;     // [R + 2W] bucket of each record
    SRec* ss_tmp;        // bucket staging rows (large batches: merge-sort scratch)
    int32_t* lb_meta;    // large-batch bucketed sort: offsets, passes, per-pass chunk prefixes
    int32_t* lb_hist;    // [2 * lb_hist_cap] per-block bucket counts and their scan
    int64_t lb_hist_cap;
    int64_t ss_tmp_cap;
    bool large;          // large-batch mode (large_batch_mode): merge sort, overlap edges
    bool dir_join;       // directory entries of the sorted keys by merge-join (large batches; long keys over a
                         // small directory, engine.hip edges_read_check)
    bool rounds;         // the decision by rounds (k_decide_rounds, rounds_fit): no overlap pairs
    bool rc_fused;       // this batch's history read check ran in the sort's bucket launch
    // live ingest: the slot of write 0's begin (0: 2R, the view's own
    // layout).  k_live_ingest does not know R before the final word, so a live
    // batch's writes sit at 2 caps.R + 2w -- a gap after the reads that every
    // stage addresses through write_base() -- and job 1's bucket count is the
    // one its scatter used (the capacities' 2W, lv_nb1)
    int64_t lv_wbase;
    int32_t lv_nb1;
    // rounds mode (kernels_batch.hip k_decide_rounds)
    int32_t* rq;         // [2R] sorted write endpoints <= each read's begin / < its end
    int32_t* plist;      // [R + W] candidate reads: some write of the batch may overlap them (duplicates)
    uint8_t* wnew;       // [2W + 64] sorted write endpoint p starts a new distinct key
    int32_t* winv;       // [2W] sorted position of each write endpoint (by slot - write_base)
    int32_t* wcov;       // [2W] write cover: begins minus ends among the sorted write endpoints up to each
    uint2* items;        // [R + W] the rounds' writes and reads when they do not fit in LDS
    int64_t list_cap;    // entries of plist (items: 2 * list_cap)
    bool ws_deferred;    // this batch's write searches wait for launch_write_search
    bool edges_fused;    // rounds mode: the edge lanes wait for launch_decide (blocks of the decision launch)
    uint64_t* ss_gsamp;  // [2 * 3 * 4096] global sample scratch of the sort's overflow guard
    uint32_t* rstamp;    // [R] per read: the batch (rseq) that put it on plist
    uint32_t rseq;
    // overlap edges (large / sparse batches)
    int32_t* et;         // [edge_cap] reader of each overlap pair
    int32_t* eu;         // [edge_cap] earlier writer
    int32_t* csr;        // [edge_cap] sources bucketed by reader
    int32_t* comb_blk;   // [2 * (combine blocks + 1)] multi-block combine: per-block sums, opens
    int32_t* dec_blk;    // [2 * (T / 256 + 2)] grid decision: dependents and their sources per block
    int64_t edge_cap;
    // combined write ranges [W], as positions of their begin / end among the
    // sorted write endpoints (sw: the records hold the keys, in key order)
    int32_t* cb_pos;
    int32_t* ce_pos;
    KeyArrays rkb, rke;  // [W] their keys, compact (written by k_plan_ranges)
    // where each write's begin / end fall in the pre-batch history [W]
    // (searched speculatively beside the read check, before the decision)
    WriteHits wh;
    // insertion plan [W]
    int32_t* pb; int32_t* ib; int32_t* pe; int32_t* ie;
    uint8_t* need_e;
    int64_t* vb;
    // per-directory-entry accumulators of the merge plan [cap_dir + 2]; zero
    // (jlo INT32_MAX, jhi -1) between batches -- k_plan_scan resets them
    PageAcc acc;
    int64_t* blk_agg;    // [plan blocks * 6] per-block plan aggregates (2 start states x 3 packed words)
    int32_t* blk_diff;   // [plan blocks]
    // affected pages, compacted [cap_dir + 2]
    int32_t* aff_list;   // directory entry
    int32_t* aff_jlo; int32_t* aff_jhi;  // combined ranges touching it
    int32_t* aff_nn;     // new entries landing
    int32_t* aff_parts;  // output pages
    int32_t* aff_nn_off; int32_t* aff_parts_off; int32_t* aff_extra_off; int32_t* aff_free_off;
    int64_t* aff_start;  // start[] of its first output page
    int32_t* aff_page;   // its pool page and boundary count
    int32_t* aff_cnt;
    int32_t* freed_list; // pages the merge frees, pushed after its pops
    int32_t* full_list;  // affected pages the merge rewrites (not in place)
    // large batches (k_page_join): the reads whose end lies past their
    // begin's page [R + 2W + 64]
    int32_t* pj_fall;
    int64_t pj_cap;
    // new-entry scratch [2W]
    Pool ne;             // key + version of new entries in page order
    int32_t* ne_ins;     // insertion index in the old page
    // page descriptors produced by rebuilds [cap]
    int32_t* desc_page; int32_t* desc_cnt; int32_t* desc_nr; int64_t* desc_max;
    uint64_t* desc_fhi; uint64_t* desc_flo; uint32_t* desc_fmeta; const uint8_t** desc_ftail;
    // compaction window
    uint8_t* win_keep;   // [window pages * PAGE]
    int32_t* win_cnt;    // survivors per window page
    int32_t* win_off;    // [win_cap_pages + 1]
    int32_t win_cap_pages;
    // scan scratch
    int64_t* scan_tmp;   // [>= 1024]
    // verdict
    uint8_t* verdict;
};

// the slot of write 0's begin in this batch's key arrays (BatchBufs::lv_wbase)
inline int64_t write_base(const BatchBufs& b, const fdbcs_batch_view& v) {
    return b.lv_wbase ? b.lv_wbase : 2 * (int64_t)v.read_count;
}

struct HistBufs {
    Pool pool;
    int32_t cap_pages;
    int32_t* free_stack;
    int32_t* px_list;  // [cap_pages] directory entries of rewritten pages (k_dir_px -> k_page_px)
    int px_par = 0;    // which Scalars::n_pxd counts the next list
    Dir dir[2];
    int32_t cap_dir;
    uint8_t* tail_arena;
    uint64_t tail_cap;
    // removal key (device copy)
    uint64_t* rk_hi; uint64_t* rk_lo; uint32_t* rk_meta; uint8_t* rk_tail;  // rk_tail: 30008 bytes
    // exact sharded mode: this engine's key range (unbounded by default)
    ShardBounds shard;
    uint8_t* shard_tails;  // device copies of the bounds' tails [2][SHARD_TAIL_STRIDE]
    // host-mapped copy of the scalars, written by the kernel that ends a batch
    // (the host reads it after a stream sync instead of issuing a copy)
    Scalars* mirror;
    const volatile Scalars* mirror_host;  // (the same memory, host address)
    // the host has seen Scalars::px_on (sticky): from then on every directory
    // gets its prefix skips rebuilt (k_dir_px); before, none was ever built
    bool px_host = false;
};

// ---- scans (scan.hip) ----
// Exclusive scan of n (device-resident count *n_ptr, or n_host if n_ptr null)
// int32 values; out[n] = total.  Optional *total_out.
void scan_i32(const int32_t* in, int32_t* out, const int32_t* n_ptr, int32_t n_host, int32_t* total_out,
              int64_t* tmp, hipStream_t s);
void scan_i64_from_i32(const int32_t* in, int64_t* out, const int32_t* n_ptr, int32_t n_host, int64_t* total_out,
                       int64_t* tmp, hipStream_t s);

// ---- batch stages (kernels_batch.hip) ----
// scatter: the sort splitters exist (an earlier batch) -- the ingest puts
// the sort records into their buckets itself (launch_sort_ranges(scattered))
// hd: the directory the batch's read check will search (its bmax2 level is
// built here, from the maxima the last history update left)
// Live ingest (kernels_batch.hip).  launch_live_ingest: the persistent kernel
// that encodes the per-transaction stream from host-mapped memory as the
// host publishes it (prog: host-mapped progress words, stage.h), launched
// when the batch begins; parity: the sort counters' (cs->sorts & 1).
// After the host's final word nothing is left to place: the writes and
// their sort records are at write_base (BatchBufs::lv_wbase), the per-batch
// resets ran in the kernel's prologue.  launch_live_reset: undo a failed live batch's partial work
// before the whole stream is ingested again.
// gen: the live batch's generation (tags the progress words in Scalars)
void launch_live_ingest(BatchBufs& b, Scalars* sc, const LiveCaps& caps, int64_t oldest, int parity,
                        const uint8_t* stream, uint64_t stream_cap, const uint64_t* toff, const uint64_t* prog,
                        UnpackOut view, const LmArgs* lm, uint32_t gen, const Dir& hd, const LiveTune& tune,
                        hipStream_t s);
void launch_live_reset(BatchBufs& b, Scalars* sc, int parity, hipStream_t s);
// lm: an attached sample's load-metrics roll (staged batches only; null: none)
void launch_ingest(const fdbcs_batch_view& v, int64_t oldest, BatchBufs& b, Scalars* sc, bool scatter, int parity,
                   const Dir& hd, hipStream_t s, bool sharded = false, const LmArgs* lm = nullptr);

// h (optional): the history the batch's read check searches -- the check of
// every read then runs in the sort's bucket launch (b.rc_fused), and the next
// launch_edges_read_check leaves it out; v0: as launch_edges_read_check's
// guard false: no k_ss_guard launch after a scattering ingest (run_batch's
// adaptive policy, SORT_GUARD_MAXC); an overflowed bucket is then ranked by
// the bucket kernel's global path, and the next batch's splitters come from
// this batch's sorted output
bool launch_sort_ranges(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, bool sample, int parity,
                        bool scattered, hipStream_t s, HistBufs* h = nullptr, int cur = 0, int64_t v0 = 0,
                        bool guard = true);
// run_batch launches the sort's overflow guard only when the last finished
// batch's largest bucket (Scalars::ss_maxc) reached this, or it was bucketed
// twice (half of a bucket's 512-record staging row)
constexpr int SORT_GUARD_MAXC = 256;
int64_t sort_staging_records(int R, int W, bool large);
// Large-batch mode (T > LARGE_T, or forced by FDBCS_TEST_LARGE_BATCH for tests):
// the endpoint sort is a merge sort (no per-batch splitter balance limits)
// and the decision walks the overlap edges on the grid (k_dec_*) instead of
// one workgroup's rounds (k_decide_rounds).  Up to MAX_T transactions.
constexpr int64_t LARGE_T = 65536;
constexpr int64_t MAX_T = 1310720;  // k_dec_walk keeps a committed bit per txn in LDS (160 KiB)
bool large_batch_mode(int64_t T);
int64_t lb_meta_words();
int64_t lb_hist_words(int R, int W);
// history read check + intra-batch overlap edges, one launch
// defer_ws: leave the write searches (WriteHits, for the merge) to
// launch_write_search, after the verdicts
void launch_edges_read_check(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t v0,
                             hipStream_t s, bool defer_ws = false);
void launch_write_search(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t v0,
                         hipStream_t s);
// Host-mapped verdict output of the decision (early verdicts): the verdicts,
// a system-scope fence, then one 16-byte store {seq, sc->err, sc->last_err, 0}
// at flag (16-byte aligned).
struct EarlyOut {
    uint8_t* verdict;
    uint32_t* flag;
    uint32_t seq;
};
// split: the combine is left to launch_combine (issued after the verdicts).
// eo: write the verdicts there (returns true if this batch's decision does;
// the grid decision of large batches does not).
// h (single-workgroup decision, write searches deferred by the read check):
// the write searches run as extra blocks of the decision's launch
bool launch_decide(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, uint8_t* verdict, hipStream_t s,
                   bool split = false, const EarlyOut* eo = nullptr, HistBufs* h = nullptr, int cur = 0,
                   int64_t v0 = 0);
// k_decide_rounds keeps its state in LDS: batches up to this shape
bool rounds_fit(int64_t T, int64_t W);
void launch_combine(const fdbcs_batch_view& v, BatchBufs& b, Scalars* sc, hipStream_t s);
// exact sharded mode: per-transaction exchange flags (0 / 1 history conflict /
// 2 tooOld) out of and back into the batch state; a foreign edge list in
void launch_flags_out(const BatchBufs& b, int T, uint8_t* flags, hipStream_t s);
void launch_flags_in(BatchBufs& b, int T, const uint8_t* flags, hipStream_t s);
void launch_set_edges(BatchBufs& b, Scalars* sc, int T, const int32_t* et, const int32_t* eu, int64_t n,
                      hipStream_t s);
void configure_batch_kernels();

// ---- history stages (kernels_hist.hip) ----
int plan_blocks(int cap_dir);
void launch_merge(const fdbcs_batch_view& v, BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t now,
                  int64_t v0, bool end_of_batch, hipStream_t s);
// sharded mode: this shard's part of the global compaction window (local indices)
struct WinExplicit {
    int64_t a, b;
    int keep_first;
    int64_t prev;
};
void launch_compact(BatchBufs& b, HistBufs& h, int cur, Scalars* sc, int64_t oldest, hipStream_t s,
                    const WinExplicit* win = nullptr);
void launch_key_at(HistBufs& h, int cur, Scalars* sc, int64_t g, uint64_t* out, uint8_t* out_tail, hipStream_t s);
void launch_dir_finish(HistBufs& h, int cur, Scalars* sc, BatchBufs& b, hipStream_t s);
void launch_sidx_build(HistBufs& h, int which, Scalars* sc, hipStream_t s);
void launch_reset_history(HistBufs& h, int cur, Scalars* sc, hipStream_t s);
void launch_gather(HistBufs& h, int cur, Scalars* sc, Pool out, hipStream_t s);
void launch_push_free(HistBufs& h, int32_t from_top, int32_t first_id, int32_t count, hipStream_t s);
void launch_relocate_tails(HistBufs& h, const uint8_t* old_base, uint64_t old_cap, const uint8_t* new_base,
                           uint64_t new_cap, hipStream_t s);

// fdbcs_sharded: the protocol's exchange-side steps on the device (kernels_hist.hip)
constexpr int SH_WORDS = 4;  // int64 words per shard in exchange 1 (slots) and 2 (infos)
void launch_sh_init(Scalars* sc, int64_t v0, bool reset_owner, hipStream_t s);
void launch_sh_slot_out(const Scalars* sc, int64_t* slots, int rank, int G, hipStream_t s);
void launch_sh_carry(Scalars* sc, const int64_t* slots, int rank, int64_t v0, hipStream_t s);
void launch_sh_info_out(const Scalars* sc, int64_t* send, int rank, bool bounded, hipStream_t s);
void launch_sh_plan(HistBufs& h, int cur, Scalars* sc, const int64_t* infos, int rank, int G, int64_t v0, bool compact,
                    hipStream_t s);
// bytes per shard-bound tail copy: a multiple of 8, since tails are read a
// word at a time (tail_cmp) and a misaligned word load returns the aligned
// word's bytes (a 30,017-byte stride put the upper bound's tail off by one
// byte and made every compare against a bound longer than 17 bytes wrong)
constexpr size_t SHARD_TAIL_STRIDE = ((size_t)FDBCS_MAX_KEY + 16 + 7) & ~(size_t)7;
// the HIP device an engine lives on (engine.hip)
int engine_device(const fdbcs* cs);
// The load-metrics roll inside the per-transaction ingest (common.h LmArgs).
// engine_lm_attach: the sample `owner` (its draw counter at *seq, read at each
// detect) rolls with every staged batch of cs from now on (owner null: none).
// engine_lm_take: the last detected batch's entries, if it was rolled for
// (owner, seq, offset_per_key) and no batch ran since.  sample_unlink
// (load_metrics.hip): cs is being destroyed, its attached sample forgets it.
struct LmTake {
    int64_t count;
    const LmEntry* ent;
    const uint8_t* bytes;
    size_t cap_n, cap_b;
};
void engine_lm_attach(fdbcs* cs, const void* owner, const uint64_t* seq, uint64_t seed, int64_t units,
                      int64_t offset_per_key);
bool engine_lm_take(fdbcs* cs, const void* owner, uint64_t seq, int64_t offset_per_key, LmTake& out);
void sample_unlink(const void* owner, const fdbcs* cs);
// protocol B's edge exchange (kernels_hist.hip)
void launch_sh_edges_count(const Scalars* sc, int64_t* slots, int rank, int G, int64_t edge_cap, hipStream_t s);
void launch_sh_edges_pack(const BatchBufs& b, const Scalars* sc, int64_t M, int32_t* send, hipStream_t s);
void launch_sh_edges_cat_fixed(const int32_t* recv, const int64_t* slots, int G, int64_t M, int32_t* cat_et,
                               int32_t* cat_eu, Scalars* sc, hipStream_t s);

// fdbcs_nth_after (kernels_hist.hip): query keys (encoded; tails 8-byte
// aligned, zero padded, in device memory) -> out[3q] = hi, lo, meta (~0: past
// the end) and the tail words at out_tail + q * tail_stride
struct NthArgs {
    Pool pool;
    Dir dir;
    const Scalars* sc;
    int n;
    const uint64_t* qhi;
    const uint64_t* qlo;
    const uint32_t* qmeta;
    const uint8_t* const* qtail;
    const int64_t* steps;
    uint64_t* out;
    uint8_t* out_tail;
    uint32_t tail_stride;
};
void launch_nth_after(HistBufs& h, int cur, const Scalars* sc, const NthArgs& a, hipStream_t s);

}  // namespace fdbcs_dev
