// engine.hip -- host orchestration and the C ABI (include/fdbcs.h).
//
// One fdbcs object = one ConflictSet (fdbserver/SkipList.cpp:926-954) whose
// history lives in HBM.  ConflictBatch calls (ConflictSet.h:32-60) are staged
// in host memory, shipped with one H2D copy, resolved by the kernel pipeline
// below on the set's HIP stream, and the verdicts come back with one D2H copy.
// Pipeline order follows ConflictBatch::detectConflicts (SkipList.cpp:
// 1163-1208): read check -> intra-batch -> combine -> merge -> verdicts ->
// compaction.
#include <hip/hip_runtime.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "kernels.h"
#include "stage.h"

using namespace fdbcs_dev;

namespace {

static inline int64_t cdiv64(int64_t a, int64_t b) { return (a + b - 1) / b; }
// where the scalar snapshot of an early verdict sits in the verdict staging
static inline size_t vpin_scalars_off(int64_t T) { return ((size_t)T + 63) & ~(size_t)63; }

#define HIPOK(x)                                    \
    do {                                            \
        hipError_t e_ = (x);                        \
        if (e_ != hipSuccess) {                     \
            last_hip_error() = e_;                  \
            return FDBCS_E_HIP;                     \
        }                                           \
    } while (0)

hipError_t& last_hip_error() {
    static thread_local hipError_t e = hipSuccess;
    return e;
}

template <typename T>
int dalloc(T*& p, int64_t n) {
    p = nullptr;
    if (n <= 0) n = 1;
    void* q = nullptr;
    hipError_t e = hipMalloc(&q, (size_t)n * sizeof(T));
    if (e != hipSuccess) {
        last_hip_error() = e;
        return FDBCS_E_NOMEM;
    }
    // (FDBCS_POISON=<byte>, debugging: fresh device memory holds that pattern,
    // so a kernel that reads a buffer before anything wrote it misbehaves the
    // same way on every run instead of on whatever a freed buffer left)
    static const int poison = getenv("FDBCS_POISON") ? (int)strtol(getenv("FDBCS_POISON"), nullptr, 0) : -1;
    if (poison >= 0) {  // (the null stream does not order the engine's non-blocking streams: wait for it)
        hipMemset(q, poison & 0xFF, (size_t)n * sizeof(T));
        hipDeviceSynchronize();
    }
    p = static_cast<T*>(q);
    return FDBCS_OK;
}

template <typename T>
void dfree(T*& p) {
    if (p) {
        hipDeviceSynchronize();  // (growth only: a pipelined batch may still be using the buffer)
        hipFree((void*)p);
    }
    p = nullptr;
}

// host-side key encoding identical to k_encode
void encode_host(const uint8_t* p, uint32_t L, uint64_t& hi, uint64_t& lo, uint32_t& meta) {
    hi = lo = 0;
    uint32_t b16 = 0;
    for (uint32_t i = 0; i < std::min<uint32_t>(L, 17); i++) {
        uint64_t c = p[i];
        if (i < 8) hi |= c << (56 - 8 * i);
        else if (i < 16) lo |= c << (56 - 8 * (i - 8));
        else b16 = (uint32_t)c;
    }
    meta = (b16 << 24) | L;
}

// ~35,000 ranges per config-2 batch are checked on the host: inline word
// compares instead of a libc call per key.
inline uint64_t ld64(const uint8_t* p) {
    uint64_t x;
    memcpy(&x, p, 8);
    return x;
}

// keycmp (SkipList.cpp:113-120 order) eight bytes at a time
int keycmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t n = std::min(al, bl);
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint64_t x = ld64(a + i), y = ld64(b + i);
        if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y) ? -1 : 1;
    }
    for (; i < n; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}


}  // namespace

struct fdbcs {
    int device = 0;
    hipStream_t stream = nullptr;
    HistBufs h{};
    BatchBufs b{};
    Scalars* sc = nullptr;       // device
    Scalars* sc_host = nullptr;  // pinned mirror
    Scalars* sc_mapped = nullptr;  // host-mapped copies the batch-ending kernels write (HistBufs::mirror): two
                                   // slots, by run_batch parity (mirror_batch), so the one an earlier batch
                                   // published stays readable while the next batch's update runs
    Scalars* mirror_dev = nullptr;  // (their device address)
    int cur = 0;
    int64_t v0 = 0;
    int64_t oldest = 0;
    // capacities of the per-batch buffers
    int64_t capT = -1, capR = -1, capW = -1, capSlots = -1, capBtail = -1, capEdges = -1, capRowWords = -1;
    int64_t capDirB = -1, capWinPages = -1, capDesc = -1, capSortRec = -1;
    // last known device state (valid after a synchronized batch)
    int64_t known_D = 1, known_free = 0, known_H = 0;
    uint64_t known_tail = 0;
    int64_t pending_pages = 0;   // worst-case pages consumed by unsynchronized batches
    uint64_t pending_tail = 0;
    // host staging of ConflictBatch::addTransaction (SkipList.cpp:979-1008):
    // stage.h (pinned record stream, chunked H2D, k_unpack at detect)
    bool in_batch = false;
    TxnStage st;
    uint64_t stage_key_total = 0;  // the staged batch's key bytes while it runs (TxnStage::key_total)
    // pinned host staging + device input staging
    uint8_t* pin = nullptr;
    size_t pin_cap = 0;
    uint8_t* din = nullptr;
    size_t din_cap = 0;
    uint8_t* vpin = nullptr;  // verdict pinned
    size_t vpin_cap = 0;
    // stage timing
    bool timing = false;
    int32_t borrow_flags = 0;  // fdbcs_config.flags (FDBCS_BORROW_*)
    hipEvent_t ev[8] = {};
    // early verdicts: D2H of the verdicts and a scalar snapshot right after
    // the decision; the history update keeps running behind them
    hipEvent_t ev_verdict = nullptr;
    bool vev_rec = true;  // ev_verdict was recorded for the batch in flight (else its fallback is ev_end)
    // host-mapped verdict area the decision kernel writes (kernels.h EarlyOut):
    // [0] flag, [4] err, [8] last_err, verdicts from byte 64
    uint8_t* vmap = nullptr;
    uint8_t* vmap_dev = nullptr;
    size_t vmap_cap = 0;
    uint32_t vseq = 0;
    bool early_mapped = false;  // the batch in flight writes vmap

    // exact sharded mode: scratch for a key read back at a local index
    uint64_t* key_out = nullptr;     // hi, lo, meta
    uint8_t* key_out_tail = nullptr;
    uint8_t* rk_stage = nullptr;     // pinned: removalKey in (hi, lo, meta, tail) form, both directions
    double stage_us[7] = {0};
    bool have_times = false;
    // device view of the last batch staged by a host path (fdbcs_last_device_batch)
    fdbcs_batch_view last_dv{};
    bool have_last_dv = false;
    int64_t last_wbase = 0;  // a live batch's writes in last_dv sit from here (0: 2R); moved on export
    bool have_quantiles = false;  // sample-sort splitters from an earlier batch exist
    bool sparse_edges = false;    // exact sharded protocol B: this shard exports its overlap edges
    bool edges_known = false;     // sc_host->edges_total is this batch's (set by fdbcs_shard_check)
    int64_t last_T = 0, last_R = 0, last_W = 0;  // shape of the last batch (stats)
    int64_t sorts = 0;                           // sorts launched (sort-counter parity)
    // pipelined host batches (fdbcs_batch_submit_packed / fdbcs_batch_wait): two
    // staging slots, so batch k+1's host packing and H2D copy (copy stream)
    // overlap batch k's kernels
    struct Slot {
        uint8_t* pin = nullptr;
        size_t pin_cap = 0;
        uint8_t* din = nullptr;
        size_t din_cap = 0;
        uint8_t* vpin = nullptr;
        size_t vpin_cap = 0;
        uint8_t* dverd = nullptr;
        int64_t dverd_cap = 0;
        hipEvent_t copied = nullptr, done = nullptr;
        int64_t T = 0;
        const volatile Scalars* mirror = nullptr;  // the mirror slot its run_batch published into
    } slot[2];
    hipStream_t copy_stream = nullptr;
    // end of the last run_batch's history update (its scalars are then in the
    // host-mapped mirror: ensure_history refreshes its budget without a sync)
    hipEvent_t ev_end = nullptr;  // (= ev_slot[] of the last run_batch's mirror slot)
    bool end_mirror = false;
    // the two mirror slots: the run_batch that published into each (batches;
    // ~0: none) and the end event recorded behind it; last_need_*: the
    // budget the latest run_batch reserved
    hipEvent_t ev_slot[2] = {nullptr, nullptr};
    uint64_t mirror_batch[2] = {~0ull, ~0ull};
    int64_t last_need_pages = 0;
    uint64_t last_need_tail = 0;
    int64_t sub_head = 0, sub_tail = 0;  // batches submitted / waited for
    // The Resolver's load-metrics roll (iopsSample, Resolver.actor.cpp:146-151)
    // of an attached sample (fdbcs_sample_attach), done by the per-transaction
    // ingest while it encodes the ranges; the entries land in pinned host
    // memory and their count arrives with the verdicts, so
    // fdbcs_sample_add_batch needs no launch and no wait (load_metrics.hip).
    struct Lm {
        const void* owner = nullptr;    // the attached fdbcs_sample
        const uint64_t* seq = nullptr;  // its draw counter (read at each detect)
        uint64_t seed = 0;
        int64_t units = 0, opk = 0;
        LmEntry* ent = nullptr;  // pinned: the sampled entries
        uint8_t* bytes = nullptr;  // pinned: their begin keys (16-byte pieces)
        size_t cap_n = 0, cap_b = 0;
        bool armed = false;       // this batch's ingest rolls
        bool rolled = false;      // the last detected batch was rolled ...
        uint64_t rolled_seq = 0;  // ... with this draw counter
        int64_t count = 0;        // ... into this many entries
        uint64_t batch = 0;       // ... and it was batch number `batch`
        // ... on the host instead (a protocol-B shard's adds, fdbcs_sharded:
        // lm_ent / lm_bytes): the entries' home; null: the pinned buffers above
        const LmEntry* host_ent = nullptr;
        const uint8_t* host_bytes = nullptr;
        size_t host_nb = 0;
    } lm;
    uint64_t batches = 0;  // batches run (run_batch / sh_run)
    // live ingest (k_live_ingest)
    uint32_t lv_gen = 0;   // generation of the last live batch
    bool lv_lm = false;    // the live kernel rolls for the attached sample
    int64_t lv_prev_T = 0, lv_prev_R = 0, lv_prev_W = 0;  // shape of the last per-transaction batch
    uint64_t lv_prev_K = 0;
    int64_t lv_done = 0, lv_cancelled = 0;  // batches ingested live / cancelled on the way (stats)
    LiveTune lv_tune;      // the live kernel's shape (FDBCS_LIVE_BLOCKS / _SPEC / _TIMEOUT_US)
    uint64_t lv_kb = 0;    // the key bytes the open live batch's buffers were sized for (live_begin)
};

namespace {

int alloc_pool(fdbcs* cs, int32_t pages) {
    HistBufs& h = cs->h;
    int r;
    h.cap_pages = pages;
    const int64_t slots = (int64_t)pages * PAGE;
    if ((r = dalloc(h.pool.hi, slots)) || (r = dalloc(h.pool.lo, slots)) || (r = dalloc(h.pool.meta, slots)) ||
        (r = dalloc(h.pool.ver, slots)) || (r = dalloc(h.pool.tail, slots)) || (r = dalloc(h.pool.pidx, slots / PIDX_STRIDE)) ||
        (r = dalloc(h.pool.hmask, (int64_t)pages * HM_WORDS)) || (r = dalloc(h.free_stack, pages)) ||
        (r = dalloc(h.pool.px, slots)) || (r = dalloc(h.pool.pxidx, slots / PIDX_STRIDE)) ||
        (r = dalloc(h.pool.pskip, pages)) || (r = dalloc(h.px_list, (int64_t)pages + 1)))
        return r;
    // (on the engine's non-blocking stream: a null-stream memset is not
    // ordered against grow_pool's copies and k_dir_px / k_page_px behind it)
    HIPOK(hipMemsetAsync(h.pool.pskip, 0, (size_t)pages * sizeof(int32_t), cs->stream));
    h.cap_dir = pages + 1;
    for (int d = 0; d < 2; d++) {
        Dir& x = h.dir[d];
        if ((r = dalloc(x.page, h.cap_dir)) || (r = dalloc(x.cnt, h.cap_dir)) || (r = dalloc(x.nr, h.cap_dir)) ||
            (r = dalloc(x.maxv, h.cap_dir)) ||
            (r = dalloc(x.start, h.cap_dir + 1)) || (r = dalloc(x.fhi, h.cap_dir)) || (r = dalloc(x.flo, h.cap_dir)) ||
            (r = dalloc(x.fmeta, h.cap_dir)) || (r = dalloc(x.ftail, h.cap_dir)) ||
            (r = dalloc(x.bmax, h.cap_dir / 64 + 2)) || (r = dalloc(x.bmax2, h.cap_dir / BMAX2_SPAN + 2)) ||
            (r = dalloc(x.sidx, sidx_off(h.cap_dir, SIDX_LEVELS + 1))) || (r = dalloc(x.fpx, h.cap_dir)) ||
            (r = dalloc(x.spx, sidx_off(h.cap_dir, SIDX_LEVELS + 1))) ||
            (r = dalloc(x.wsk, wsk_off(h.cap_dir, SIDX_LEVELS + 1))))
            return r;
        HIPOK(hipMemsetAsync(x.wsk, 0, wsk_off(h.cap_dir, SIDX_LEVELS + 1) * sizeof(int32_t), cs->stream));
        x.cap = h.cap_dir;
    }
    return FDBCS_OK;
}

void free_pool(HistBufs& h) {
    dfree(h.pool.hi); dfree(h.pool.lo); dfree(h.pool.meta); dfree(h.pool.ver); dfree(h.pool.tail);
    dfree(h.pool.pidx); dfree(h.pool.hmask); dfree(h.free_stack);
    dfree(h.pool.px); dfree(h.pool.pxidx); dfree(h.pool.pskip); dfree(h.px_list);
    for (int d = 0; d < 2; d++) {
        Dir& x = h.dir[d];
        dfree(x.page); dfree(x.cnt); dfree(x.nr); dfree(x.maxv); dfree(x.start); dfree(x.fhi); dfree(x.flo); dfree(x.fmeta);
        dfree(x.ftail); dfree(x.bmax); dfree(x.bmax2); dfree(x.sidx); dfree(x.fpx); dfree(x.spx); dfree(x.wsk);
    }
}

void adopt_scalars(fdbcs* cs) {
    cs->known_D = cs->sc_host->D;
    cs->known_free = cs->sc_host->free_top;
    cs->known_H = cs->sc_host->H;
    cs->known_tail = cs->sc_host->tail_used;
    cs->pending_pages = 0;
    cs->pending_tail = 0;
}

int ensure_pinned(uint8_t*& p, size_t& cap, size_t need) {
    if (need <= cap) return FDBCS_OK;
    if (p) hipHostFree(p);
    p = nullptr;
    size_t n = std::max(need, cap * 2);
    hipError_t e = hipHostMalloc((void**)&p, n, hipHostMallocDefault);
    if (e != hipSuccess) {
        last_hip_error() = e;
        cap = 0;
        return FDBCS_E_NOMEM;
    }
    cap = n;
    return FDBCS_OK;
}

// FDBCS_VERBOSE=1: log every buffer growth (reallocations stall the stream)
static bool verbose() {
    static const bool v = getenv("FDBCS_VERBOSE") != nullptr;
    return v;
}
#define GROWLOG(...) \
    do { \
        if (verbose()) fprintf(stderr, "# fdbcs grow: " __VA_ARGS__); \
    } while (0)

// A live batch still open (between fdbcs_batch_begin and fdbcs_batch_detect)
// holds the stream with its kernel: anything else that queues on the stream,
// or waits for it, first cancels it (the kernel leaves, its partial work is
// undone behind it; the batch is then ingested whole at detectConflicts).
void live_quiesce(fdbcs* cs) {
    if (!cs->st.live_active()) return;
    cs->b.lv_wbase = 0;  // (whatever runs next lays its batch out as the view does)
    cs->b.lv_nb1 = 0;
    cs->st.live_cancel();
    launch_live_reset(cs->b, cs->sc, (int)(cs->sorts & 1), cs->stream);
}

int sync_state(fdbcs* cs) {
    live_quiesce(cs);
    HIPOK(hipMemcpyAsync(cs->sc_host, cs->sc, sizeof(Scalars), hipMemcpyDeviceToHost, cs->stream));
    HIPOK(hipStreamSynchronize(cs->stream));
    adopt_scalars(cs);
    return FDBCS_OK;
}

// (a path other than run_batch changed the state behind the mirror slots:
// reset, load, pool or tail growth, the sharded steps)
void mirrors_stale(fdbcs* cs) {
    cs->end_mirror = false;
    cs->mirror_batch[0] = cs->mirror_batch[1] = ~0ull;
}

// The scalars after everything issued: from the host-mapped mirror when the
// last run_batch (which publishes them at its end) has finished; else from
// the one before it, whose slot the last batch's update does not touch (the
// budget then keeps what the last batch reserved, last_need_*).  When the
// device is the bottleneck the last batch's update is still running at the
// next batch's ensure_history: the stream sync this used to take there (one
// batch in four to eight at config 2) held the next launches back.  Else a
// stream sync.
int refresh_state(fdbcs* cs) {
    if (cs->end_mirror && cs->batches) {
        const uint64_t n = cs->batches - 1;  // (inside run_batch: batch n + 1 is being set up)
        static const bool prev = !getenv("FDBCS_MIRROR_PREV") || atoi(getenv("FDBCS_MIRROR_PREV"));  // (A/B)
        const int backs = prev ? (int)std::min<uint64_t>(n, 1) : 0;
        for (int back = 0; back <= backs; back++) {
            const int slot = (int)((n - back) & 1);
            if (cs->mirror_batch[slot] != n - back || hipEventQuery(cs->ev_slot[slot]) != hipSuccess) continue;
            memcpy(cs->sc_host, (const void*)(cs->sc_mapped + slot), sizeof(Scalars));
            adopt_scalars(cs);
            if (back) {
                cs->pending_pages = cs->last_need_pages;
                cs->pending_tail = cs->last_need_tail;
            }
            return FDBCS_OK;
        }
    }
    return sync_state(cs);
}

// The sort's overflow guard (k_ss_guard, ≈ 4.6 us a batch even when it finds
// nothing): launched unless the last finished batch's buckets stayed well
// inside their staging rows (Scalars::ss_maxc below SORT_GUARD_MAXC, not
// bucketed twice), read from its mirror slot (refresh_state's).  A bucket
// that overflows without it is ranked by the bucket kernel's global path --
// the same result, slower for that batch -- and the next batch's splitters
// come from this one's sorted output.  FDBCS_SORT_GUARD=1 / 0: always / never.
bool sort_guard(fdbcs* cs) {
    const char* e = getenv("FDBCS_SORT_GUARD");  // (read per batch: tests switch it)
    const int env = e ? atoi(e) : -1;
    if (env >= 0) return env != 0;
    if (!cs->end_mirror || cs->batches < 2) return true;
    const uint64_t n = cs->batches - 1;  // (inside run_batch: the latest published batch)
    for (int back = 0; back <= 1; back++) {
        const int slot = (int)((n - back) & 1);
        if (cs->mirror_batch[slot] != n - back || hipEventQuery(cs->ev_slot[slot]) != hipSuccess) continue;
        const Scalars* m = cs->sc_mapped + slot;
        return m->ss_resample != 0 || m->ss_maxc >= SORT_GUARD_MAXC;
    }
    return true;
}

// Wait for the stream.  FDBCS_SYNC_SPIN=1: poll instead of the runtime's
// blocking wait (the resolver thread stays on its core).
int wait_stream(fdbcs* cs) {
    static const bool spin = getenv("FDBCS_SYNC_SPIN") && atoi(getenv("FDBCS_SYNC_SPIN"));
    if (!spin) {
        HIPOK(hipStreamSynchronize(cs->stream));
        return FDBCS_OK;
    }
    for (;;) {
        const hipError_t e = hipStreamQuery(cs->stream);
        if (e == hipSuccess) return FDBCS_OK;
        if (e != hipErrorNotReady) {
            last_hip_error() = e;
            return FDBCS_E_HIP;
        }
        _mm_pause();
    }
}

// Wait for an event (FDBCS_SYNC_SPIN as wait_stream).
int wait_event(hipEvent_t ev) {
    static const bool spin = getenv("FDBCS_SYNC_SPIN") && atoi(getenv("FDBCS_SYNC_SPIN"));
    if (!spin) {
        HIPOK(hipEventSynchronize(ev));
        return FDBCS_OK;
    }
    for (;;) {
        const hipError_t e = hipEventQuery(ev);
        if (e == hipSuccess) return FDBCS_OK;
        if (e != hipErrorNotReady) {
            last_hip_error() = e;
            return FDBCS_E_HIP;
        }
        _mm_pause();
    }
}

// After a batch: its last kernel has written the scalars to the mapped copy.
int sync_batch(fdbcs* cs) {
    int r;
    if ((r = wait_stream(cs))) return r;
    memcpy(cs->sc_host, (const void*)cs->h.mirror_host, sizeof(Scalars));  // (the slot of the last publish)
    adopt_scalars(cs);
    return FDBCS_OK;
}

// Grow the page pool (and directories) to at least `pages`, preserving content.
int grow_pool(fdbcs* cs, int64_t pages) {
    int r;
    if ((r = sync_state(cs))) return r;
    mirrors_stale(cs);  // (the slots' free counts are the old pool's)
    HistBufs old = cs->h;
    int64_t np = std::max<int64_t>(pages, (int64_t)old.cap_pages * 2);
    GROWLOG("pool %d -> %lld pages (asked %lld)\n", old.cap_pages, (long long)np, (long long)pages);
    if (np > INT32_MAX / 2) return FDBCS_E_CAPACITY;
    if ((r = alloc_pool(cs, (int32_t)np))) return r;
    HistBufs& h = cs->h;
    const size_t os = (size_t)old.cap_pages * PAGE;
    hipStream_t s = cs->stream;
    HIPOK(hipMemcpyAsync(h.pool.hi, old.pool.hi, os * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.lo, old.pool.lo, os * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.meta, old.pool.meta, os * 4, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.ver, old.pool.ver, os * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.tail, old.pool.tail, os * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.pidx, old.pool.pidx, os / PIDX_STRIDE * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.hmask, old.pool.hmask, (size_t)old.cap_pages * HM_WORDS * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.px, old.pool.px, os * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.pxidx, old.pool.pxidx, os / PIDX_STRIDE * 8, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.pskip, old.pool.pskip, (size_t)old.cap_pages * 4, hipMemcpyDeviceToDevice, s));
    HIPOK(hipMemcpyAsync(h.free_stack, old.free_stack, (size_t)old.cap_pages * 4, hipMemcpyDeviceToDevice, s));
    const size_t od = (size_t)old.cap_dir;
    for (int d = 0; d < 2; d++) {
        HIPOK(hipMemcpyAsync(h.dir[d].page, old.dir[d].page, od * 4, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].cnt, old.dir[d].cnt, od * 4, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].nr, old.dir[d].nr, od * 4, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].maxv, old.dir[d].maxv, od * 8, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].start, old.dir[d].start, (od + 1) * 8, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].fhi, old.dir[d].fhi, od * 8, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].flo, old.dir[d].flo, od * 8, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].fmeta, old.dir[d].fmeta, od * 4, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].ftail, old.dir[d].ftail, od * 8, hipMemcpyDeviceToDevice, s));
        HIPOK(hipMemcpyAsync(h.dir[d].bmax, old.dir[d].bmax, (od / 64 + 2) * 8, hipMemcpyDeviceToDevice, s));
        // (bmax2 is rebuilt by every ingest, but a live batch's was built by
        // its kernel during the adds: run_batch may grow the pool after that)
        HIPOK(hipMemcpyAsync(h.dir[d].bmax2, old.dir[d].bmax2, (od / BMAX2_SPAN + 2) * 8, hipMemcpyDeviceToDevice, s));
    }
    launch_sidx_build(h, cs->cur, cs->sc, s);  // index levels are laid out by capacity
    launch_push_free(h, (int32_t)cs->known_free, old.cap_pages, (int32_t)(np - old.cap_pages), s);
    HIPOK(hipStreamSynchronize(s));
    free_pool(old);
    cs->known_free += np - old.cap_pages;
    Scalars tmp = *cs->sc_host;
    tmp.free_top = (int32_t)cs->known_free;
    HIPOK(hipMemcpyAsync(&cs->sc->free_top, &tmp.free_top, sizeof(int32_t), hipMemcpyHostToDevice, s));
    HIPOK(hipStreamSynchronize(s));
    cs->capDirB = -1;  // per-batch arrays sized by cap_dir must be re-sized
    return FDBCS_OK;
}

// Grow the tail arena so that each half holds at least need_half bytes; each
// old half lands at the start of the same new half (pointers relocated).
int grow_tail(fdbcs* cs, uint64_t need_half) {
    int r;
    if ((r = sync_state(cs))) return r;
    mirrors_stale(cs);  // (the slots' tail figures are the old arena's)
    HistBufs& h = cs->h;
    const uint64_t ncap = std::max<uint64_t>(2 * need_half + 16, h.tail_cap * 2);
    GROWLOG("tail arena %llu -> %llu bytes\n", (unsigned long long)h.tail_cap, (unsigned long long)ncap);
    uint8_t* na = nullptr;
    if ((r = dalloc(na, (int64_t)ncap))) return r;
    const uint64_t oh = tail_half_bytes(h.tail_cap), nh = tail_half_bytes(ncap);
    HIPOK(hipMemcpyAsync(na, h.tail_arena, oh, hipMemcpyDeviceToDevice, cs->stream));
    HIPOK(hipMemcpyAsync(na + nh, h.tail_arena + oh, oh, hipMemcpyDeviceToDevice, cs->stream));
    launch_relocate_tails(h, h.tail_arena, h.tail_cap, na, ncap, cs->stream);
    HIPOK(hipStreamSynchronize(cs->stream));
    dfree(h.tail_arena);
    h.tail_arena = na;
    h.tail_cap = ncap;
    return FDBCS_OK;
}

int alloc_keys(KeyArrays& k, int64_t n) {
    int r;
    if ((r = dalloc(k.hi, n)) || (r = dalloc(k.lo, n)) || (r = dalloc(k.meta, n)) || (r = dalloc(k.tail, n)))
        return r;
    return FDBCS_OK;
}
void free_keys(KeyArrays& k) { dfree(k.hi); dfree(k.lo); dfree(k.meta); dfree(k.tail); }

void free_plan(BatchBufs& b) {
    dfree(b.acc.er); dfree(b.acc.nn); dfree(b.acc.jlo); dfree(b.acc.jhi); dfree(b.acc.diff);
    dfree(b.blk_agg); dfree(b.blk_diff);
    dfree(b.aff_list); dfree(b.aff_jlo); dfree(b.aff_jhi); dfree(b.aff_nn); dfree(b.aff_parts);
    dfree(b.aff_nn_off); dfree(b.aff_parts_off); dfree(b.aff_extra_off); dfree(b.aff_free_off); dfree(b.aff_start);
    dfree(b.freed_list); dfree(b.full_list); dfree(b.aff_page); dfree(b.aff_cnt);
}

void free_batch(BatchBufs& b) {
    dfree(b.too_old); dfree(b.hist); dfree(b.committed); dfree(b.verdict); dfree(b.dec_blk);
    dfree(b.deg); dfree(b.off); dfree(b.cur); dfree(b.dep_list); dfree(b.dep_idx); dfree(b.cbits);
    dfree(b.read_txn); dfree(b.read_snap); dfree(b.write_txn);
    dfree(b.keys.hi); dfree(b.keys.lo); dfree(b.keys.meta); dfree(b.keys.tail); dfree(b.btail);
    dfree(b.rec_r0); dfree(b.rec_w0); dfree(b.sw_slot);
    dfree(b.ss_cnt); dfree(b.ss_gsamp); dfree(b.ss_q); dfree(b.ss_qt); dfree(b.ss_bkt); dfree(b.ss_tmp); dfree(b.lb_meta); dfree(b.lb_hist);
    dfree(b.et); dfree(b.eu); dfree(b.csr);
    dfree(b.rq); dfree(b.rstamp); dfree(b.plist); dfree(b.items); dfree(b.wnew); dfree(b.winv); dfree(b.wcov);
    dfree(b.pj_fall);
    dfree(b.cb_pos); dfree(b.ce_pos); dfree(b.comb_blk); free_keys(b.rkb); free_keys(b.rke);
    dfree(b.pb); dfree(b.ib); dfree(b.pe); dfree(b.ie); dfree(b.need_e); dfree(b.vb);
    dfree(b.wh.b); dfree(b.wh.e);
    free_plan(b);
    dfree(b.ne.hi); dfree(b.ne.lo); dfree(b.ne.meta); dfree(b.ne.ver); dfree(b.ne.tail); dfree(b.ne_ins);
    dfree(b.desc_page); dfree(b.desc_cnt); dfree(b.desc_nr); dfree(b.desc_max); dfree(b.desc_fhi); dfree(b.desc_flo);
    dfree(b.desc_fmeta); dfree(b.desc_ftail);
    dfree(b.win_keep); dfree(b.win_cnt); dfree(b.win_off);
    dfree(b.scan_tmp);
}


int grow_edges(BatchBufs& b, int64_t n) {
    int r;
    dfree(b.et); dfree(b.eu); dfree(b.csr);
    b.edge_cap = 0;
    if ((r = dalloc(b.et, n)) || (r = dalloc(b.eu, n)) || (r = dalloc(b.csr, n))) return r;
    b.edge_cap = n;
    return FDBCS_OK;
}

// Size the per-batch buffers (grow only).
int ensure_batch(fdbcs* cs, int64_t T, int64_t R, int64_t W, uint64_t key_bytes) {
    BatchBufs& b = cs->b;
    int r;
    hipStream_t s = cs->stream;
    if (T > MAX_T) return FDBCS_E_CAPACITY;  // DESIGN.md §Large batches
    b.large = large_batch_mode(T);
    b.rounds = !b.large && !cs->sparse_edges && rounds_fit(T, W);
    if (!b.scan_tmp && (r = dalloc(b.scan_tmp, 1024))) return r;
    if (T > cs->capT) {
        GROWLOG("T %lld\n", (long long)T);
        int64_t n = std::max<int64_t>(T, 1024);
        dfree(b.too_old); dfree(b.hist); dfree(b.committed); dfree(b.verdict); dfree(b.dec_blk);
        dfree(b.deg); dfree(b.off); dfree(b.cur); dfree(b.dep_list); dfree(b.dep_idx); dfree(b.cbits);
        if ((r = dalloc(b.too_old, n + 64)) || (r = dalloc(b.hist, n + 64)) || (r = dalloc(b.committed, n)) ||
            (r = dalloc(b.verdict, n)) || (r = dalloc(b.deg, n)) || (r = dalloc(b.off, n + 1)) ||
            (r = dalloc(b.cur, n)) || (r = dalloc(b.dep_list, n)) || (r = dalloc(b.dep_idx, n)) ||
            (r = dalloc(b.cbits, n / 64 + 2)) ||
            (r = dalloc(b.dec_blk, 2 * (n / 256 + 2))))
            return r;
        cs->capT = n;
    }
    int64_t need_edges = 1;
    if (!b.rounds) {
        // overlap edges (duplicates kept): a first guess linear in the batch;
        // run_batch grows the list and re-runs the search if a batch overflows it
        const char* test_cap = getenv("FDBCS_TEST_EDGE_CAP");  // (tests: reach the overflow path)
        need_edges = test_cap ? std::max(1, atoi(test_cap)) : std::max<int64_t>(1 << 20, 2 * (R + W));
    }
    if (need_edges > b.edge_cap && (r = grow_edges(b, need_edges))) return r;
    if (R > cs->capR) {
        GROWLOG("R %lld\n", (long long)R);
        int64_t n = std::max<int64_t>(R, 1024);
        dfree(b.read_txn); dfree(b.read_snap); dfree(b.rec_r0); dfree(b.rq); dfree(b.rstamp);
        if ((r = dalloc(b.read_txn, n)) || (r = dalloc(b.read_snap, n)) || (r = dalloc(b.rec_r0, n)) ||
            (r = dalloc(b.rq, 2 * n)) || (r = dalloc(b.rstamp, n)))
            return r;
        if (hipMemsetAsync(b.rstamp, 0, (size_t)n * 4, cs->stream) != hipSuccess) return FDBCS_E_HIP;
        b.rseq = 0;
        cs->capR = n;
    }
    if (W > cs->capW) {
        GROWLOG("W %lld\n", (long long)W);
        int64_t n = std::max<int64_t>(W, 1024);
        dfree(b.write_txn); dfree(b.rec_w0); dfree(b.sw_slot);
        dfree(b.cb_pos); dfree(b.ce_pos); dfree(b.comb_blk); free_keys(b.rkb); free_keys(b.rke);
        dfree(b.pb); dfree(b.ib); dfree(b.pe); dfree(b.ie); dfree(b.need_e); dfree(b.vb);
        dfree(b.wh.b); dfree(b.wh.e);
        dfree(b.ne.hi); dfree(b.ne.lo); dfree(b.ne.meta); dfree(b.ne.ver); dfree(b.ne.tail); dfree(b.ne_ins);
        dfree(b.wnew); dfree(b.winv); dfree(b.wcov);
        if ((r = dalloc(b.wnew, 2 * n + 64)) || (r = dalloc(b.winv, 2 * n)) || (r = dalloc(b.wcov, 2 * n))) return r;
        if ((r = dalloc(b.write_txn, n + 32)) ||  // +32: read as 32-entry words by k_decide_rounds
             (r = dalloc(b.rec_w0, 2 * n)) || (r = dalloc(b.sw_slot, 2 * n)) ||
            (r = dalloc(b.cb_pos, n)) || (r = dalloc(b.ce_pos, n)) || (r = dalloc(b.comb_blk, 2 * (n / 2048 + 2))) ||
            (r = alloc_keys(b.rkb, n)) ||
            (r = alloc_keys(b.rke, n)) || (r = dalloc(b.pb, n)) ||
            (r = dalloc(b.ib, n)) || (r = dalloc(b.pe, n)) || (r = dalloc(b.ie, n)) || (r = dalloc(b.need_e, n)) ||
            (r = dalloc(b.vb, n)) || (r = dalloc(b.ne.hi, 2 * n)) || (r = dalloc(b.ne.lo, 2 * n)) ||
            (r = dalloc(b.ne.meta, 2 * n)) || (r = dalloc(b.ne.ver, 2 * n)) || (r = dalloc(b.ne.tail, 2 * n)) ||
            (r = dalloc(b.ne_ins, 2 * n)) || (r = dalloc(b.wh.b, n)) || (r = dalloc(b.wh.e, n)))
            return r;
        cs->capW = n;
    }
    if (++b.rseq == 0) {  // (stamps wrapped: clear them)
        if (b.rstamp && hipMemsetAsync(b.rstamp, 0, (size_t)cs->capR * 4, cs->stream) != hipSuccess) return FDBCS_E_HIP;
        b.rseq = 1;
    }
    if (R + W > b.list_cap) {
        const int64_t n = std::max<int64_t>(R + W, 4096);
        dfree(b.plist); dfree(b.items);
        b.list_cap = 0;
        if ((r = dalloc(b.plist, n)) || (r = dalloc(b.items, 2 * n))) return r;
        b.list_cap = n;
    }
    if (!b.ss_cnt) {
        if ((r = dalloc(b.ss_cnt, 2 * 3 * 1024)) || (r = dalloc(b.ss_q, 2 * 1024)) ||
            (r = dalloc(b.ss_qt, 2 * 1024 * SS_QT)) || (r = dalloc(b.ss_gsamp, 2 * 3 * 4096)))
            return r;
        HIPOK(hipMemsetAsync(b.ss_qt, 0, 2 * 1024 * SS_QT, s));
        HIPOK(hipMemsetAsync(b.ss_cnt, 0, 2 * 3 * 1024 * sizeof(int32_t), s));  // (kernels_batch.hip SS_CNT per parity)
        HIPOK(hipMemsetAsync(b.ss_q, 0, 2 * 1024 * sizeof(SRec), s));  // equal records: valid (sorted) splitters
    }
    if (!b.lb_meta && (r = dalloc(b.lb_meta, lb_meta_words()))) return r;
    if (b.large && R + 2 * W + 64 > b.pj_cap) {  // (k_page_join's lists)
        const int64_t n = R + 2 * W + 64;
        dfree(b.pj_fall);
        b.pj_cap = 0;
        if ((r = dalloc(b.pj_fall, n))) return r;
        b.pj_cap = n;
    }
    if (b.large && lb_hist_words((int)R, (int)W) + 1 > b.lb_hist_cap) {
        const int64_t n = lb_hist_words((int)R, (int)W) + 1;
        dfree(b.lb_hist);
        b.lb_hist_cap = 0;
        if ((r = dalloc(b.lb_hist, 2 * n))) return r;
        b.lb_hist_cap = n;
    }
    if (R + 2 * W > cs->capSortRec) {
        const int64_t n = std::max<int64_t>(R + 2 * W, 4096);
        dfree(b.ss_bkt);
        if ((r = dalloc(b.ss_bkt, n))) return r;
        cs->capSortRec = n;
    }
    const int64_t stage = sort_staging_records((int)R, (int)W, b.large);
    if (stage > b.ss_tmp_cap) {
        const int64_t n = std::max<int64_t>(stage, 1 << 16);
        dfree(b.ss_tmp);
        if ((r = dalloc(b.ss_tmp, n))) return r;
        b.ss_tmp_cap = n;
    }
    const int64_t slots = 2 * (R + W);
    if (slots > cs->capSlots) {
        GROWLOG("slots %lld\n", (long long)slots);
        int64_t n = std::max<int64_t>(slots, 4096);
        free_keys(b.keys);
        if ((r = alloc_keys(b.keys, n))) return r;
        cs->capSlots = n;
    }
    const uint64_t btail_need = key_bytes + 8 * (uint64_t)slots + 64;
    if ((int64_t)btail_need > cs->capBtail) {
        GROWLOG("btail %llu\n", (unsigned long long)btail_need);
        uint64_t n = std::max<uint64_t>(btail_need, 1 << 16);
        dfree(b.btail);
        if ((r = dalloc(b.btail, (int64_t)n))) return r;
        b.btail_cap = n;
        cs->capBtail = (int64_t)n;
    }
    const int64_t win_pages = 3 * std::max<int64_t>(W, 1024) + 16;
    if (win_pages > cs->capWinPages) {
        GROWLOG("win pages %lld\n", (long long)win_pages);
        dfree(b.win_keep); dfree(b.win_cnt); dfree(b.win_off);
        if ((r = dalloc(b.win_keep, win_pages * PAGE)) || (r = dalloc(b.win_cnt, win_pages)) ||
            (r = dalloc(b.win_off, win_pages + 2)))
            return r;
        b.win_cap_pages = (int32_t)win_pages;
        cs->capWinPages = win_pages;
    }
    const int64_t cd = cs->h.cap_dir;
    if (cd > cs->capDirB) {
        free_plan(b);
        const int64_t n = cd + 2;
        const int64_t nblk = plan_blocks((int)cd) + 1;
        if ((r = dalloc(b.acc.er, n)) || (r = dalloc(b.acc.nn, n)) || (r = dalloc(b.acc.jlo, n)) ||
            (r = dalloc(b.acc.jhi, n)) || (r = dalloc(b.acc.diff, n)) || (r = dalloc(b.blk_agg, 6 * nblk)) ||
            (r = dalloc(b.blk_diff, nblk)) || (r = dalloc(b.aff_list, n)) || (r = dalloc(b.aff_jlo, n)) ||
            (r = dalloc(b.aff_jhi, n)) || (r = dalloc(b.aff_nn, n)) || (r = dalloc(b.aff_parts, n)) ||
            (r = dalloc(b.aff_nn_off, n)) || (r = dalloc(b.aff_parts_off, n)) || (r = dalloc(b.aff_extra_off, n)) ||
            (r = dalloc(b.aff_free_off, n)) || (r = dalloc(b.aff_start, n)) || (r = dalloc(b.freed_list, n)) ||
            (r = dalloc(b.aff_page, n)) || (r = dalloc(b.aff_cnt, n)) || (r = dalloc(b.full_list, n)))
            return r;
        HIPOK(hipMemsetAsync(b.acc.er, 0, n * 4, s));
        HIPOK(hipMemsetAsync(b.acc.nn, 0, n * 4, s));
        HIPOK(hipMemsetAsync(b.acc.diff, 0, n * 4, s));
        HIPOK(hipMemsetAsync(b.acc.jlo, 0x7F, n * 4, s));  // "no range yet" (> any range index)
        HIPOK(hipMemsetAsync(b.acc.jhi, 0xFF, n * 4, s));  // -1
        cs->capDirB = cd;
    }
    // page descriptors: the merge makes at most cap_dir of them, the compaction
    // window initialises 2 per window page
    const int64_t nd = std::max<int64_t>(cd + 2, 2 * cs->capWinPages + 2);
    if (nd > cs->capDesc) {
        dfree(b.desc_page); dfree(b.desc_cnt); dfree(b.desc_nr); dfree(b.desc_max); dfree(b.desc_fhi); dfree(b.desc_flo);
        dfree(b.desc_fmeta); dfree(b.desc_ftail);
        if ((r = dalloc(b.desc_page, nd)) || (r = dalloc(b.desc_cnt, nd)) || (r = dalloc(b.desc_nr, nd)) ||
            (r = dalloc(b.desc_max, nd)) ||
            (r = dalloc(b.desc_fhi, nd)) || (r = dalloc(b.desc_flo, nd)) || (r = dalloc(b.desc_fmeta, nd)) ||
            (r = dalloc(b.desc_ftail, nd)))
            return r;
        cs->capDesc = nd;
    }
    return FDBCS_OK;
}

// Make sure the pool and the tail arena can absorb one more batch of W writes
// in the worst case.
int ensure_history(fdbcs* cs, int64_t W, uint64_t write_tail_bytes) {
    int r;
    // (worst case: every affected page splits; the directory bound counts the
    // pages the unsynchronized batches may have added)
    auto need_pages = [&]() {
        const int64_t naff_max = std::min<int64_t>(cs->known_D + cs->pending_pages + 1, 2 * W + 2);
        return 2 * naff_max + 2 * cdiv64(2 * W, FILL) + cdiv64(3 * W + 10 + 2 * PAGE, FILL) + 8;
    };
    int64_t need = need_pages();
    if (cs->known_free - cs->pending_pages < need) {
        if (cs->pending_pages) {
            if ((r = refresh_state(cs))) return r;
            need = need_pages();  // (the exact directory size now: the pending bound was loose --
                                  // config 5's unsynchronized batches asked a 312 GB pool)
        }
        if (cs->known_free < need) {
            const int64_t used = cs->h.cap_pages - cs->known_free;
            if ((r = grow_pool(cs, used + 4 * need + 1024))) return r;  // (slack: fewer syncs behind early verdicts)
        }
    }
    const uint64_t tneed = write_tail_bytes + 8 * 2 * (uint64_t)W + 64;
    // merges allocate in the current half; the compaction's GC moves never
    // take it past its middle, so since the last sync the used part is at
    // most max(known, half / 2) plus the merges
    const uint64_t half = tail_half_bytes(cs->h.tail_cap);
    auto fits = [&](uint64_t pend) { return std::max(cs->known_tail, half / 2) + pend + tneed <= half; };
    if (!fits(cs->pending_tail)) {
        if (cs->pending_tail && (r = refresh_state(cs))) return r;
        if (!fits(0)) {
            if ((r = grow_tail(cs, 2 * (cs->known_tail + 2 * tneed + (1 << 20))))) return r;
        }
    }
    cs->pending_pages += need;
    cs->pending_tail += tneed;
    cs->last_need_pages = need;
    cs->last_need_tail = tneed;
    return FDBCS_OK;
}

// History read check + overlap edges.  Large batches keep duplicate edges in
// a list sized linearly in the batch: if it overflowed, grow it to the count
// the kernel reached and search again (the read check is idempotent; the
// per-reader source counts restart from zero).
// Directory entries of the batch's keys by one merge-join of the sorted keys
// with the directory's first keys (k_dir_join) instead of a search-index
// descent per key: large batches.  FDBCS_DIR_JOIN=1: every batch (A/B and
// tests).  Measured for long keys over a small directory (config 4, keys
// sharing 64-byte prefixes, D ~ 9 K): read check + edges 367 us with the join
// against 275 us without -- the join's merge-path compares are tail compares
// too, and the end keys and page searches remain.
bool want_dir_join(const fdbcs* cs) {
    static const bool force = getenv("FDBCS_DIR_JOIN") && atoi(getenv("FDBCS_DIR_JOIN"));
    return cs->b.large || force;
}

int edges_read_check(fdbcs* cs, const fdbcs_batch_view& v, int64_t v0, bool defer_ws = false) {
    BatchBufs& b = cs->b;
    hipStream_t s = cs->stream;
    b.dir_join = want_dir_join(cs);
    launch_edges_read_check(v, b, cs->h, cs->cur, cs->sc, v0, s, defer_ws && b.rounds);
    if (b.rounds) return FDBCS_OK;  // (no overlap pairs: k_decide_rounds)
    int32_t total = 0;
    HIPOK(hipMemcpyAsync(&total, &cs->sc->edges_total, sizeof(total), hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    if (total >= 0 && total <= b.edge_cap) return FDBCS_OK;
    if (total < 0) return FDBCS_E_CAPACITY;  // (more than 2^31 overlap pairs in one batch)
    GROWLOG("edges %d\n", total);
    int r;
    if ((r = grow_edges(b, (int64_t)total + total / 4 + 1024))) return r;
    HIPOK(hipMemsetAsync(b.deg, 0, (size_t)v.txn_count * sizeof(int32_t), s));
    HIPOK(hipMemsetAsync(&cs->sc->edges_total, 0, sizeof(int32_t), s));
    launch_edges_read_check(v, b, cs->h, cs->cur, cs->sc, v0, s);
    return FDBCS_OK;
}

void record(fdbcs* cs, int i) {
    if (cs->timing) hipEventRecord(cs->ev[i], cs->stream);
}

// per-stage HIP-event times of the batch just synchronized (stage timing on)
void read_stage_times(fdbcs* cs) {
    if (!cs->timing) return;
    float ms;
    const int map[7][2] = {{0, 1}, {1, 2}, {2, 3}, {3, 4}, {4, 5}, {5, 6}, {0, 6}};
    for (int i = 0; i < 7; i++) {
        hipEventElapsedTime(&ms, cs->ev[map[i][0]], cs->ev[map[i][1]]);
        cs->stage_us[i] = ms * 1000.0;
    }
    cs->have_times = true;
}

// The whole detectConflicts pipeline on a device-resident batch.
// early: copy the verdicts and a scalar snapshot to cs->vpin right after the
// decision and record ev_verdict (finish with verdict_wait).
int debug_check_dir(fdbcs* cs, const char* where);

int run_batch(fdbcs* cs, const fdbcs_batch_view& v, int64_t now, int64_t new_oldest, uint8_t* dev_verdict,
              bool sync, bool early = false, const LmArgs* lm = nullptr) {
    int r;
    const int64_t T = v.txn_count, R = v.read_count, W = v.write_count;
    if (T < 0 || R < 0 || W < 0) return FDBCS_E_ARG;
    cs->batches++;
    cs->edges_known = false;
    cs->have_last_dv = false;  // (the host paths set it again once this batch succeeded)
    cs->last_wbase = 0;
    // (a staged batch's keys can outnumber its stream's bytes: point ranges
    // share theirs, stage.hip)
    const bool live = cs->b.staged.live;
    uint64_t kb = std::max<uint64_t>(v.key_bytes_len, cs->stage_key_total);
    if (live) {
        // k_live_ingest wrote this batch's keys, tails and sort records during
        // the adds: ensure_batch must not move any buffer (a moved btail left
        // keys.tail pointing into freed memory).  live_begin sized them for
        // the capacities the batch stayed within, stream padding included.
        if (kb > cs->lv_kb) return FDBCS_E_STATE;
        kb = cs->lv_kb;
    }
    const BatchBufs held = cs->b;
    if ((r = ensure_batch(cs, T, R, W, kb))) return r;
    if (live && (held.btail != cs->b.btail || held.keys.hi != cs->b.keys.hi || held.keys.tail != cs->b.keys.tail ||
                 held.ss_tmp != cs->b.ss_tmp || held.ss_bkt != cs->b.ss_bkt || held.read_txn != cs->b.read_txn ||
                 held.write_txn != cs->b.write_txn || held.too_old != cs->b.too_old || held.wcov != cs->b.wcov))
        return FDBCS_E_STATE;  // (cannot happen: the capacities bound every size; never compute on moved buffers)
    if ((r = ensure_history(cs, W, kb))) return r;
    if (early && (r = ensure_pinned(cs->vpin, cs->vpin_cap, vpin_scalars_off(T) + sizeof(Scalars)))) return r;
    if (early && (size_t)T + 64 > cs->vmap_cap) {
        if (cs->vmap) hipHostFree(cs->vmap);
        cs->vmap = cs->vmap_dev = nullptr;
        cs->vmap_cap = 0;
        const size_t n = std::max<size_t>((size_t)T + 64, 2 * cs->vmap_cap) + 4096;
        if (hipHostMalloc((void**)&cs->vmap, n, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return FDBCS_E_NOMEM;
        memset(cs->vmap, 0, n);
        HIPOK(hipHostGetDevicePointer((void**)&cs->vmap_dev, cs->vmap, 0));
        cs->vmap_cap = n;
        cs->vseq = 0;
    }
    cs->last_T = T;
    cs->last_R = R;
    cs->last_W = W;
    BatchBufs& b = cs->b;
    HistBufs& h = cs->h;
    hipStream_t s = cs->stream;
    Scalars* sc = cs->sc;
    record(cs, 0);
    static const bool no_fuse = getenv("FDBCS_SEPARATE_SCATTER") != nullptr;  // (A/B measurements)
    // steady state: the ingest scatters the sort records (large batches merge-sort instead)
    const bool scatter = cs->have_quantiles && !no_fuse && !b.large;
    if (live) {  // k_live_ingest encoded the batch during the adds (writes from b.lv_wbase)
        cs->lv_done++;
    } else {
        b.lv_wbase = 0;  // (the view's own layout: writes from 2R)
        b.lv_nb1 = 0;
        if (b.staged.live_failed) {
            launch_live_reset(b, sc, (int)(cs->sorts & 1), s);
            cs->lv_cancelled++;
        }
        launch_ingest(v, cs->oldest, b, sc, scatter, (int)(cs->sorts & 1), cs->h.dir[cs->cur], s,
                      (cs->h.shard.has_lo | cs->h.shard.has_hi) != 0, lm);
    }
    record(cs, 1);
    if (launch_sort_ranges(v, b, sc, !cs->have_quantiles, (int)(cs->sorts & 1), scatter, s, &cs->h, cs->cur, cs->v0,
                           sort_guard(cs))) {
        cs->sorts++;
        cs->have_quantiles = true;
    }
    record(cs, 2);
    if ((r = edges_read_check(cs, v, cs->v0, early))) return r;
    record(cs, 3);
    EarlyOut eo{};
    if (early && !dev_verdict) {
        if (++cs->vseq == 0) cs->vseq = 1;
        eo = EarlyOut{cs->vmap_dev + 64, reinterpret_cast<uint32_t*>(cs->vmap_dev), cs->vseq};
    }
    // (the single-workgroup decision combines in the same launch, after it has
    // raised the verdict flag; the grid decision's combine follows the copies)
    const bool split = early && !b.rounds;
    // (the deferred write searches run as extra blocks of the decision's
    // launch: it holds one CU; a side stream cost ~7 us of event latency
    // before the decision)
    cs->early_mapped = launch_decide(v, b, sc, dev_verdict ? dev_verdict : b.verdict, s, split,
                                     eo.flag ? &eo : nullptr, &cs->h, cs->cur, cs->v0);
    if (early) {
        if (!cs->early_mapped) {  // (the grid decision of large batches: copies)
            if (T) HIPOK(hipMemcpyAsync(cs->vpin, dev_verdict ? dev_verdict : b.verdict, (size_t)T, hipMemcpyDeviceToHost, s));
            HIPOK(hipMemcpyAsync(cs->vpin + vpin_scalars_off(T), sc, sizeof(Scalars), hipMemcpyDeviceToHost, s));
        }
        // (mapped verdicts: the host polls their flag, and its fallback waits
        // for ev_end -- a marker here held the next launch ~10 us: A/B knob
        // FDBCS_VERDICT_EVENT=1)
        static const bool vev = getenv("FDBCS_VERDICT_EVENT") && atoi(getenv("FDBCS_VERDICT_EVENT"));
        cs->vev_rec = !cs->early_mapped || vev;
        if (cs->vev_rec) HIPOK(hipEventRecord(cs->ev_verdict, s));
        launch_write_search(v, b, cs->h, cs->cur, sc, cs->v0, s);  // (grid decision: for the merge, after the verdicts)
        if (split) launch_combine(v, b, sc, s);  // (the combined write ranges: after the verdicts)
    }
    record(cs, 4);
    const bool compact = new_oldest > cs->oldest;
    const int mslot = (int)(cs->batches & 1);  // (this batch's mirror slot: refresh_state)
    h.mirror = cs->mirror_dev + mslot;
    h.mirror_host = cs->sc_mapped + mslot;
    launch_merge(v, b, h, cs->cur, sc, now, cs->v0, !compact, s);
    cs->cur ^= 1;
    if ((r = debug_check_dir(cs, "merge"))) return r;
    record(cs, 5);
    if (compact) {
        launch_compact(b, h, cs->cur, sc, new_oldest, s);
        cs->cur ^= 1;
        if ((r = debug_check_dir(cs, "compaction"))) return r;
    }
    record(cs, 6);
    if (compact) cs->oldest = new_oldest;
    cs->ev_end = cs->ev_slot[mslot];
    HIPOK(hipEventRecord(cs->ev_end, s));
    cs->mirror_batch[mslot] = cs->batches;
    cs->end_mirror = true;
    if (sync) {
        if ((r = sync_batch(cs))) return r;
        read_stage_times(cs);
        if (cs->sc_host->last_err) return cs->sc_host->last_err;
    }
    return FDBCS_OK;
}

// The early verdicts of run_batch(early): wait for them (not for the history
// update behind them) and check the scalar snapshot taken with them: err =
// this batch's stages so far, last_err = the previous batch's history update
// (so a failed update is reported by the next detectConflicts).
int verdict_wait(fdbcs* cs, int64_t T, uint8_t* verdict, int64_t* lm_count = nullptr, int64_t* sh_max = nullptr) {
    int r;
    if (cs->early_mapped) {
        // poll the flag the decision kernel sets after its verdicts (no copy,
        // no interrupt); past ~2 ms block on the batch's end instead
        const uint32_t* flag = reinterpret_cast<const uint32_t*>(cs->vmap);
        const auto t0 = std::chrono::steady_clock::now();
        for (int it = 1; __atomic_load_n(flag, __ATOMIC_ACQUIRE) != cs->vseq; it++) {
            _mm_pause();
            if ((it & 255) == 0 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) {
                if ((r = wait_event(cs->vev_rec ? cs->ev_verdict : cs->ev_end))) return r;
                if (__atomic_load_n(flag, __ATOMIC_ACQUIRE) != cs->vseq) return FDBCS_E_HIP;
                break;
            }
        }
        const int32_t* err = reinterpret_cast<const int32_t*>(cs->vmap + 4);
        if (err[0]) return err[0];
        if (err[1]) return err[1];
        if (lm_count) *lm_count = (int64_t)reinterpret_cast<const uint32_t*>(cs->vmap)[3];
        if (sh_max) *sh_max = (int64_t)reinterpret_cast<const uint32_t*>(cs->vmap)[4];
        if (T) memcpy(verdict, cs->vmap + 64, (size_t)T);
        return FDBCS_OK;
    }
    if ((r = wait_event(cs->ev_verdict))) return r;
    const Scalars* snap = reinterpret_cast<const Scalars*>(cs->vpin + vpin_scalars_off(T));
    if (snap->err) return snap->err;
    if (snap->last_err) return snap->last_err;
    if (lm_count) *lm_count = snap->lm_count;
    if (sh_max) *sh_max = snap->sh_max;
    if (T) memcpy(verdict, cs->vpin, (size_t)T);
    return FDBCS_OK;
}

// Arm the attached sample's roll for the staged batch dv: its pinned outputs
// hold every range (a batch whose ranges were all sampled) and every key
// byte of the record stream (the begin keys sampled are disjoint parts of it).
int lm_arm(fdbcs* cs, uint64_t n_ranges, uint64_t key_bytes, LmArgs& la) {
    fdbcs::Lm& L = cs->lm;
    // Room for every range of a small batch; a large one samples ~0.6 % of its
    // ranges (config 5: ~54 K of 9 M), so 64 K + 1/16 of them, with up to 128
    // bytes of key each (16-byte pieces).  A batch past either capacity is
    // rolled again by fdbcs_sample_add_batch's synchronous path (the kernel
    // counts past the capacity and stops writing).
    const size_t n = (size_t)std::min<uint64_t>(n_ranges, 65536 + n_ranges / 16);
    const size_t nb = (size_t)std::min<uint64_t>((uint64_t)key_bytes + 16 * n_ranges + 64, (uint64_t)n * 128 + 65536);
    auto grow = [](auto*& p, size_t& cap, size_t need, size_t elem) {
        if (need <= cap && p) return (int)FDBCS_OK;
        const size_t c = std::max<size_t>(need + need / 4, 4096);
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        // (coherent: the ingest's blocks on every XCD store here and the host
        // reads right after the verdict flag; from default pinned memory the
        // stores of XCDs other than the deciding one's could still sit in
        // their L2 -- a sampled key then read as zeros)
        if (hipHostMalloc((void**)&p, c * elem, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return (int)FDBCS_E_NOMEM;
        cap = c;
        return (int)FDBCS_OK;
    };
    int r;
    if ((r = grow(L.ent, L.cap_n, n, sizeof(LmEntry))) || (r = grow(L.bytes, L.cap_b, nb, 1))) return r;
    la = LmArgs{1, L.seed, *L.seq, L.units, L.opk, L.ent, L.bytes, (uint32_t)std::min<size_t>(L.cap_n, UINT32_MAX),
                (uint64_t)L.cap_b};
    L.rolled_seq = *L.seq;
    return FDBCS_OK;
}

// FDBCS_LIVE=0: no live ingest (A/B measurements)
bool live_enabled() {
    static const bool on = !(getenv("FDBCS_LIVE") && !atoi(getenv("FDBCS_LIVE"))) &&
                           !getenv("FDBCS_SEPARATE_SCATTER") && !getenv("FDBCS_SEPARATE_UNPACK");
    return on;
}

// Live ingest: at fdbcs_batch_begin, k_live_ingest is queued
// behind the previous batch's history update and encodes this batch's
// transactions while the Resolver is still adding them (TxnStage publishes its
// progress every FDBCS_LIVE_PUB transactions); detectConflicts then starts
// at the sort (the writes sit at 2 caps.R + 2w, BatchBufs::lv_wbase).  Capacities: the last batch's shape plus
// a quarter -- a batch that outgrows them is cancelled on the way and ingested
// whole, as without live ingest.  Only the steady state goes live: splitters
// from an earlier batch, an unsharded set, small batches, no stage timing.
void live_begin(fdbcs* cs) {
    cs->lv_lm = false;
    auto up = [](int64_t x) { return x + x / 4 + 256; };
    LiveCaps c{};
    c.T = (int32_t)std::min<int64_t>(up(cs->lv_prev_T), LARGE_T);
    c.R = (int32_t)up(cs->lv_prev_R);
    c.W = (int32_t)up(cs->lv_prev_W);
    c.key_bytes = cs->lv_prev_K + cs->lv_prev_K / 4 + 65536;
    // A borrowed batch: helper threads pack it during the adds and copy it to
    // the device as it grows (TxnStage::begin_helpers), and detectConflicts
    // ingests it whole from device memory -- the live kernel's PCIe reads,
    // no longer paced by the adds, were the slower way in.
    // FDBCS_BORROW_LIVE=1: the helpers publish to the live kernel instead.
    // (Large batches pack at detect on every host thread: pack_borrowed.)
    const char* bl = getenv("FDBCS_BORROW_LIVE");  // (read per batch: tests switch it)
    const bool borrow_live = bl && atoi(bl);
    if (cs->st.borrowing() && !borrow_live) {
        if (cs->lv_prev_T > 0 && !large_batch_mode(c.T) && !large_batch_mode(cs->lv_prev_T)) cs->st.begin_helpers(c);
        return;
    }
    if (!live_enabled() || cs->timing || !cs->have_quantiles || cs->lv_prev_T <= 0 || cs->sparse_edges ||
        (cs->h.shard.has_lo | cs->h.shard.has_hi))
        return;
    if (large_batch_mode(c.T) || large_batch_mode(cs->lv_prev_T)) return;
    // the batch buffers at their final size before the kernel writes them (the
    // detect's ensure_batch must not move them): keys and the stream's bytes
    // (run_batch asks max(stream bytes, key bytes): the stream's bound
    // counts the publishes' padding, TxnStage::live_stream_bound)
    const uint64_t kb = std::max<uint64_t>(c.key_bytes, cs->st.live_stream_bound(c));
    BatchBufs& b = cs->b;
    if (ensure_batch(cs, c.T, c.R, c.W, kb) || !b.rounds) return;  // (the live kernel leaves the reads unsorted)
    if (cs->st.begin_live(c)) return;
    cs->lv_kb = kb;
    LmArgs la{};
    cs->lv_lm = cs->lm.owner && lm_arm(cs, (uint64_t)c.R + c.W, c.key_bytes, la) == FDBCS_OK;
    if (++cs->lv_gen == 0) cs->lv_gen = 1;
    launch_live_ingest(b, cs->sc, c, cs->oldest, (int)(cs->sorts & 1), cs->st.stream_dev(), cs->st.stream_cap(),
                       cs->st.toff_dev(), cs->st.prog_dev(), cs->st.live_view(), cs->lv_lm ? &la : nullptr,
                       cs->lv_gen, cs->h.dir[cs->cur], cs->lv_tune, cs->stream);
}

void lm_release(fdbcs::Lm& L) {
    if (L.ent) hipHostFree(L.ent);
    if (L.bytes) hipHostFree(L.bytes);
    L.ent = nullptr;
    L.bytes = nullptr;
    L.cap_n = L.cap_b = 0;
}

// FDBCS_DEBUG_DIR (debugging): after each history stage, wait and check the
// current directory against its pages -- start[] the prefix of nr[], nr[] the
// real slots of cnt[] under the hole mask, the copied first key the page's
// first slot, start[D] = H -- and name the stage and entry that broke it.
int debug_check_dir(fdbcs* cs, const char* where) {
    static const bool on = getenv("FDBCS_DEBUG_DIR") != nullptr;
    if (!on) return FDBCS_OK;
    int r;
    if ((r = sync_state(cs))) return r;
    const HistBufs& h = cs->h;
    const Dir& d = h.dir[cs->cur];
    const int64_t D = cs->sc_host->D, H = cs->sc_host->H;
    if (D < 1 || D > d.cap) {
        fprintf(stderr, "FDBCS_DEBUG_DIR %s: D=%lld out of [1, %d]\n", where, (long long)D, d.cap);
        return FDBCS_E_STATE;
    }
    std::vector<int32_t> page(D), cnt(D), nr(D);
    std::vector<int64_t> start(D + 1);
    std::vector<uint64_t> fhi(D);
    HIPOK(hipMemcpy(page.data(), d.page, D * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(cnt.data(), d.cnt, D * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(nr.data(), d.nr, D * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(start.data(), d.start, (D + 1) * 8, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(fhi.data(), d.fhi, D * 8, hipMemcpyDeviceToHost));
    int64_t acc = 0;
    for (int64_t x = 0; x < D; x++) {
        const char* bad = nullptr;
        uint64_t hm[HM_WORDS] = {0, 0, 0, 0}, hi0 = 0;
        if (page[x] < 0 || page[x] >= h.cap_pages) bad = "page id";
        else if (cnt[x] < 0 || cnt[x] > PAGE) bad = "cnt";
        else if (start[x] != acc) bad = "start";
        if (!bad) {
            HIPOK(hipMemcpy(hm, h.pool.hmask + (int64_t)page[x] * HM_WORDS, sizeof hm, hipMemcpyDeviceToHost));
            int holes = 0;
            for (int i = 0; i < cnt[x]; i++) holes += (int)((hm[i >> 6] >> (i & 63)) & 1);
            if (cnt[x] - holes != nr[x]) bad = "nr vs hole mask";
            if (cnt[x] > 0) {
                HIPOK(hipMemcpy(&hi0, h.pool.hi + (int64_t)page[x] * PAGE, 8, hipMemcpyDeviceToHost));
                if (hi0 != fhi[x]) bad = "first key";
            }
        }
        if (bad) {
            fprintf(stderr, "FDBCS_DEBUG_DIR %s: entry %lld of %lld: %s (page %d cnt %d nr %d start %lld expected %lld)\n",
                    where, (long long)x, (long long)D, bad, page[x], cnt[x], nr[x], (long long)start[x], (long long)acc);
            return FDBCS_E_STATE;
        }
        acc += nr[x];
    }
    if (start[D] != acc || H != acc) {
        fprintf(stderr, "FDBCS_DEBUG_DIR %s: start[D]=%lld H=%lld boundaries %lld\n", where, (long long)start[D],
                (long long)H, (long long)acc);
        return FDBCS_E_STATE;
    }
    return FDBCS_OK;
}

int reset_history(fdbcs* cs, int64_t v) {
    cs->v0 = v;
    cs->cur = 0;
    launch_reset_history(cs->h, cs->cur, cs->sc, cs->stream);
    mirrors_stale(cs);
    launch_dir_finish(cs->h, cs->cur, cs->sc, cs->b, cs->stream);
    int r = sync_state(cs);
    return r ? r : debug_check_dir(cs, "reset");
}


// Lay a host batch view out in one pinned buffer, copy it to the device in one
// transfer and return the device-side view.
struct StageLayout {
    size_t o_snap, o_ro, o_wo, o_ko, o_kl, o_kb, total;
};

StageLayout stage_layout(const fdbcs_batch_view& hv) {
    const int64_t T = hv.txn_count, R = hv.read_count, W = hv.write_count, slots = 2 * (R + W);
    auto al = [](size_t x) { return (x + 15) & ~size_t(15); };
    StageLayout L;
    L.o_snap = 0;
    L.o_ro = al(L.o_snap + 8 * T);
    L.o_wo = al(L.o_ro + 4 * (T + 1));
    L.o_ko = al(L.o_wo + 4 * (T + 1));
    L.o_kl = al(L.o_ko + 8 * slots);
    L.o_kb = al(L.o_kl + 4 * slots);
    L.total = al(L.o_kb + hv.key_bytes_len + 16);
    return L;
}

// Host work over a whole (large) batch split across threads: f(lo, hi) on
// [0, n) in `parts` pieces, the calling thread taking the first.  One thread
// below `serial` items.  FDBCS_HOST_THREADS caps the count (default: 16, the
// GPU box's CPU share, or fewer cores).
template <class F>
void parallel_for(int64_t n, int64_t serial, F f) {
    static const int cap = [] {
        const char* e = getenv("FDBCS_HOST_THREADS");
        const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
        return std::max(1, e ? atoi(e) : std::min(16, hw));
    }();
    const int parts = n < serial ? 1 : (int)std::min<int64_t>(cap, (n + serial - 1) / serial);
    if (parts <= 1) {
        f((int64_t)0, n);
        return;
    }
    std::vector<std::thread> th;
    th.reserve(parts - 1);
    for (int k = 1; k < parts; k++) th.emplace_back([&, k] { f(n * k / parts, n * (k + 1) / parts); });
    f((int64_t)0, n / parts);
    for (auto& t : th) t.join();
}

// (a config-5 batch -- 10^6 transactions, ~0.4 GB laid out -- packs on
// several threads: one memcpy thread moves ~10 GB/s)
void stage_fill(const fdbcs_batch_view& hv, const StageLayout& L, uint8_t* p) {
    const int64_t T = hv.txn_count, slots = 2 * ((int64_t)hv.read_count + hv.write_count);
    struct Piece {
        uint8_t* d;
        const void* s;
        size_t n;
    };
    const Piece pc[6] = {{p + L.o_snap, hv.snapshot, T ? 8 * (size_t)T : 0},
                         {p + L.o_ro, hv.read_off, 4 * (size_t)(T + 1)},
                         {p + L.o_wo, hv.write_off, 4 * (size_t)(T + 1)},
                         {p + L.o_ko, hv.key_off, slots ? 8 * (size_t)slots : 0},
                         {p + L.o_kl, hv.key_len, slots ? 4 * (size_t)slots : 0},
                         {p + L.o_kb, hv.key_bytes, (size_t)hv.key_bytes_len}};
    size_t total = 0;
    for (const Piece& x : pc) total += x.n;
    // the pieces as one byte range [0, total), cut into equal shares
    parallel_for((int64_t)total, 16 << 20, [&](int64_t lo, int64_t hi) {
        size_t o = 0;
        for (const Piece& x : pc) {
            const int64_t a = std::max<int64_t>(lo, (int64_t)o), b = std::min<int64_t>(hi, (int64_t)(o + x.n));
            if (a < b) memcpy(x.d + (a - o), static_cast<const uint8_t*>(x.s) + (a - o), (size_t)(b - a));
            o += x.n;
        }
    });
}

fdbcs_batch_view stage_view(const fdbcs_batch_view& hv, const StageLayout& L, uint8_t* din) {
    fdbcs_batch_view dv = hv;
    dv.snapshot = (const int64_t*)(din + L.o_snap);
    dv.read_off = (const int32_t*)(din + L.o_ro);
    dv.write_off = (const int32_t*)(din + L.o_wo);
    dv.key_off = (const uint64_t*)(din + L.o_ko);
    dv.key_len = (const uint32_t*)(din + L.o_kl);
    dv.key_bytes = din + L.o_kb;
    return dv;
}

int ensure_device_bytes(uint8_t*& p, size_t& cap, size_t need) {
    if (need <= cap) return FDBCS_OK;
    const size_t n = std::max(need, cap * 2);
    dfree(p);
    cap = 0;
    int r;
    if ((r = dalloc(p, (int64_t)n))) return r;
    cap = n;
    return FDBCS_OK;
}

int stage_batch(fdbcs* cs, const fdbcs_batch_view& hv, fdbcs_batch_view& dv) {
    const StageLayout L = stage_layout(hv);
    int r;
    if ((r = ensure_pinned(cs->pin, cs->pin_cap, L.total))) return r;
    if ((r = ensure_device_bytes(cs->din, cs->din_cap, L.total))) return r;
    // the previous batch's H2D must be done before overwriting the pinned buffer
    HIPOK(hipStreamSynchronize(cs->stream));
    stage_fill(hv, L, cs->pin);
    HIPOK(hipMemcpyAsync(cs->din, cs->pin, L.total, hipMemcpyHostToDevice, cs->stream));
    dv = stage_view(hv, L, cs->din);
    return FDBCS_OK;
}

// preconditions checked on the host so that no device state changes on a bad batch
int check_host_view(const fdbcs_batch_view& hv) {
    if (hv.txn_count < 0 || hv.read_count < 0 || hv.write_count < 0) return FDBCS_E_ARG;
    const int64_t nr = (int64_t)hv.read_count + hv.write_count;
    std::atomic<int> key_err{0}, range_err{0};
    parallel_for(nr, 1 << 18, [&](int64_t lo, int64_t hi) {
        for (int64_t i = lo; i < hi; i++) {
            if (hv.key_len[2 * i] > FDBCS_MAX_KEY || hv.key_len[2 * i + 1] > FDBCS_MAX_KEY) {
                key_err.store(1, std::memory_order_relaxed);
                continue;
            }
            if (keycmp(hv.key_bytes + hv.key_off[2 * i], hv.key_len[2 * i], hv.key_bytes + hv.key_off[2 * i + 1],
                       hv.key_len[2 * i + 1]) >= 0)
                range_err.store(1, std::memory_order_relaxed);
        }
    });
    if (key_err.load()) return FDBCS_E_KEY;  // (the key check first, as before)
    return range_err.load() ? FDBCS_E_RANGE : FDBCS_OK;
}

// detectConflicts on a staged device view, verdicts to the host.  The call
// returns once the verdicts are back (the Resolver needs them
// on return); the history update (merge, compaction) is still running and the
// next batch's kernels queue behind it on the stream.  With stage timing on,
// the whole batch is waited for (the stage events).
// staged: a per-transaction batch (its ingest reads the record stream and,
// with a sample attached, rolls the load metrics on the way)
int finish_detect(fdbcs* cs, const fdbcs_batch_view& dv, int64_t now, int64_t new_oldest, uint8_t* verdict,
                  bool staged = false) {
    int r;
    const int64_t T = dv.txn_count;
    const bool early = !cs->timing;
    LmArgs la{};
    const bool live = staged && cs->b.staged.live;
    // (a live batch's kernel rolled already, armed when the batch began)
    const bool roll = staged && cs->lm.owner &&
                      (live ? cs->lv_lm
                            : lm_arm(cs, (uint64_t)dv.read_count + dv.write_count, dv.key_bytes_len, la) == FDBCS_OK);
    cs->lm.rolled = false;
    cs->lm.host_ent = nullptr;
    if ((r = run_batch(cs, dv, now, new_oldest, nullptr, false, early, roll && !live ? &la : nullptr))) return r;
    int64_t count = 0;
    if (early) {
        if ((r = verdict_wait(cs, T, verdict, &count))) return r;
    } else {
        if ((r = ensure_pinned(cs->vpin, cs->vpin_cap, (size_t)T + 1))) return r;
        if (T) HIPOK(hipMemcpyAsync(cs->vpin, cs->b.verdict, (size_t)T, hipMemcpyDeviceToHost, cs->stream));
        if ((r = sync_batch(cs))) return r;
        read_stage_times(cs);
        if (cs->sc_host->last_err) return cs->sc_host->last_err;
        if (T) memcpy(verdict, cs->vpin, (size_t)T);
        count = cs->sc_host->lm_out_count;
    }
    if (roll) {
        cs->lm.rolled = true;
        cs->lm.count = count;
        cs->lm.batch = cs->batches;
    }
    return FDBCS_OK;
}

int detect_host_view(fdbcs* cs, const fdbcs_batch_view& hv, int64_t now, int64_t new_oldest, uint8_t* verdict) {
    int r;
    live_quiesce(cs);
    if (cs->sub_head != cs->sub_tail) return FDBCS_E_ARG;  // (pipelined batches still in flight)
    if ((r = check_host_view(hv))) return r;
    fdbcs_batch_view dv;
    cs->have_last_dv = false;
    cs->last_wbase = 0;
    if ((r = stage_batch(cs, hv, dv))) return r;
    if ((r = finish_detect(cs, dv, now, new_oldest, verdict))) return r;
    cs->last_dv = dv;
    cs->have_last_dv = true;
    return FDBCS_OK;
}

// removalKey from host bytes (synchronous: the host copies are temporaries)
int set_removal_key(fdbcs* cs, const uint8_t* key, uint32_t len) {
    if (len > FDBCS_MAX_KEY) return FDBCS_E_KEY;
    uint64_t rh, rl;
    uint32_t rm;
    encode_host(key, len, rh, rl, rm);
    std::vector<uint8_t> rt(FDBCS_MAX_KEY + 16, 0);
    if (len > 17) memcpy(rt.data(), key + 17, len - 17);
    hipStream_t s = cs->stream;
    HistBufs& h = cs->h;
    HIPOK(hipMemcpyAsync(h.rk_hi, &rh, 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.rk_lo, &rl, 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.rk_meta, &rm, 4, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.rk_tail, rt.data(), len > 17 ? ((len - 17 + 7) & ~7u) : 8, hipMemcpyHostToDevice, s));
    HIPOK(hipStreamSynchronize(s));
    return FDBCS_OK;
}

// key bytes from its (hi, lo, meta) encoding and tail bytes
std::vector<uint8_t> decode_key(uint64_t hi, uint64_t lo, uint32_t meta, const uint8_t* tail) {
    const uint32_t len = meta & LEN_MASK;
    std::vector<uint8_t> k(len);
    for (uint32_t i = 0; i < len; i++) {
        if (i < 8) k[i] = (uint8_t)(hi >> (56 - 8 * i));
        else if (i < 16) k[i] = (uint8_t)(lo >> (56 - 8 * (i - 8)));
        else if (i == 16) k[i] = (uint8_t)(meta >> 24);
        else k[i] = tail[i - 17];
    }
    return k;
}

int check_batch_shape(const fdbcs_batch_view& v) {
    return v.txn_count < 0 || v.read_count < 0 || v.write_count < 0 ? FDBCS_E_ARG : FDBCS_OK;
}

}  // namespace

namespace fdbcs_dev {
int engine_device(const fdbcs* cs) { return cs->device; }

void engine_lm_attach(fdbcs* cs, const void* owner, const uint64_t* seq, uint64_t seed, int64_t units, int64_t opk) {
    live_quiesce(cs);  // (an open live batch rolls for the sample it began with)
    fdbcs::Lm& L = cs->lm;
    L.owner = owner;
    L.seq = seq;
    L.seed = seed;
    L.units = units;
    L.opk = opk;
    L.rolled = false;
}

bool engine_lm_take(fdbcs* cs, const void* owner, uint64_t seq, int64_t opk, LmTake& out) {
    const fdbcs::Lm& L = cs->lm;
    if (!L.rolled || L.owner != owner || L.batch != cs->batches || L.rolled_seq != seq || L.opk != opk) return false;
    if (L.host_ent) out = LmTake{L.count, L.host_ent, L.host_bytes, (size_t)L.count, L.host_nb};  // (the shard's host roll)
    else out = LmTake{L.count, L.ent, L.bytes, L.cap_n, L.cap_b};
    return true;
}
}  // namespace fdbcs_dev

// ============================================================== C ABI ====

extern "C" {

int fdbcs_create(fdbcs** out, int64_t v0, const fdbcs_config* cfg) {
    if (!out) return FDBCS_E_ARG;
    *out = nullptr;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return FDBCS_E_NODEV;
    fdbcs* cs = new (std::nothrow) fdbcs();
    if (!cs) return FDBCS_E_NOMEM;
    int dev = cfg && cfg->device >= 0 ? cfg->device : -1;
    if (dev < 0) {
        if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    }
    cs->device = dev;
    cs->borrow_flags = cfg ? cfg->flags & (FDBCS_BORROW_ALWAYS | FDBCS_BORROW_LARGE) : 0;
    int r = FDBCS_OK;
    auto fail = [&](int code) {
        fdbcs_destroy(cs);
        return code;
    };
    if (hipSetDevice(dev) != hipSuccess) return fail(FDBCS_E_HIP);
    if (hipStreamCreateWithFlags(&cs->stream, hipStreamNonBlocking) != hipSuccess) return fail(FDBCS_E_HIP);
    configure_batch_kernels();
    if ((r = dalloc(cs->sc, 1))) return fail(r);
    if (hipHostMalloc((void**)&cs->sc_host, sizeof(Scalars), hipHostMallocDefault) != hipSuccess)
        return fail(FDBCS_E_NOMEM);
    memset(cs->sc_host, 0, sizeof(Scalars));
    if (hipHostMalloc((void**)&cs->sc_mapped, 2 * sizeof(Scalars), hipHostMallocMapped | hipHostMallocCoherent) !=
            hipSuccess ||
        hipHostGetDevicePointer((void**)&cs->mirror_dev, cs->sc_mapped, 0) != hipSuccess)
        return fail(FDBCS_E_NOMEM);
    memset(cs->sc_mapped, 0, 2 * sizeof(Scalars));
    cs->h.mirror = cs->mirror_dev;
    cs->h.mirror_host = cs->sc_mapped;
    for (int i = 0; i < 2; i++)
        if (hipEventCreateWithFlags(&cs->ev_slot[i], hipEventDisableTiming) != hipSuccess) return fail(FDBCS_E_HIP);
    // Every initialisation goes on the engine's own stream: it is
    // non-blocking, so the legacy null stream (hipMemset, hipMemcpy) does not
    // order against the kernels that follow on it.
    if (hipMemsetAsync(cs->sc, 0, sizeof(Scalars), cs->stream) != hipSuccess) return fail(FDBCS_E_HIP);
    int64_t max_hist = cfg && cfg->max_history > 0 ? cfg->max_history : (1 << 20);
    int64_t pages = std::max<int64_t>(1024, cdiv64(max_hist, FILL) * 2);
    if ((r = alloc_pool(cs, (int32_t)pages))) return fail(r);
    uint64_t tcap = cfg && cfg->tail_arena_bytes > 0 ? (uint64_t)cfg->tail_arena_bytes : (64ull << 20);
    if ((r = dalloc(cs->h.tail_arena, (int64_t)tcap))) return fail(r);
    cs->h.tail_cap = tcap;
    if ((r = dalloc(cs->h.rk_hi, 1)) || (r = dalloc(cs->h.rk_lo, 1)) || (r = dalloc(cs->h.rk_meta, 1)) ||
        (r = dalloc(cs->h.rk_tail, FDBCS_MAX_KEY + 16)))
        return fail(r);
    if (hipMemsetAsync(cs->h.rk_hi, 0, 8, cs->stream) || hipMemsetAsync(cs->h.rk_lo, 0, 8, cs->stream) ||
        hipMemsetAsync(cs->h.rk_meta, 0, 4, cs->stream))
        return fail(FDBCS_E_HIP);
    if ((r = dalloc(cs->h.shard_tails, 2 * (int64_t)SHARD_TAIL_STRIDE)) || (r = dalloc(cs->key_out, 3)) ||
        (r = dalloc(cs->key_out_tail, FDBCS_MAX_KEY + 16)))
        return fail(r);
    if (hipHostMalloc((void**)&cs->rk_stage, 24 + FDBCS_MAX_KEY + 64, hipHostMallocDefault) != hipSuccess)
        return fail(FDBCS_E_NOMEM);
    if (hipMemsetAsync(cs->h.shard_tails, 0, 2 * SHARD_TAIL_STRIDE, cs->stream) != hipSuccess)
        return fail(FDBCS_E_HIP);
    cs->h.shard = ShardBounds{};
    for (int i = 0; i < 8; i++)
        if (hipEventCreate(&cs->ev[i]) != hipSuccess) return fail(FDBCS_E_HIP);
    if (hipEventCreateWithFlags(&cs->ev_verdict, hipEventDisableTiming) != hipSuccess) return fail(FDBCS_E_HIP);
    if ((r = ensure_batch(cs, 1024, 1024, 1024, 1 << 16))) return fail(r);
    if ((r = reset_history(cs, v0))) return fail(r);
    cs->oldest = 0;
    if (hipStreamCreateWithFlags(&cs->copy_stream, hipStreamNonBlocking) != hipSuccess) return fail(FDBCS_E_HIP);
    {
        const char* c = getenv("FDBCS_STAGE_CHUNK");  // bytes per streamed H2D chunk of the per-transaction path
        if ((r = cs->st.configure(cs->stream, cs->copy_stream, c ? strtoull(c, nullptr, 0) : 512 << 10))) return fail(r);
        // the live kernel's shape (kernels.h LiveTune; tests run each)
        if (const char* e = getenv("FDBCS_LIVE_BLOCKS")) cs->lv_tune.blocks = std::min(1024, std::max(2, atoi(e)));
        if (const char* e = getenv("FDBCS_LIVE_SPEC")) cs->lv_tune.spec = atoi(e) != 0;
        if (const char* e = getenv("FDBCS_LIVE_TIMEOUT_US"))
            cs->lv_tune.timeout_ticks = std::max<uint64_t>(1, strtoull(e, nullptr, 0)) * 100;  // (100 MHz)
    }

    *out = cs;
    return FDBCS_OK;
}

int fdbcs_clear(fdbcs* cs, int64_t v) {
    if (cs) live_quiesce(cs);
    if (!cs) return FDBCS_E_ARG;
    return reset_history(cs, v);  // oldestVersion and removalKey are kept (SkipList.cpp:957-959)
}

int fdbcs_set_version(fdbcs* cs, int64_t v) { return fdbcs_clear(cs, v); }

void fdbcs_destroy(fdbcs* cs) {
    if (!cs) return;
    live_quiesce(cs);
    if (cs->stream) hipStreamSynchronize(cs->stream);
    if (cs->lm.owner) sample_unlink(cs->lm.owner, cs);  // (an attached sample forgets this engine)
    lm_release(cs->lm);
    free_batch(cs->b);
    free_pool(cs->h);
    dfree(cs->h.tail_arena);
    dfree(cs->h.rk_hi); dfree(cs->h.rk_lo); dfree(cs->h.rk_meta); dfree(cs->h.rk_tail);
    dfree(cs->h.shard_tails); dfree(cs->key_out); dfree(cs->key_out_tail);
    if (cs->rk_stage) hipHostFree(cs->rk_stage);
    dfree(cs->sc);
    dfree(cs->din);
    if (cs->sc_host) hipHostFree(cs->sc_host);
    if (cs->sc_mapped) hipHostFree(cs->sc_mapped);
    if (cs->pin) hipHostFree(cs->pin);
    if (cs->vpin) hipHostFree(cs->vpin);
    for (auto& S : cs->slot) {
        if (S.pin) hipHostFree(S.pin);
        if (S.vpin) hipHostFree(S.vpin);
        dfree(S.din);
        dfree(S.dverd);
        if (S.copied) hipEventDestroy(S.copied);
        if (S.done) hipEventDestroy(S.done);
    }
    for (int i = 0; i < 8; i++)
        if (cs->ev[i]) hipEventDestroy(cs->ev[i]);
    if (cs->ev_verdict) hipEventDestroy(cs->ev_verdict);
    if (cs->vmap) hipHostFree(cs->vmap);
    cs->st.release();  // (its destructor would otherwise synchronize a destroyed stream)
    if (cs->copy_stream) hipStreamDestroy(cs->copy_stream);
    for (auto e : cs->ev_slot)
        if (e) hipEventDestroy(e);
    if (cs->stream) hipStreamDestroy(cs->stream);
    delete cs;
}

int fdbcs_batch_begin(fdbcs* cs) {
    if (!cs) return FDBCS_E_ARG;
    if (cs->sub_head != cs->sub_tail) return FDBCS_E_STATE;  // (pipelined batches still in flight)
    live_quiesce(cs);  // (a live batch begun and never detected)
    int r;
    // (borrowed batches: stage.h TxnStage::begin; FDBCS_BORROW_LARGE follows
    // the previous batch's size, as the live capacities do)
    const bool borrow = (cs->borrow_flags & FDBCS_BORROW_ALWAYS) ||
                        ((cs->borrow_flags & FDBCS_BORROW_LARGE) && cs->lv_prev_T >= FDBCS_BORROW_MIN_TXNS);
    if ((r = cs->st.begin(borrow))) return r;
    cs->have_last_dv = false;  // (the staged bytes of the last batch are overwritten from here on)
    cs->last_wbase = 0;
    cs->in_batch = true;
    live_begin(cs);
    return FDBCS_OK;
}

// ConflictBatch::addTransaction (SkipList.cpp:979-1008): stage.h.
int fdbcs_batch_add(fdbcs* cs, int64_t read_snapshot, const fdbcs_range* reads, int32_t nreads,
                    const fdbcs_range* writes, int32_t nwrites) {
    if (!cs) return FDBCS_E_ARG;
    if (!cs->in_batch) return FDBCS_E_STATE;
    return cs->st.add(read_snapshot, reads, nreads, writes, nwrites);
}

int32_t fdbcs_batch_txn_count(const fdbcs* cs) { return cs ? (int32_t)cs->st.txns() : 0; }

int64_t fdbcs_batch_refused_txn(const fdbcs* cs) { return cs ? cs->st.refused_at() : -1; }

int fdbcs_batch_skip(fdbcs* cs, int32_t n) {
    if (!cs) return FDBCS_E_ARG;
    if (!cs->in_batch) return FDBCS_E_STATE;
    return cs->st.skip(n);
}

// ConflictBatch::detectConflicts (SkipList.cpp:1163-1208) on the staged batch:
// the staging finishes (last chunk, record offsets, k_unpack builds the batch
// view on the device), the pipeline runs, the verdicts come back.
int fdbcs_batch_detect(fdbcs* cs, int64_t now, int64_t new_oldest, uint8_t* verdict) {
    if (!cs) return FDBCS_E_ARG;
    if (!cs->in_batch) return FDBCS_E_STATE;
    const int64_t T = cs->st.txns();
    if (T && !verdict) return FDBCS_E_ARG;
    cs->in_batch = false;
    cs->have_last_dv = false;
    cs->last_wbase = 0;
    int r;
    fdbcs_batch_view dv;
    if ((r = cs->st.finish(dv, &cs->b.staged))) {
        // (a borrowed batch refused at detect: whatever a live kernel did for it is undone, as a cancel's)
        if (cs->st.began_live()) {
            cs->b.lv_wbase = 0;
            cs->b.lv_nb1 = 0;
            cs->b.staged = StagedBatch{};
            launch_live_reset(cs->b, cs->sc, (int)(cs->sorts & 1), cs->stream);
        }
        return r;
    }
    cs->stage_key_total = cs->st.key_total();
    cs->lv_prev_T = dv.txn_count;  // (the next batch's live capacities)
    cs->lv_prev_R = dv.read_count;
    cs->lv_prev_W = dv.write_count;
    cs->lv_prev_K = cs->st.key_total();
    const int64_t wbase = cs->b.staged.live ? cs->b.lv_wbase : 0;
    r = finish_detect(cs, dv, now, new_oldest, verdict, true);
    cs->stage_key_total = 0;
    cs->b.staged = StagedBatch{};  // (the ingest that reads it was launched)
    cs->b.lv_wbase = 0;            // (every stage of the batch was launched)
    cs->b.lv_nb1 = 0;
    if (r) return r;
    cs->last_dv = dv;
    cs->last_wbase = wbase;
    cs->have_last_dv = true;
    return FDBCS_OK;
}

int fdbcs_batch_detect_packed(fdbcs* cs, const fdbcs_batch_view* hb, int64_t now, int64_t new_oldest,
                              uint8_t* verdict) {
    if (!cs || !hb) return FDBCS_E_ARG;
    if (hb->txn_count && !verdict) return FDBCS_E_ARG;
    return detect_host_view(cs, *hb, now, new_oldest, verdict);
}

int fdbcs_batch_submit_packed(fdbcs* cs, const fdbcs_batch_view* hb, int64_t now, int64_t new_oldest) {
    if (cs) live_quiesce(cs);
    if (cs) cs->have_last_dv = false;
    if (cs) cs->last_wbase = 0;
    if (!cs || !hb || cs->in_batch) return FDBCS_E_ARG;
    if (cs->sub_head - cs->sub_tail >= 2) return FDBCS_E_ARG;  // two in flight: fdbcs_batch_wait first
    const fdbcs_batch_view& hv = *hb;
    int r;
    if ((r = check_host_view(hv))) return r;
    fdbcs::Slot& S = cs->slot[cs->sub_head & 1];
    if (!S.copied && (hipEventCreateWithFlags(&S.copied, hipEventDisableTiming) != hipSuccess ||
                      hipEventCreateWithFlags(&S.done, hipEventDisableTiming) != hipSuccess))
        return FDBCS_E_HIP;
    const StageLayout L = stage_layout(hv);
    const int64_t T = hv.txn_count;
    // (this slot's previous batch was waited for: its buffers are free)
    if ((r = ensure_pinned(S.pin, S.pin_cap, L.total)) || (r = ensure_device_bytes(S.din, S.din_cap, L.total)) ||
        (r = ensure_pinned(S.vpin, S.vpin_cap, (size_t)T + 1)))
        return r;
    if (T + 1 > S.dverd_cap) {
        dfree(S.dverd);
        S.dverd_cap = 0;
        if ((r = dalloc(S.dverd, T + 1))) return r;
        S.dverd_cap = T + 1;
    }
    stage_fill(hv, L, S.pin);  // host packing overlaps the batch in flight
    HIPOK(hipMemcpyAsync(S.din, S.pin, L.total, hipMemcpyHostToDevice, cs->copy_stream));
    HIPOK(hipEventRecord(S.copied, cs->copy_stream));
    HIPOK(hipStreamWaitEvent(cs->stream, S.copied, 0));
    const fdbcs_batch_view dv = stage_view(hv, L, S.din);
    if ((r = run_batch(cs, dv, now, new_oldest, S.dverd, false))) return r;
    if (T) HIPOK(hipMemcpyAsync(S.vpin, S.dverd, (size_t)T, hipMemcpyDeviceToHost, cs->stream));
    HIPOK(hipEventRecord(S.done, cs->stream));
    S.T = T;
    S.mirror = cs->h.mirror_host;
    cs->sub_head++;
    return FDBCS_OK;
}

int fdbcs_batch_wait(fdbcs* cs, uint8_t* verdict) {
    if (cs) live_quiesce(cs);
    if (!cs || cs->sub_tail == cs->sub_head) return FDBCS_E_ARG;
    fdbcs::Slot& S = cs->slot[cs->sub_tail & 1];
    int r;
    cs->sub_tail++;
    if (cs->sub_tail == cs->sub_head) {  // nothing else in flight: adopt the device scalars
        if ((r = sync_batch(cs))) return r;
        if (cs->sc_host->last_err) return cs->sc_host->last_err;
    } else {
        HIPOK(hipEventSynchronize(S.done));
        const int32_t e = (S.mirror ? S.mirror : cs->h.mirror_host)->last_err;  // (this batch's slot)
        if (e) return e;
    }
    if (S.T && verdict) memcpy(verdict, S.vpin, (size_t)S.T);
    return FDBCS_OK;
}

int fdbcs_detect_device(fdbcs* cs, const fdbcs_batch_view* db, int64_t now, int64_t new_oldest,
                        uint8_t* dev_verdict, int sync) {
    if (cs) live_quiesce(cs);
    if (!cs || !db) return FDBCS_E_ARG;
    return run_batch(cs, *db, now, new_oldest, dev_verdict, sync != 0);
}

int64_t fdbcs_history_size(fdbcs* cs) {
    if (cs) live_quiesce(cs);
    if (!cs) return FDBCS_E_ARG;
    int r = sync_state(cs);
    return r ? r : cs->known_H;
}

int64_t fdbcs_header_version(const fdbcs* cs) { return cs ? cs->v0 : 0; }
int64_t fdbcs_oldest_version(const fdbcs* cs) { return cs ? cs->oldest : 0; }

int64_t fdbcs_dump_history(fdbcs* cs, int64_t cap, int64_t* versions, uint32_t* key_len, uint64_t* key_off,
                           uint8_t* key_bytes, uint64_t key_bytes_cap) {
    if (cs) live_quiesce(cs);
    if (!cs) return FDBCS_E_ARG;
    int r;
    if ((r = sync_state(cs))) return r;
    const int64_t H = cs->known_H;
    if (H > cap) return FDBCS_E_CAPACITY;
    if (H == 0) return 0;
    Pool out{};
    if ((r = dalloc(out.hi, H)) || (r = dalloc(out.lo, H)) || (r = dalloc(out.meta, H)) || (r = dalloc(out.ver, H)) ||
        (r = dalloc(out.tail, H))) {
        dfree(out.hi); dfree(out.lo); dfree(out.meta); dfree(out.ver); dfree(out.tail);
        return r;
    }
    launch_gather(cs->h, cs->cur, cs->sc, out, cs->stream);
    std::vector<uint64_t> hi(H), lo(H), tail(H);
    std::vector<uint32_t> meta(H);
    std::vector<uint8_t> arena(cs->h.tail_cap);  // (both halves: survivors may still be in the old one)
    hipMemcpyAsync(hi.data(), out.hi, H * 8, hipMemcpyDeviceToHost, cs->stream);
    hipMemcpyAsync(lo.data(), out.lo, H * 8, hipMemcpyDeviceToHost, cs->stream);
    hipMemcpyAsync(meta.data(), out.meta, H * 4, hipMemcpyDeviceToHost, cs->stream);
    hipMemcpyAsync(versions, out.ver, H * 8, hipMemcpyDeviceToHost, cs->stream);
    hipMemcpyAsync(tail.data(), out.tail, H * 8, hipMemcpyDeviceToHost, cs->stream);
    hipMemcpyAsync(arena.data(), cs->h.tail_arena, cs->h.tail_cap, hipMemcpyDeviceToHost, cs->stream);
    hipError_t e = hipStreamSynchronize(cs->stream);
    dfree(out.hi); dfree(out.lo); dfree(out.meta); dfree(out.ver); dfree(out.tail);
    if (e != hipSuccess) return FDBCS_E_HIP;
    uint64_t off = 0;
    const uint64_t abase = (uint64_t)(uintptr_t)cs->h.tail_arena;
    for (int64_t i = 0; i < H; i++) {
        const uint32_t len = meta[i] & LEN_MASK;
        if (off + len > key_bytes_cap) return FDBCS_E_CAPACITY;
        uint8_t* d = key_bytes + off;
        for (uint32_t k = 0; k < std::min<uint32_t>(len, 17); k++) {
            if (k < 8) d[k] = (uint8_t)(hi[i] >> (56 - 8 * k));
            else if (k < 16) d[k] = (uint8_t)(lo[i] >> (56 - 8 * (k - 8)));
            else d[k] = (uint8_t)(meta[i] >> 24);
        }
        if (len > 17) {
            const uint64_t t = tail[i] - abase;
            if (t + (len - 17) > arena.size()) return FDBCS_E_STATE;
            memcpy(d + 17, arena.data() + t, len - 17);
        }
        key_len[i] = len;
        key_off[i] = off;
        off += len;
    }
    return H;
}

int fdbcs_load_history(fdbcs* cs, int64_t n, const int64_t* versions, const uint32_t* key_len,
                       const uint64_t* key_off, const uint8_t* key_bytes, int64_t v0, int64_t oldest,
                       const uint8_t* removal_key, uint32_t removal_key_len) {
    if (cs) live_quiesce(cs);
    if (!cs || n < 0) return FDBCS_E_ARG;
    if (removal_key_len > FDBCS_MAX_KEY) return FDBCS_E_KEY;
    int r;
    for (int64_t i = 0; i + 1 < n; i++)
        if (keycmp(key_bytes + key_off[i], key_len[i], key_bytes + key_off[i + 1], key_len[i + 1]) >= 0)
            return FDBCS_E_RANGE;
    const int64_t np = std::max<int64_t>(1, cdiv64(n, FILL));
    uint64_t tail_bytes = 0;
    for (int64_t i = 0; i < n; i++)
        if (key_len[i] > 17) tail_bytes += ((uint64_t)key_len[i] - 17 + 7) & ~7ull;
    if ((r = sync_state(cs))) return r;
    if (np + 64 > cs->h.cap_pages) {
        if ((r = grow_pool(cs, 2 * np + 1024))) return r;
    }
    if (tail_bytes + 64 > tail_half_bytes(cs->h.tail_cap) / 2) {  // (loaded into half 0)
        if ((r = grow_tail(cs, 2 * tail_bytes + (1 << 20)))) return r;
    }
    if ((r = ensure_batch(cs, 1024, 1024, 1024, 1 << 16))) return r;
    if ((r = reset_history(cs, v0))) return r;
    HistBufs& h = cs->h;
    const int64_t slots = np * PAGE;
    std::vector<uint64_t> hi(slots, 0), lo(slots, 0), tail(slots, 0);
    std::vector<uint32_t> meta(slots, 0);
    std::vector<int64_t> ver(slots, 0);
    std::vector<uint8_t> arena(tail_bytes + 8, 0);
    std::vector<int32_t> dpage(np), dcnt(np), dnr(np);
    std::vector<uint64_t> hmask((size_t)np * HM_WORDS, 0);
    std::vector<int64_t> dmax(np);
    std::vector<uint64_t> dfhi(np), dflo(np), dftail(np);
    std::vector<uint32_t> dfmeta(np);
    const uint64_t abase = (uint64_t)(uintptr_t)h.tail_arena;
    uint64_t toff = 0;
    for (int64_t p = 0; p < np; p++) {
        const int64_t a = n * p / np, e = n * (p + 1) / np;
        const int pn = (int)(e - a), g = spread_gap(pn);  // pages are written with holes (common.h)
        dpage[p] = (int32_t)p;
        dcnt[p] = spread_used(pn);
        dnr[p] = pn;
        for (int w = 0; w < HM_WORDS; w++) hmask[(size_t)p * HM_WORDS + w] = spread_mask_word(pn, w);
        int64_t mx = INT64_MIN;
        for (int64_t i = a; i < e; i++) {
            const int m = (int)(i - a);
            const int64_t sl = p * PAGE + spread_slot(m, g);
            encode_host(key_bytes + key_off[i], key_len[i], hi[sl], lo[sl], meta[sl]);
            ver[sl] = versions[i];
            mx = std::max(mx, versions[i]);
            if (key_len[i] > 17) {
                const uint32_t t = key_len[i] - 17;
                memcpy(arena.data() + toff, key_bytes + key_off[i] + 17, t);
                tail[sl] = abase + toff;
                toff += (t + 7) & ~7u;
            }
            if (spread_hole_after(m, pn, g)) {  // the hole repeats its predecessor exactly
                hi[sl + 1] = hi[sl]; lo[sl + 1] = lo[sl]; meta[sl + 1] = meta[sl];
                ver[sl + 1] = ver[sl]; tail[sl + 1] = tail[sl];
            }
        }
        dmax[p] = mx;
        const int64_t s0 = p * PAGE;
        dfhi[p] = hi[s0]; dflo[p] = lo[s0]; dfmeta[p] = meta[s0]; dftail[p] = tail[s0];
    }
    hipStream_t s = cs->stream;
    HIPOK(hipMemcpyAsync(h.pool.hi, hi.data(), slots * 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.lo, lo.data(), slots * 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.meta, meta.data(), slots * 4, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.ver, ver.data(), slots * 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.tail, tail.data(), slots * 8, hipMemcpyHostToDevice, s));
    std::vector<uint64_t> pidx(slots / PIDX_STRIDE);
    for (int64_t i = 0; i < (int64_t)pidx.size(); i++) pidx[i] = hi[i * PIDX_STRIDE];
    HIPOK(hipMemcpyAsync(h.pool.pidx, pidx.data(), pidx.size() * 8, hipMemcpyHostToDevice, s));
    if (toff) HIPOK(hipMemcpyAsync(h.tail_arena, arena.data(), toff, hipMemcpyHostToDevice, s));
    Dir& d = h.dir[cs->cur];
    HIPOK(hipMemcpyAsync(d.page, dpage.data(), np * 4, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d.cnt, dcnt.data(), np * 4, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d.nr, dnr.data(), np * 4, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(h.pool.hmask, hmask.data(), hmask.size() * 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemsetAsync(h.pool.pskip, 0xFF, (size_t)np * sizeof(int32_t), s));  // (k_page_px after the directory)
    HIPOK(hipMemcpyAsync(d.maxv, dmax.data(), np * 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d.fhi, dfhi.data(), np * 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d.flo, dflo.data(), np * 8, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d.fmeta, dfmeta.data(), np * 4, hipMemcpyHostToDevice, s));
    HIPOK(hipMemcpyAsync(d.ftail, dftail.data(), np * 8, hipMemcpyHostToDevice, s));
    // free stack: pages [np, cap) ; scalars
    HIPOK(hipStreamSynchronize(s));
    Scalars tmp;
    memset(&tmp, 0, sizeof(tmp));
    tmp.D = (int32_t)np;
    tmp.free_top = 0;
    tmp.tail_used = toff;
    tmp.px_on = toff > 0 || cs->sc_host->px_on;  // (long keys loaded: the prefix skips)
    if (tmp.px_on) h.px_host = true;
    HIPOK(hipMemcpyAsync(cs->sc, &tmp, sizeof(Scalars), hipMemcpyHostToDevice, s));
    launch_push_free(h, 0, (int32_t)np, (int32_t)(h.cap_pages - np), s);
    HIPOK(hipStreamSynchronize(s));
    tmp.free_top = (int32_t)(h.cap_pages - np);
    HIPOK(hipMemcpyAsync(cs->sc, &tmp, sizeof(Scalars), hipMemcpyHostToDevice, s));
    mirrors_stale(cs);
    launch_dir_finish(h, cs->cur, cs->sc, cs->b, s);
    if ((r = set_removal_key(cs, removal_key, removal_key_len))) return r;
    cs->v0 = v0;
    cs->oldest = oldest;
    if ((r = sync_state(cs))) return r;
    return debug_check_dir(cs, "load_history");
}

int32_t fdbcs_removal_key(fdbcs* cs, uint8_t* buf, int32_t cap) {
    if (cs) live_quiesce(cs);
    if (!cs) return FDBCS_E_ARG;
    uint64_t hi = 0, lo = 0;
    uint32_t meta = 0;
    std::vector<uint8_t> t(FDBCS_MAX_KEY + 16);
    hipStreamSynchronize(cs->stream);
    hipMemcpy(&hi, cs->h.rk_hi, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&lo, cs->h.rk_lo, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&meta, cs->h.rk_meta, 4, hipMemcpyDeviceToHost);
    const uint32_t len = meta & LEN_MASK;
    if (len > 17) hipMemcpy(t.data(), cs->h.rk_tail, len - 17, hipMemcpyDeviceToHost);
    std::vector<uint8_t> k(len);
    for (uint32_t i = 0; i < len; i++) {
        if (i < 8) k[i] = (uint8_t)(hi >> (56 - 8 * i));
        else if (i < 16) k[i] = (uint8_t)(lo >> (56 - 8 * (i - 8)));
        else if (i == 16) k[i] = (uint8_t)(meta >> 24);
        else k[i] = t[i - 17];
    }
    if (buf && cap > 0) memcpy(buf, k.data(), std::min<int64_t>(cap, len));
    return (int32_t)len;
}

int fdbcs_enable_stage_timing(fdbcs* cs, int on) {
    if (cs) live_quiesce(cs);
    if (!cs) return FDBCS_E_ARG;
    cs->timing = on != 0;
    return FDBCS_OK;
}

int fdbcs_stage_times(fdbcs* cs, double* out_us, int cap) {
    if (!cs || !out_us) return FDBCS_E_ARG;
    if (!cs->have_times) return 0;
    int n = std::min(cap, 7);
    for (int i = 0; i < n; i++) out_us[i] = cs->stage_us[i];
    return n;
}

int fdbcs_batch_stats(fdbcs* cs, int64_t* out, int cap) {
    if (!cs || !out) return FDBCS_E_ARG;
    int r;
    if ((r = sync_state(cs))) return r;  // (detect returns before the history update ends)
    const Scalars& h = *cs->sc_host;
    const int64_t v[FDBCS_STATS] = {cs->last_T, cs->last_R, cs->last_W, h.n_comb, h.n_aff, h.D, h.H, h.win_np,
                                    h.win_surv, h.n_dep, h.jac_iters, h.ss_resample, h.ss_maxc,
                                    (int64_t)cs->h.tail_cap, (int64_t)h.tail_used, h.tail_half, cs->lv_done,
                                    cs->lv_cancelled, cs->st.live_timeouts()};
    const int n = std::min(cap, (int)FDBCS_STATS);
    for (int i = 0; i < n; i++) out[i] = v[i];
    return n;
}

int fdbcs_debug_prefix_skips(fdbcs* cs, int64_t* out, int cap) {
    if (!cs || !out) return FDBCS_E_ARG;
    int r;
    if ((r = sync_state(cs))) return r;
    const HistBufs& h = cs->h;
    const Dir& d = h.dir[cs->cur];
    const int D = cs->sc_host->D;
    std::vector<int32_t> wsk((size_t)(D + 15) / 16), page(D), pskip(h.cap_pages);
    HIPOK(hipMemcpy(wsk.data(), d.wsk, wsk.size() * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(page.data(), d.page, (size_t)D * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(pskip.data(), h.pool.pskip, (size_t)h.cap_pages * 4, hipMemcpyDeviceToHost));
    int64_t v[3] = {0, 0, 0};
    for (int32_t x : wsk) v[0] += x > 0;
    for (int32_t p : page) {
        v[1] += pskip[p] > 0;
        v[2] += pskip[p] < 0;
    }
    const int n = std::min(cap, 3);
    for (int i = 0; i < n; i++) out[i] = v[i];
    return n;
}

int fdbcs_debug_phases(fdbcs* cs, int64_t* out, int cap) {
    if (cs) live_quiesce(cs);
#ifdef FDBCS_PHASES
    if (!cs || !out) return FDBCS_E_ARG;
    const int n = std::min(cap, 32);
    int r;
    if ((r = sync_state(cs))) return r;
    for (int i = 0; i < n; i++) out[i] = cs->sc_host->ph[i];
    return n;
#else
    (void)cs; (void)out; (void)cap;
    return 0;
#endif
}

void* fdbcs_stream(fdbcs* cs) { return cs ? (void*)cs->stream : nullptr; }

int fdbcs_last_device_batch(fdbcs* cs, fdbcs_batch_view* out) {
    if (cs) live_quiesce(cs);
    if (!cs || !out) return FDBCS_E_ARG;
    if (!cs->have_last_dv) return FDBCS_E_STATE;
    fdbcs_batch_view& v = cs->last_dv;
    const int64_t R2 = 2 * (int64_t)v.read_count, n = 2 * (int64_t)v.write_count;
    if (cs->last_wbase && cs->last_wbase != R2 && n) {
        // a live batch's view has its writes after a gap (BatchBufs::lv_wbase):
        // moved down to 2R once, through a scratch copy (the two ranges overlap)
        void* tmp = nullptr;
        HIPOK(hipMalloc(&tmp, (size_t)n * 12));
        uint64_t* koff = const_cast<uint64_t*>(v.key_off);
        uint32_t* klen = const_cast<uint32_t*>(v.key_len);
        uint64_t* t_off = static_cast<uint64_t*>(tmp);
        uint32_t* t_len = reinterpret_cast<uint32_t*>(t_off + n);
        hipStream_t s = cs->stream;
        hipError_t e = hipMemcpyAsync(t_off, koff + cs->last_wbase, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(t_len, klen + cs->last_wbase, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(koff + R2, t_off, (size_t)n * 8, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipMemcpyAsync(klen + R2, t_len, (size_t)n * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipStreamSynchronize(s);
        hipFree(tmp);
        HIPOK(e);
    }
    cs->last_wbase = 0;
    *out = v;
    return FDBCS_OK;
}

const char* fdbcs_strerror(int status) {
    switch (status) {
        case FDBCS_OK: return "ok";
        case FDBCS_E_HIP: return hipGetErrorString(last_hip_error());
        case FDBCS_E_NOMEM: return "out of memory";
        case FDBCS_E_RANGE: return "conflict range with begin >= end";
        case FDBCS_E_STATE: return "call out of order";
        case FDBCS_E_ARG: return "bad argument";
        case FDBCS_E_KEY: return "key longer than FDBCS_MAX_KEY";
        case FDBCS_E_NODEV: return "no HIP device";
        case FDBCS_E_CAPACITY: return "device capacity exceeded";
        default: return "unknown status";
    }
}

const char* fdbcs_version(void) { return "fdbcs gfx950 0.1.0"; }

}  // extern "C"

// ===================================================== exact sharded mode ====
// SURVEY.md §8e protocol A: every GPU holds the history of one key range,
// receives the whole batch, and the host exchanges between the phases.

int fdbcs_set_shard(fdbcs* cs, const uint8_t* lo, uint32_t lo_len, int has_lo, const uint8_t* hi, uint32_t hi_len,
                    int has_hi) {
    if (cs) live_quiesce(cs);
    if (!cs || lo_len > FDBCS_MAX_KEY || hi_len > FDBCS_MAX_KEY) return FDBCS_E_ARG;
    ShardBounds sb{};
    sb.has_lo = has_lo != 0;
    sb.has_hi = has_hi != 0;
    const uint8_t* src[2] = {lo, hi};
    const uint32_t len[2] = {lo_len, hi_len};
    Key* dst[2] = {&sb.lo, &sb.hi};
    for (int k = 0; k < 2; k++) {
        uint32_t m;
        encode_host(src[k], len[k], dst[k]->hi, dst[k]->lo, m);
        dst[k]->meta = m;
        uint8_t* t = cs->h.shard_tails + (size_t)k * SHARD_TAIL_STRIDE;
        dst[k]->tail = len[k] > 17 ? t : nullptr;
        if (len[k] > 17) {
            std::vector<uint8_t> buf(((len[k] - 17 + 7) & ~7u), 0);
            memcpy(buf.data(), src[k] + 17, len[k] - 17);
            HIPOK(hipMemcpyAsync(t, buf.data(), buf.size(), hipMemcpyHostToDevice, cs->stream));  // (engine stream)
            HIPOK(hipStreamSynchronize(cs->stream));
        }
    }
    cs->h.shard = sb;
    return FDBCS_OK;
}

int fdbcs_shard_check(fdbcs* cs, const fdbcs_batch_view* db, int64_t now, int64_t new_oldest, int64_t carry_in,
                      uint8_t* dev_hist) {
    if (cs) live_quiesce(cs);
    if (cs) mirrors_stale(cs);  // (refresh_state: the mirror follows run_batch only)
    (void)now;
    (void)new_oldest;
    if (!cs || !db) return FDBCS_E_ARG;
    cs->batches++;
    const fdbcs_batch_view& v = *db;
    int r;
    if ((r = check_batch_shape(v))) return r;
    cs->have_last_dv = false;
    cs->last_wbase = 0;
    if ((r = ensure_batch(cs, v.txn_count, v.read_count, v.write_count, std::max<uint64_t>(v.key_bytes_len, cs->stage_key_total)))) return r;
    if ((r = ensure_history(cs, v.write_count, std::max<uint64_t>(v.key_bytes_len, cs->stage_key_total)))) return r;
    cs->last_T = v.txn_count;
    cs->last_R = v.read_count;
    cs->last_W = v.write_count;
    cs->v0 = carry_in;
    BatchBufs& b = cs->b;
    hipStream_t s = cs->stream;
    const bool scatter = cs->have_quantiles && !b.large;
    // FDBCS_DEBUG_SYNC: wait after each stage and name the one that failed (fault hunting)
    static const bool dbg = getenv("FDBCS_DEBUG_SYNC") != nullptr;
    auto stage_ok = [&](const char* what) {
        if (!dbg) return FDBCS_OK;
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            fprintf(stderr, "fdbcs debug: %s failed: %s (T=%d R=%d W=%d D=%d cap=%d)\n", what, hipGetErrorString(e),
                    v.txn_count, v.read_count, v.write_count, (int)cs->known_D, cs->h.cap_dir);
            return FDBCS_E_HIP;
        }
        return FDBCS_OK;
    };
    launch_ingest(v, cs->oldest, b, cs->sc, scatter, (int)(cs->sorts & 1), cs->h.dir[cs->cur], s,
                  (cs->h.shard.has_lo | cs->h.shard.has_hi) != 0);
    if ((r = stage_ok("ingest"))) return r;
    if (launch_sort_ranges(v, b, cs->sc, !cs->have_quantiles, (int)(cs->sorts & 1), scatter, s, &cs->h, cs->cur,
                           carry_in)) {
        cs->sorts++;
        cs->have_quantiles = true;
    }
    if ((r = stage_ok("sort"))) return r;
    if ((r = edges_read_check(cs, v, carry_in))) return r;
    if ((r = stage_ok("read check"))) return r;
    if (dev_hist) launch_flags_out(b, v.txn_count, dev_hist, s);
    // the edge count rides the sync below (fdbcs_shard_edge_count reads it without another round trip)
    HIPOK(hipMemcpyAsync(&cs->sc_host->edges_total, &cs->sc->edges_total, sizeof(int32_t), hipMemcpyDeviceToHost,
                         s));
    HIPOK(hipStreamSynchronize(s));
    cs->edges_known = true;
    return FDBCS_OK;
}

int fdbcs_shard_apply(fdbcs* cs, const fdbcs_batch_view* db, int64_t now, int64_t new_oldest, int64_t carry_in,
                      const uint8_t* removal_key, int32_t removal_key_len, const uint8_t* dev_hist,
                      uint8_t* dev_verdict, int64_t* info) {
    if (cs) live_quiesce(cs);
    if (cs) mirrors_stale(cs);  // (refresh_state: the mirror follows run_batch only)
    if (!cs || !db || !info || removal_key_len > FDBCS_MAX_KEY) return FDBCS_E_ARG;
    cs->edges_known = false;
    const fdbcs_batch_view& v = *db;
    BatchBufs& b = cs->b;
    hipStream_t s = cs->stream;
    int r;
    cs->v0 = carry_in;
    if (removal_key_len >= 0) {  // the previous compaction's removalKey, staged through pinned memory
        HistBufs& h = cs->h;
        uint8_t* st = cs->rk_stage;
        uint64_t rh, rl;
        uint32_t rm;
        encode_host(removal_key, (uint32_t)removal_key_len, rh, rl, rm);
        memcpy(st, &rh, 8);
        memcpy(st + 8, &rl, 8);
        memcpy(st + 16, &rm, 4);
        const uint32_t tl = removal_key_len > 17 ? (uint32_t)removal_key_len - 17 : 0;
        if (tl) memcpy(st + 24, removal_key + 17, tl);
        HIPOK(hipMemcpyAsync(h.rk_hi, st, 8, hipMemcpyHostToDevice, s));
        HIPOK(hipMemcpyAsync(h.rk_lo, st + 8, 8, hipMemcpyHostToDevice, s));
        HIPOK(hipMemcpyAsync(h.rk_meta, st + 16, 4, hipMemcpyHostToDevice, s));
        if (tl) HIPOK(hipMemcpyAsync(h.rk_tail, st + 24, (tl + 7) & ~7u, hipMemcpyHostToDevice, s));
    }
    if (dev_hist) launch_flags_in(b, v.txn_count, dev_hist, s);
    launch_decide(v, b, cs->sc, dev_verdict ? dev_verdict : b.verdict, s);
    const bool compact = new_oldest > cs->oldest;
    launch_merge(v, b, cs->h, cs->cur, cs->sc, now, carry_in, !compact, s);
    cs->cur ^= 1;
    if ((r = compact ? sync_state(cs) : sync_batch(cs))) return r;
    const Scalars& h = *cs->sc_host;
    info[0] = h.H;
    info[1] = compact ? h.win_g0 : -1;
    info[2] = h.last_ver;
    info[3] = (cs->h.shard.has_lo | cs->h.shard.has_hi) ? h.n_comb_own : h.n_comb;  // (one shard: all of them)
    return h.last_err ? h.last_err : (compact ? h.err : 0);
}

static constexpr uint32_t RK_TAIL_FAST = 256;  // tail bytes fetched with the key's fixed part

int fdbcs_shard_set_protocol(fdbcs* cs, int sparse_edges) {
    if (!cs || cs->in_batch) return FDBCS_E_ARG;
    cs->sparse_edges = sparse_edges != 0;
    return FDBCS_OK;
}

int64_t fdbcs_shard_edge_count(fdbcs* cs) {
    if (cs) live_quiesce(cs);
    if (!cs) return FDBCS_E_ARG;
    if (cs->edges_known) return cs->sc_host->edges_total;  // (copied by fdbcs_shard_check)
    int32_t n = 0;
    HIPOK(hipMemcpyAsync(&n, &cs->sc->edges_total, sizeof(n), hipMemcpyDeviceToHost, cs->stream));
    HIPOK(hipStreamSynchronize(cs->stream));
    return n;
}

int fdbcs_shard_get_edges(fdbcs* cs, int32_t* dev_et, int32_t* dev_eu, int64_t n) {
    if (cs) live_quiesce(cs);
    if (!cs || n < 0 || n > cs->b.edge_cap || (n && (!dev_et || !dev_eu))) return FDBCS_E_ARG;
    if (n) {
        HIPOK(hipMemcpyAsync(dev_et, cs->b.et, (size_t)n * 4, hipMemcpyDeviceToDevice, cs->stream));
        HIPOK(hipMemcpyAsync(dev_eu, cs->b.eu, (size_t)n * 4, hipMemcpyDeviceToDevice, cs->stream));
    }
    HIPOK(hipStreamSynchronize(cs->stream));
    return FDBCS_OK;
}

int fdbcs_shard_set_edges(fdbcs* cs, const int32_t* dev_et, const int32_t* dev_eu, int64_t n) {
    if (cs) live_quiesce(cs);
    if (!cs || n < 0 || n > INT32_MAX || (n && (!dev_et || !dev_eu))) return FDBCS_E_ARG;
    cs->edges_known = false;
    BatchBufs& b = cs->b;
    if (b.rounds) return FDBCS_E_ARG;  // (protocol B only: fdbcs_shard_set_protocol)
    int r;
    if (n > b.edge_cap && (r = grow_edges(b, n + n / 4 + 1024))) return r;
    launch_set_edges(b, cs->sc, (int)cs->last_T, dev_et, dev_eu, n, cs->stream);
    return FDBCS_OK;
}

int fdbcs_shard_compact(fdbcs* cs, int64_t a, int64_t b, int keep_first, int64_t prev_version, int64_t new_oldest,
                        int64_t key_index, uint8_t* key_buf, int32_t key_cap, int64_t* info) {
    if (cs) live_quiesce(cs);
    if (cs) mirrors_stale(cs);  // (refresh_state: the mirror follows run_batch only)
    // (the window lies in the history the last apply left: known_H, synchronized there)
    if (!cs || !info || a < 0 || b < a || b > cs->known_H || key_index >= cs->known_H) return FDBCS_E_ARG;
    hipStream_t s = cs->stream;
    static const bool dbg = getenv("FDBCS_DEBUG_SYNC") != nullptr;  // (fault hunting: name the failing step)
    auto step_ok = [&](const char* what) {
        if (!dbg) return FDBCS_OK;
        const hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            fprintf(stderr, "fdbcs debug: shard_compact %s failed: %s (a=%lld b=%lld H=%lld D=%d key=%lld win_cap=%d)\n",
                    what, hipGetErrorString(e), (long long)a, (long long)b, (long long)cs->known_H, (int)cs->known_D,
                    (long long)key_index, (int)cs->b.win_cap_pages);
            return FDBCS_E_HIP;
        }
        return FDBCS_OK;
    };
    int r;
    if (key_index >= 0) {  // the boundary that becomes removalKey, read before the compaction moves it
        launch_key_at(cs->h, cs->cur, cs->sc, key_index, cs->key_out, cs->key_out_tail, s);
        if ((r = step_ok("key_at"))) return r;
        HIPOK(hipMemcpyAsync(cs->rk_stage, cs->key_out, 24, hipMemcpyDeviceToHost, s));
        HIPOK(hipMemcpyAsync(cs->rk_stage + 24, cs->key_out_tail, RK_TAIL_FAST, hipMemcpyDeviceToHost, s));
    }
    const WinExplicit w{a, b, keep_first, prev_version};
    launch_compact(cs->b, cs->h, cs->cur, cs->sc, new_oldest, s, &w);
    if ((r = step_ok("window"))) return r;
    cs->cur ^= 1;
    if (new_oldest > cs->oldest) cs->oldest = new_oldest;
    if ((r = sync_batch(cs))) return r;
    info[0] = cs->sc_host->H;
    info[1] = cs->sc_host->last_ver;
    info[2] = -1;
    if (key_index >= 0) {
        uint64_t k3[3];
        memcpy(k3, cs->rk_stage, 24);
        const uint32_t len = (uint32_t)k3[2] & LEN_MASK;
        if (len > 17 + RK_TAIL_FAST)  // a long key: the rest of its tail
            HIPOK(hipMemcpy(cs->rk_stage + 24 + RK_TAIL_FAST, cs->key_out_tail + RK_TAIL_FAST,
                            len - 17 - RK_TAIL_FAST, hipMemcpyDeviceToHost));
        const std::vector<uint8_t> k = decode_key(k3[0], k3[1], (uint32_t)k3[2], cs->rk_stage + 24);
        info[2] = (int64_t)k.size();
        if (key_buf && key_cap > 0) memcpy(key_buf, k.data(), std::min<size_t>((size_t)key_cap, k.size()));
    }
    return cs->sc_host->last_err;
}

// ============================================= exact sharded resolver ====
// fdbcs_sharded: one Resolver over G GPUs (SURVEY.md §8e protocol A) behind
// the C ABI.  Rank g's engine holds the keys [bound[g-1], bound[g]); every
// rank receives the whole batch.  Per batch, all on the engine's stream:
//   check (history read check clipped to the shard, carry-in from the
//   device) -> exchange 1: MAX all-reduce of [G slots | T abort flags] ->
//   k_sh_carry -> the decision (identical on every rank; verdicts to
//   host-mapped memory) -> combine -> this shard's merge -> exchange 2:
//   all-gather of (H, g0, last, own begins) -> k_sh_plan (compaction part,
//   next removalKey's owner, next check's carry-in) -> compaction ->
//   k_sh_slot_out for the next exchange 1.
// The host waits once per batch, for the verdicts.  Exchanges: RCCL on the
// stream (one GPU per rank), or host callbacks (fdbcs_comm_ops: tests, gloo).
#include <rccl/rccl.h>

struct fdbcs_sharded {
    fdbcs* cs = nullptr;
    int rank = 0, world = 1;
    int64_t v0 = 0;
    ncclComm_t comm = nullptr;
    fdbcs_comm_ops ops{};
    bool host_ops = false;
    uint8_t* x1 = nullptr;      // device: [G slots | T flags]
    int64_t x1_cap = 0;
    int64_t* x2 = nullptr;      // device: [SH_WORDS send | G x SH_WORDS gathered]
    uint8_t* hx = nullptr;      // pinned staging of the host-callback exchanges
    size_t hx_cap = 0;
    bool in_batch = false;
    // protocol B (fdbcs_sharded_set_protocol)
    int proto = FDBCS_PROTOCOL_A;
    bool presplit = false;                 // the caller's adds carry only this rank's ranges
    std::vector<uint8_t> lo, hi;           // this rank's keys [lo, hi) (host copies, for the add filter)
    bool has_lo = false, has_hi = false;
    std::vector<fdbcs_range> keep;         // the add filter's output
    int32_t* ebuf = nullptr;               // device: [send 2M | recv G x 2M | readers E | writers E]
    int64_t ebuf_cap = 0;                  // (int32 elements)
    int64_t ecap = 4096;                   // edge pairs per shard in the exchange (grows on a short batch)
    int64_t ecap0 = 4096;                  // the floor it decays back to (FDBCS_TEST_SH_ECAP in tests)
    int64_t retries = 0;                   // batches whose exchange was short and ran again (stats)
    // (one burst used to raise every later batch's all-gather for
    // good) the largest shard count of each of the last ECAP_WINDOW batches,
    // which every rank reads from its own verdicts -- the same values on
    // every rank, so every rank resizes at the same batch
    static constexpr int ECAP_WINDOW_MAX = 64;
    int ecap_window = 32;
    int64_t need_ring[ECAP_WINDOW_MAX] = {};
    int64_t need_seen = 0;                 // batches recorded since the last resize
    int64_t last_max = 0;                  // the last batch's largest shard count (stats)
    int64_t shrinks = 0;                   // (stats)
    std::atomic<bool> aborted{false};      // fdbcs_sharded_abort (any thread)
    // The communicator is touched by the rank's own thread (init, enqueues,
    // progress polls) and by fdbcs_sharded_abort from another one: every use
    // holds comm_mu, and an aborted communicator (freed by ncclCommAbort) is
    // marked dead instead of being cleared under the owner's feet.
    std::mutex comm_mu;
    bool comm_dead = false;                // (guarded by comm_mu)
    // A load sample attached to this rank's engine (the Resolver attaches to
    // conflictSetDevice = rank 0's): under protocol B the rank keeps only the
    // ranges on its keys, so its ingest cannot roll the batch as one resolver
    // would (and sh_run's ingest does not roll under A either).  The adds roll
    // every range of every transaction on the host instead -- the Resolver's
    // order (writes, then reads), positions over the whole batch
    // (Resolver.actor.cpp:146-151) -- so the sample is the one-GPU sample
    // exactly (fdbcs_sharded_batch_add).  Not with FDBCS_SHARD_PRESPLIT (the
    // adds never see the whole transaction): the sample then covers the
    // rank's share.
    bool lm_host = false;
    uint64_t lm_seq = 0, lm_pos = 0;
    std::vector<LmEntry> lm_ent;
    std::vector<uint8_t> lm_bytes;
};

namespace {

size_t sh_slot_bytes(const fdbcs_sharded* sh) { return (size_t)sh->world * SH_WORDS * 8; }

// One RCCL call on the rank's communicator.  Communicators are created
// non-blocking (fdbcs_sharded_comm_init), so a call may return ncclInProgress
// (the initialisation, a lazy connection); the rank then polls the
// communicator -- under comm_mu, re-checking `aborted` -- so that
// fdbcs_sharded_abort can end a wait for a peer that never joins.
template <class F>
int sh_nccl(fdbcs_sharded* sh, F call) {
    ncclResult_t res;
    {
        std::lock_guard<std::mutex> lk(sh->comm_mu);
        if (sh->aborted.load(std::memory_order_acquire) || !sh->comm || sh->comm_dead) return FDBCS_E_STATE;
        res = call(sh->comm);
    }
    for (int it = 0; res == ncclInProgress; it++) {
        if (it < 4096) _mm_pause();
        else std::this_thread::sleep_for(std::chrono::microseconds(50));
        std::lock_guard<std::mutex> lk(sh->comm_mu);
        if (sh->aborted.load(std::memory_order_acquire) || sh->comm_dead) return FDBCS_E_STATE;
        if (ncclCommGetAsyncError(sh->comm, &res) != ncclSuccess) return FDBCS_E_HIP;
    }
    return res == ncclSuccess ? FDBCS_OK : FDBCS_E_HIP;
}

// a non-blocking communicator of `world` ranks (polled to completion by sh_nccl)
int sh_comm_init(fdbcs_sharded* sh, const uint8_t* comm_id) {
    ncclUniqueId u;
    memcpy(u.internal, comm_id, FDBCS_COMM_ID_BYTES);
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    {
        std::lock_guard<std::mutex> lk(sh->comm_mu);
        if (sh->aborted.load(std::memory_order_acquire) || sh->comm) return FDBCS_E_STATE;
        const ncclResult_t res = ncclCommInitRankConfig(&sh->comm, sh->world, u, sh->rank, &cfg);
        if (res != ncclSuccess && res != ncclInProgress) {
            sh->comm = nullptr;
            return FDBCS_E_HIP;
        }
    }
    ncclResult_t st = ncclInProgress;
    return sh_nccl(sh, [&](ncclComm_t c) {
        if (ncclCommGetAsyncError(c, &st) != ncclSuccess) return ncclInternalError;
        return st;
    });
}

int sh_allreduce_max(fdbcs_sharded* sh, uint8_t* dev, size_t n) {
    hipStream_t s = sh->cs->stream;
    if (sh->aborted || (!sh->host_ops && !sh->comm)) return FDBCS_E_STATE;
    if (!sh->host_ops)
        return sh_nccl(sh, [&](ncclComm_t c) { return ncclAllReduce(dev, dev, n, ncclUint8, ncclMax, c, s); });
    int r;
    if ((r = ensure_pinned(sh->hx, sh->hx_cap, n))) return r;
    HIPOK(hipMemcpyAsync(sh->hx, dev, n, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    if (sh->ops.allreduce_max_u8(sh->ops.ctx, sh->hx, n)) return FDBCS_E_HIP;
    HIPOK(hipMemcpyAsync(dev, sh->hx, n, hipMemcpyHostToDevice, s));
    HIPOK(hipStreamSynchronize(s));  // (hx is reused by the next exchange)
    return FDBCS_OK;
}

int sh_allgather(fdbcs_sharded* sh, const void* dev_send, void* dev_recv, size_t n = SH_WORDS * 8) {
    hipStream_t s = sh->cs->stream;
    if (sh->aborted || (!sh->host_ops && !sh->comm)) return FDBCS_E_STATE;
    if (!sh->host_ops)
        return sh_nccl(sh, [&](ncclComm_t c) { return ncclAllGather(dev_send, dev_recv, n, ncclUint8, c, s); });
    int r;
    if ((r = ensure_pinned(sh->hx, sh->hx_cap, n * (sh->world + 1)))) return r;
    HIPOK(hipMemcpyAsync(sh->hx, dev_send, n, hipMemcpyDeviceToHost, s));
    HIPOK(hipStreamSynchronize(s));
    if (sh->ops.allgather_u8(sh->ops.ctx, sh->hx, sh->hx + n, n)) return FDBCS_E_HIP;
    HIPOK(hipMemcpyAsync(dev_recv, sh->hx + n, n * (size_t)sh->world, hipMemcpyHostToDevice, s));
    HIPOK(hipStreamSynchronize(s));
    return FDBCS_OK;
}

// Protocol B, after the check: exchange 1 (the abort flags and slots, which
// carry every shard's edge count) and then the union of the shards' overlap
// edges as this shard's list -- at a fixed capacity of sh->ecap pairs per
// shard, so the host enqueues the whole batch without reading anything
// (the counts used to be polled from host-mapped memory
// mid-batch to size the all-gather).  When some shard's list does not fit
// (or overflowed its own buffer) k_sh_edges_cat_fixed marks the batch
// E_SH_RETRY: the decision's verdicts say so, every history stage after it
// leaves the history as it was, and sh_run searches again and repeats the
// exchange with a larger capacity -- on every rank alike, since all of them
// see the same gathered counts.
int sh_exchange_b(fdbcs_sharded* sh, const fdbcs_batch_view& v, size_t slots, uint8_t* flags) {
    fdbcs* cs = sh->cs;
    BatchBufs& b = cs->b;
    hipStream_t s = cs->stream;
    const int64_t T = v.txn_count;
    int64_t* sl = reinterpret_cast<int64_t*>(sh->x1);
    int r;
    const int64_t M = sh->ecap, G = sh->world;
    const int64_t need = 2 * M * (2 * G + 1);  // send | recv G x | concatenated G x, int32 pairs
    if (need > sh->ebuf_cap) {
        HIPOK(hipStreamSynchronize(s));  // (the previous batch's exchange may still read it)
        if (sh->ebuf) hipFree(sh->ebuf);
        sh->ebuf = nullptr;
        sh->ebuf_cap = 0;
        if ((r = dalloc(sh->ebuf, need))) return r;
        sh->ebuf_cap = need;
    }
    // (the gathered list's home is this shard's list: sized before its search,
    // sh_run -- growing it here would drop the edges just found)
    if (M * G > b.edge_cap) return FDBCS_E_STATE;
    launch_sh_edges_count(cs->sc, sl, sh->rank, sh->world, b.edge_cap, s);
    if (T) launch_flags_out(b, (int)T, flags, s);
    if ((r = sh_allreduce_max(sh, sh->x1, slots + (size_t)T))) return r;
    int32_t* send = sh->ebuf;
    int32_t* recv = send + 2 * M;
    int32_t* cat = recv + 2 * M * G;
    // Host collectives (rehearsals, tests) hold the gathered counts on the
    // host already (sh_allreduce_max synchronizes): with no edge anywhere the
    // lists' all-gather -- another synchronous host round -- is skipped and
    // the received lists are zeros, as a gather of empty lists would leave them.
    bool any = true;
    if (sh->host_ops) {
        const int64_t* hs = reinterpret_cast<const int64_t*>(sh->hx);
        any = false;
        for (int64_t g = 0; g < G; g++) any |= hs[g * SH_WORDS + 2] != 0 || hs[g * SH_WORDS + 3] != 0;
    }
    if (any) {
        launch_sh_edges_pack(b, cs->sc, M, send, s);
        if ((r = sh_allgather(sh, send, recv, (size_t)(2 * M) * 4))) return r;
    } else {
        HIPOK(hipMemsetAsync(recv, 0, (size_t)(2 * M * G) * sizeof(int32_t), s));
    }
    launch_sh_edges_cat_fixed(recv, sl, (int)G, M, cat, cat + M * G, cs->sc, s);
    launch_set_edges(b, cs->sc, (int)T, cat, cat + M * G, -(M * G), s);
    return FDBCS_OK;
}

// Protocol B's exchange capacity follows the recent batches down again: once
// a whole window of batches (sh->ecap_window, each recorded after its
// verdicts) needed at most half of it, it drops to that need plus a quarter
// and min(1024, ecap0) (never below ecap0), and the exchange
// buffer is released so that it is sized again for the new capacity.
void sh_ecap_decay(fdbcs_sharded* sh) {
    sh->need_ring[sh->need_seen % sh->ecap_window] = sh->last_max;
    if (++sh->need_seen < sh->ecap_window || sh->ecap <= sh->ecap0) return;
    int64_t mx = 0;
    for (int i = 0; i < sh->ecap_window; i++) mx = std::max(mx, sh->need_ring[i]);
    const int64_t target = std::max(sh->ecap0, mx + mx / 4 + std::min<int64_t>(1024, sh->ecap0));
    if (2 * target > sh->ecap) return;
    GROWLOG("sharded edge exchange capacity %lld -> %lld\n", (long long)sh->ecap, (long long)target);
    sh->ecap = target;
    sh->shrinks++;
    sh->need_seen = 0;
    if (sh->ebuf) {  // (the last batch's exchange may still read it)
        (void)hipStreamSynchronize(sh->cs->stream);
        hipFree(sh->ebuf);
        sh->ebuf = nullptr;
        sh->ebuf_cap = 0;
    }
}

// one batch of the sharded resolver on the device-resident view v
int sh_run(fdbcs_sharded* sh, const fdbcs_batch_view& v, int64_t now, int64_t new_oldest, uint8_t* verdict) {
    static const bool sh_mirror = !getenv("FDBCS_SH_MIRROR") || atoi(getenv("FDBCS_SH_MIRROR"));  // (A/B; 0: sync)
    if (!sh_mirror) mirrors_stale(sh->cs);
    fdbcs* cs = sh->cs;
    cs->batches++;
    int r;
    if ((r = check_batch_shape(v))) return r;
    const int64_t T = v.txn_count, R = v.read_count, W = v.write_count;
    if (T && !verdict) return FDBCS_E_ARG;
    cs->have_last_dv = false;
    cs->last_wbase = 0;
    cs->edges_known = false;
    if ((r = ensure_batch(cs, T, R, W, std::max<uint64_t>(v.key_bytes_len, cs->stage_key_total)))) return r;
    if ((r = ensure_history(cs, W, std::max<uint64_t>(v.key_bytes_len, cs->stage_key_total)))) return r;
    const size_t slots = sh_slot_bytes(sh), nx = slots + (size_t)std::max<int64_t>(T, 1);
    if ((int64_t)nx > sh->x1_cap) {  // (the slots written after the last batch are kept)
        uint8_t* nb = nullptr;
        if (hipMalloc((void**)&nb, 2 * nx) != hipSuccess) return FDBCS_E_NOMEM;
        HIPOK(hipMemsetAsync(nb, 0, 2 * nx, cs->stream));
        if (sh->x1) {
            HIPOK(hipMemcpyAsync(nb, sh->x1, slots, hipMemcpyDeviceToDevice, cs->stream));
            HIPOK(hipStreamSynchronize(cs->stream));
            hipFree(sh->x1);
        }
        sh->x1 = nb;
        sh->x1_cap = (int64_t)(2 * nx);
    }
    if (T + 64 > (int64_t)cs->vmap_cap) {
        if (cs->vmap) hipHostFree(cs->vmap);
        cs->vmap = cs->vmap_dev = nullptr;
        cs->vmap_cap = 0;
        const size_t n = (size_t)T + 64 + 4096;
        if (hipHostMalloc((void**)&cs->vmap, n, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
            return FDBCS_E_NOMEM;
        memset(cs->vmap, 0, n);
        HIPOK(hipHostGetDevicePointer((void**)&cs->vmap_dev, cs->vmap, 0));
        cs->vmap_cap = n;
        cs->vseq = 0;
    }
    cs->last_T = T;
    cs->last_R = R;
    cs->last_W = W;
    BatchBufs& b = cs->b;
    HistBufs& h = cs->h;
    hipStream_t s = cs->stream;
    Scalars* sc = cs->sc;
    uint8_t* flags = sh->x1 + slots;
    // this batch's mirror slot (refresh_state, as run_batch's): the batch-ending
    // kernel of the last attempt publishes there, the event follows the attempt
    const int mslot = (int)(cs->batches & 1);
    h.mirror = cs->mirror_dev + mslot;
    h.mirror_host = cs->sc_mapped + mslot;
    // 1-2: the check, clipped to this shard (carry-in: sc->carry_check)
    const bool scatter = cs->have_quantiles && !b.large;
    launch_ingest(v, cs->oldest, b, sc, scatter, (int)(cs->sorts & 1), cs->h.dir[cs->cur], s,
                  (cs->h.shard.has_lo | cs->h.shard.has_hi) != 0);
    if (launch_sort_ranges(v, b, sc, !cs->have_quantiles, (int)(cs->sorts & 1), scatter, s, &cs->h, cs->cur, sh->v0,
                           sort_guard(cs))) {
        cs->sorts++;
        cs->have_quantiles = true;
    }
    const int64_t oldest0 = cs->oldest;
    if (sh->proto == FDBCS_PROTOCOL_B) {
        // (the list the search fills also receives the gathered edges: sized first)
        if (sh->ecap * sh->world > b.edge_cap && (r = grow_edges(b, sh->ecap * sh->world))) return r;
        launch_edges_read_check(v, b, cs->h, cs->cur, sc, sh->v0, s);
    }
    for (int attempt = 0;; attempt++) {  // (protocol B: again after a short edge exchange)
    if (sh->proto == FDBCS_PROTOCOL_B) {
        // 3 (protocol B): exchange 1 with the edge counts, then the edges
        if ((r = sh_exchange_b(sh, v, slots, flags))) return r;
    } else {
        if ((r = edges_read_check(cs, v, sh->v0))) return r;
        if (T) launch_flags_out(b, (int)T, flags, s);
        // 3: exchange 1
        if ((r = sh_allreduce_max(sh, sh->x1, slots + (size_t)T))) return r;
    }
    launch_sh_carry(sc, reinterpret_cast<const int64_t*>(sh->x1), sh->rank, sh->v0, s);
    if (T) launch_flags_in(b, (int)T, flags, s);
    // 4: the decision, verdicts to host-mapped memory
    if (++cs->vseq == 0) cs->vseq = 1;
    const EarlyOut eo{cs->vmap_dev + 64, reinterpret_cast<uint32_t*>(cs->vmap_dev), cs->vseq};
    cs->early_mapped = launch_decide(v, b, sc, b.verdict, s, true, T ? &eo : nullptr);
    if (!cs->early_mapped && T) {
        if ((r = ensure_pinned(cs->vpin, cs->vpin_cap, vpin_scalars_off(T) + sizeof(Scalars)))) return r;
        HIPOK(hipMemcpyAsync(cs->vpin, b.verdict, (size_t)T, hipMemcpyDeviceToHost, s));
        HIPOK(hipMemcpyAsync(cs->vpin + vpin_scalars_off(T), sc, sizeof(Scalars), hipMemcpyDeviceToHost, s));
    }
    HIPOK(hipEventRecord(cs->ev_verdict, s));
    cs->vev_rec = true;
    launch_combine(v, b, sc, s);
    // 5: this shard's part of the merge (carry-in: sc->carry_apply)
    const bool compact = new_oldest > cs->oldest;
    launch_merge(v, b, h, cs->cur, sc, now, sh->v0, !compact, s);
    cs->cur ^= 1;
    // 6: exchange 2, the plan, the compaction
    int64_t* send = sh->x2;
    int64_t* infos = sh->x2 + SH_WORDS;
    launch_sh_info_out(sc, send, sh->rank, (h.shard.has_lo | h.shard.has_hi) != 0, s);
    if ((r = sh_allgather(sh, send, infos))) return r;
    launch_sh_plan(h, cs->cur, sc, infos, sh->rank, sh->world, sh->v0, compact, s);
    if (compact) {
        launch_compact(b, h, cs->cur, sc, new_oldest, s);  // (the window: k_sh_plan)
        cs->cur ^= 1;
        cs->oldest = new_oldest;
    }
    launch_sh_slot_out(sc, reinterpret_cast<int64_t*>(sh->x1), sh->rank, sh->world, s);
    if (sh_mirror) {
        cs->ev_end = cs->ev_slot[mslot];
        HIPOK(hipEventRecord(cs->ev_end, s));
        cs->mirror_batch[mslot] = cs->batches;
        cs->end_mirror = true;
    }
    // the one wait: the verdicts
    if (!T) return FDBCS_OK;
    r = verdict_wait(cs, T, verdict, nullptr, &sh->last_max);
    if (r != E_SH_RETRY) {
        if (r) return r;
        break;
    }
    // Some shard's edge list did not fit the exchange (every rank sees it
    // alike): this attempt's merge, plan and compaction left the history as
    // it was (k_plan_ranges / k_page_merge skip on the error, the directory
    // is copied to the other buffer, k_sh_plan opens no window).  Grow the
    // capacity, search the edges again (the gathered list overwrote this
    // shard's own), and run the batch from exchange 1 on once more.
    // (an error exit restores oldestVersion: the device skipped this
    // attempt's compaction.  Every rank sees the same gathered counts, so the
    // attempt limit is reached on all of them alike.)
    cs->oldest = oldest0;
    if (attempt >= 4) return FDBCS_E_CAPACITY;
    if ((r = sync_state(cs))) return r;
    mirrors_stale(cs);  // (the attempt published; the next one publishes again)
    const int64_t need = cs->sc_host->sh_need;
    sh->retries++;
    GROWLOG("sharded edge exchange short: need %lld, capacity %lld\n", (long long)need, (long long)sh->ecap);
    sh->ecap = std::max<int64_t>(2 * sh->ecap, need + need / 4 + 1024);
    HIPOK(hipMemsetAsync(&sc->err, 0, sizeof(int32_t), s));
    HIPOK(hipMemsetAsync(&sc->last_err, 0, sizeof(int32_t), s));
    HIPOK(hipMemsetAsync(&sc->sh_need, 0, sizeof(int32_t), s));
    sh->need_seen = 0;  // (the decay window restarts at a growth)
    const int64_t cap = std::max<int64_t>(need + need / 4 + 1024, sh->ecap * sh->world);
    if (cap > b.edge_cap && (r = grow_edges(b, cap))) return r;
    if (T) HIPOK(hipMemsetAsync(b.deg, 0, (size_t)T * sizeof(int32_t), s));
    HIPOK(hipMemsetAsync(&sc->edges_total, 0, sizeof(int32_t), s));
    launch_edges_read_check(v, b, cs->h, cs->cur, sc, sh->v0, s);
    }
    if (sh->proto == FDBCS_PROTOCOL_B) sh_ecap_decay(sh);
    cs->last_dv = v;
    cs->have_last_dv = true;
    return FDBCS_OK;
}

}  // namespace

extern "C" {

int fdbcs_comm_unique_id(uint8_t* id) {
    if (!id) return FDBCS_E_ARG;
    ncclUniqueId u;
    if (ncclGetUniqueId(&u) != ncclSuccess) return FDBCS_E_HIP;
    memcpy(id, u.internal, FDBCS_COMM_ID_BYTES);
    return FDBCS_OK;
}

int fdbcs_sharded_create(fdbcs_sharded** out, int32_t rank, int32_t world, const uint8_t* bound_bytes,
                         const uint64_t* bound_off, const uint32_t* bound_len, int64_t v0, const fdbcs_config* cfg,
                         const uint8_t* comm_id, const fdbcs_comm_ops* ops) {
    if (!out) return FDBCS_E_ARG;
    *out = nullptr;
    // (neither comm_id nor ops: the communicator comes later, fdbcs_sharded_comm_init)
    if (world < 1 || world > 64 || rank < 0 || rank >= world || (comm_id && ops)) return FDBCS_E_ARG;
    if (world > 1 && (!bound_bytes || !bound_off || !bound_len)) return FDBCS_E_ARG;
    if (ops && (!ops->allreduce_max_u8 || !ops->allgather_u8)) return FDBCS_E_ARG;
    fdbcs_sharded* sh = new (std::nothrow) fdbcs_sharded();
    if (!sh) return FDBCS_E_NOMEM;
    sh->rank = rank;
    sh->world = world;
    sh->v0 = v0;
    if (const char* e = getenv("FDBCS_TEST_SH_ECAP")) sh->ecap = sh->ecap0 = std::max(1, atoi(e));  // (tests: short exchanges)
    if (const char* e = getenv("FDBCS_SH_ECAP_WINDOW"))
        sh->ecap_window = std::min(fdbcs_sharded::ECAP_WINDOW_MAX, std::max(1, atoi(e)));
    auto fail = [&](int code) {
        fdbcs_sharded_destroy(sh);
        return code;
    };
    int r;
    // (no borrowed batches here: a protocol-B rank's adds hand the engine a
    // filtered copy of the ranges that lives only for the call)
    fdbcs_config local{};
    if (cfg) local = *cfg;
    local.flags &= ~(FDBCS_BORROW_ALWAYS | FDBCS_BORROW_LARGE);
    if ((r = fdbcs_create(&sh->cs, v0, &local))) return fail(r);
    fdbcs* cs = sh->cs;
    // this rank's keys: [bound[rank-1], bound[rank])
    const uint8_t* lo = rank > 0 ? bound_bytes + bound_off[rank - 1] : nullptr;
    const uint8_t* hi = rank < world - 1 ? bound_bytes + bound_off[rank] : nullptr;
    for (int g = 1; g + 1 < world; g++)  // (the header asks for strictly increasing split keys)
        if (keycmp(bound_bytes + bound_off[g - 1], bound_len[g - 1], bound_bytes + bound_off[g], bound_len[g]) >= 0)
            return fail(FDBCS_E_ARG);
    if ((r = fdbcs_set_shard(cs, lo, rank > 0 ? bound_len[rank - 1] : 0, rank > 0, hi,
                             rank < world - 1 ? bound_len[rank] : 0, rank < world - 1)))
        return fail(r);
    sh->has_lo = rank > 0;
    sh->has_hi = rank < world - 1;
    if (sh->has_lo) sh->lo.assign(lo, lo + bound_len[rank - 1]);
    if (sh->has_hi) sh->hi.assign(hi, hi + bound_len[rank]);
    if (hipMalloc((void**)&sh->x2, (size_t)(world + 1) * SH_WORDS * 8) != hipSuccess) return fail(FDBCS_E_NOMEM);
    launch_sh_init(cs->sc, v0, true, cs->stream);
    if (ops) {
        sh->ops = *ops;
        sh->host_ops = true;
    } else if (comm_id) {
        if ((r = sh_comm_init(sh, comm_id))) return fail(r);
    }
    // the first exchange 1: this shard's (empty) slot
    const size_t slots = sh_slot_bytes(sh);
    if (hipMalloc((void**)&sh->x1, 2 * (slots + 8192)) != hipSuccess) return fail(FDBCS_E_NOMEM);
    sh->x1_cap = (int64_t)(2 * (slots + 8192));
    HIPOK(hipMemsetAsync(sh->x1, 0, (size_t)sh->x1_cap, cs->stream));
    launch_sh_slot_out(cs->sc, reinterpret_cast<int64_t*>(sh->x1), rank, world, cs->stream);
    if ((r = sync_state(cs))) return fail(r);
    *out = sh;
    return FDBCS_OK;
}

int fdbcs_sharded_comm_init(fdbcs_sharded* sh, const uint8_t* comm_id) {
    if (!sh || !comm_id || sh->host_ops || sh->comm || sh->aborted) return FDBCS_E_ARG;
    HIPOK(hipSetDevice(sh->cs->device));
    return sh_comm_init(sh, comm_id);  // (non-blocking: fdbcs_sharded_abort ends a wait for a missing peer)
}

// Another thread's way out of a batch whose peer will never join: RCCL's
// in-flight collectives end (ncclCommAbort), every later call fails.  Only
// `aborted` and, under comm_mu, the communicator are touched here: the rank's
// thread is either inside an RCCL call (abort waits for it to return) or
// polls between calls and sees the flag.
int fdbcs_sharded_abort(fdbcs_sharded* sh) {
    if (!sh) return FDBCS_E_ARG;
    sh->aborted.store(true, std::memory_order_release);
    std::lock_guard<std::mutex> lk(sh->comm_mu);
    if (sh->comm && !sh->comm_dead) {
        ncclCommAbort(sh->comm);  // (frees the communicator; a pending initialisation ends too)
        sh->comm_dead = true;
    }
    return FDBCS_OK;
}

void fdbcs_sharded_destroy(fdbcs_sharded* sh) {
    if (!sh) return;
    if (sh->cs && !sh->aborted) hipStreamSynchronize(sh->cs->stream);
    if (sh->comm && !sh->comm_dead) ncclCommDestroy(sh->comm);
    if (sh->x1) hipFree(sh->x1);
    if (sh->x2) hipFree(sh->x2);
    if (sh->hx) hipHostFree(sh->hx);
    if (sh->ebuf) hipFree(sh->ebuf);
    if (sh->cs) fdbcs_destroy(sh->cs);
    delete sh;
}

fdbcs* fdbcs_sharded_local(fdbcs_sharded* sh) { return sh ? sh->cs : nullptr; }

int fdbcs_sharded_clear(fdbcs_sharded* sh, int64_t v) {
    if (!sh || sh->in_batch) return FDBCS_E_ARG;
    int r;
    if ((r = reset_history(sh->cs, v))) return r;  // oldestVersion and removalKey are kept
    sh->v0 = v;
    launch_sh_init(sh->cs->sc, v, false, sh->cs->stream);
    launch_sh_slot_out(sh->cs->sc, reinterpret_cast<int64_t*>(sh->x1), sh->rank, sh->world, sh->cs->stream);
    return sync_state(sh->cs);
}

int fdbcs_sharded_detect_device(fdbcs_sharded* sh, const fdbcs_batch_view* dev_batch, int64_t now,
                                int64_t new_oldest, uint8_t* verdict) {
    if (!sh || !dev_batch || sh->in_batch) return FDBCS_E_ARG;
    return sh_run(sh, *dev_batch, now, new_oldest, verdict);
}

// iopsSample.addAndExpire of every range's begin of one added transaction,
// writes then reads (fdbcs_sharded::lm_host)
static void sh_roll_host(fdbcs_sharded* sh, const fdbcs_range* reads, int32_t nreads, const fdbcs_range* writes,
                         int32_t nwrites) {
    const fdbcs::Lm& L = sh->cs->lm;
    for (int32_t i = 0; i < nwrites + nreads; i++) {
        const fdbcs_range& x = i < nwrites ? writes[i] : reads[i - nwrites];
        const uint64_t pos = sh->lm_pos++;
        const int64_t amt = roll_amount(roll_hash(L.seed, sh->lm_seq, pos), L.opk + (int64_t)x.begin_len, L.units);
        if (!amt) continue;
        const uint64_t off = sh->lm_bytes.size();
        sh->lm_bytes.insert(sh->lm_bytes.end(), x.begin, x.begin + x.begin_len);
        sh->lm_ent.push_back(LmEntry{amt, (uint32_t)pos, x.begin_len, off, 0});
    }
}

int fdbcs_sharded_batch_begin(fdbcs_sharded* sh) {
    if (!sh) return FDBCS_E_ARG;
    int r;
    sh->cs->lv_prev_T = 0;  // (no live ingest: sh_run ingests the whole batch)
    if ((r = fdbcs_batch_begin(sh->cs))) return r;
    sh->in_batch = true;
    const fdbcs::Lm& L = sh->cs->lm;
    sh->lm_host = !sh->presplit && sh->world > 1 && L.owner && L.seq;
    if (sh->lm_host) {
        sh->lm_seq = *L.seq;  // (the draws of the batch the sample takes next)
        sh->lm_pos = 0;
        sh->lm_ent.clear();
        sh->lm_bytes.clear();
    }
    return FDBCS_OK;
}

int fdbcs_sharded_exchange_stats(const fdbcs_sharded* sh, int64_t* out, int cap) {
    if (!sh || !out || cap < 0) return FDBCS_E_ARG;
    const int64_t v[5] = {sh->ecap, sh->retries, sh->last_max, sh->shrinks, sh->ebuf_cap};
    const int n = std::min(cap, 5);
    for (int i = 0; i < n; i++) out[i] = v[i];
    return n;
}

int fdbcs_sharded_set_protocol(fdbcs_sharded* sh, int protocol, int flags) {
    if (!sh || sh->in_batch || (protocol != FDBCS_PROTOCOL_A && protocol != FDBCS_PROTOCOL_B) ||
        (flags & ~FDBCS_SHARD_PRESPLIT))
        return FDBCS_E_ARG;
    sh->proto = protocol;
    sh->presplit = (flags & FDBCS_SHARD_PRESPLIT) != 0;
    sh->cs->sparse_edges = protocol == FDBCS_PROTOCOL_B;  // (the overlap edges are exported, no rounds)
    return FDBCS_OK;
}

int fdbcs_sharded_batch_add(fdbcs_sharded* sh, int64_t read_snapshot, const fdbcs_range* reads, int32_t nreads,
                            const fdbcs_range* writes, int32_t nwrites) {
    if (!sh) return FDBCS_E_ARG;
    if (!sh->in_batch) return FDBCS_E_STATE;
    if (sh->lm_host && sh->proto == FDBCS_PROTOCOL_A) {  // (B rolls below, after its checks)
        const int r = fdbcs_batch_add(sh->cs, read_snapshot, reads, nreads, writes, nwrites);
        if (r == FDBCS_OK) sh_roll_host(sh, reads, nreads, writes, nwrites);
        return r;
    }
    if (sh->proto == FDBCS_PROTOCOL_A || sh->presplit || sh->world == 1)
        return fdbcs_batch_add(sh->cs, read_snapshot, reads, nreads, writes, nwrites);
    // protocol B: only the ranges that intersect this rank's keys, and the
    // writes ending exactly at its first key (their end node is created here)
    // -- fdbcs_split_batch_keep_all's rule, as the proxy splits for resolvers
    // (MasterProxyServer.actor.cpp:267-307).  The transaction stays (its
    // index is global) even with nothing left.
    if (nreads < 0 || nwrites < 0 || (nreads && !reads) || (nwrites && !writes)) return FDBCS_E_ARG;
    // every rank refuses the same transactions: the checks run on all of its
    // ranges, not just the ones kept here (include/fdbcs.h fdbcs_batch_add)
    for (int32_t i = 0; i < nreads + nwrites; i++) {
        const fdbcs_range& x = i < nreads ? reads[i] : writes[i - nreads];
        if (x.begin_len > FDBCS_MAX_KEY || x.end_len > FDBCS_MAX_KEY) return FDBCS_E_KEY;
    }
    for (int32_t i = 0; i < nreads + nwrites; i++) {
        const fdbcs_range& x = i < nreads ? reads[i] : writes[i - nreads];
        if (keycmp(x.begin, x.begin_len, x.end, x.end_len) >= 0) return FDBCS_E_RANGE;
    }
    const uint8_t* lo = sh->lo.data();
    const uint8_t* hi = sh->hi.data();
    const uint32_t ll = (uint32_t)sh->lo.size(), hl = (uint32_t)sh->hi.size();
    auto hits = [&](const fdbcs_range& x) {
        return (!sh->has_lo || keycmp(x.end, x.end_len, lo, ll) > 0) &&
               (!sh->has_hi || keycmp(x.begin, x.begin_len, hi, hl) < 0);
    };
    std::vector<fdbcs_range>& k = sh->keep;
    k.clear();
    for (int32_t i = 0; i < nreads; i++)
        if (hits(reads[i])) k.push_back(reads[i]);
    const int32_t kr = (int32_t)k.size();
    for (int32_t i = 0; i < nwrites; i++)
        if (hits(writes[i]) || (sh->has_lo && keycmp(writes[i].end, writes[i].end_len, lo, ll) == 0))
            k.push_back(writes[i]);
    // (a read dropped here still makes the transaction tooOld-capable: the
    // shard holding it reports the flag, and the MAX picks it)
    const int r = fdbcs_batch_add(sh->cs, read_snapshot, k.data(), kr, k.data() + kr, (int32_t)k.size() - kr);
    // the whole transaction to the attached sample, only once it was taken
    // (as under A: a refused one uses no sample positions)
    if (r == FDBCS_OK && sh->lm_host) sh_roll_host(sh, reads, nreads, writes, nwrites);
    return r;
}

int fdbcs_sharded_batch_skip(fdbcs_sharded* sh, int32_t n) {
    if (!sh) return FDBCS_E_ARG;
    if (!sh->in_batch) return FDBCS_E_STATE;
    return fdbcs_batch_skip(sh->cs, n);
}

int fdbcs_sharded_batch_detect(fdbcs_sharded* sh, int64_t now, int64_t new_oldest, uint8_t* verdict) {
    if (!sh) return FDBCS_E_ARG;
    if (!sh->in_batch) return FDBCS_E_STATE;
    fdbcs* cs = sh->cs;
    sh->in_batch = false;
    cs->in_batch = false;
    fdbcs_batch_view dv;
    int r;
    if ((r = cs->st.finish(dv, &cs->b.staged))) return r;
    cs->stage_key_total = cs->st.key_total();
    r = sh_run(sh, dv, now, new_oldest, verdict);
    cs->stage_key_total = 0;
    cs->b.staged = StagedBatch{};
    fdbcs::Lm& L = cs->lm;
    L.rolled = false;
    L.host_ent = nullptr;
    if (r == FDBCS_OK && sh->lm_host && L.owner && L.seq) {  // this batch's host roll, for fdbcs_sample_add_batch
        L.rolled = true;
        L.rolled_seq = sh->lm_seq;
        L.count = (int64_t)sh->lm_ent.size();
        L.batch = cs->batches;
        L.host_ent = sh->lm_ent.data();
        L.host_bytes = sh->lm_bytes.data();
        L.host_nb = sh->lm_bytes.size();
    }
    sh->lm_host = false;
    return r;
}

int32_t fdbcs_sharded_removal_key_owner(fdbcs_sharded* sh) {
    if (!sh) return FDBCS_E_ARG;
    int r;
    if ((r = sync_state(sh->cs))) return r;
    return sh->cs->sc_host->sh_rk_owner;
}

int64_t fdbcs_sharded_header_version(const fdbcs_sharded* sh) { return sh ? sh->v0 : 0; }

}  // extern "C"

// ================================================== history queries ====
extern "C" int fdbcs_nth_after(fdbcs* cs, int32_t n, const uint8_t* key_bytes, const uint64_t* key_off,
                               const uint32_t* key_len, const int64_t* steps, uint8_t* out, uint32_t out_stride,
                               int32_t* out_len) {
    if (cs) live_quiesce(cs);
    if (!cs || n < 0 || (n && (!key_bytes || !key_off || !key_len || !steps || !out || !out_len))) return FDBCS_E_ARG;
    if (n == 0) return FDBCS_OK;
    hipStream_t s = cs->stream;
    // the queries, encoded; tails 8-byte aligned and zero padded (tail_cmp reads whole words)
    std::vector<uint64_t> hi(n), lo(n);
    std::vector<uint32_t> meta(n);
    std::vector<uint64_t> toff(n, ~0ull);
    uint64_t tbytes = 0;
    for (int32_t i = 0; i < n; i++) {
        if (key_len[i] > FDBCS_MAX_KEY) return FDBCS_E_KEY;
        encode_host(key_bytes + key_off[i], key_len[i], hi[i], lo[i], meta[i]);
        if (key_len[i] > 17) {
            toff[i] = tbytes;
            tbytes += ((uint64_t)key_len[i] - 17 + 7) & ~7ull;
        }
    }
    std::vector<uint8_t> tails(tbytes + 8, 0);
    for (int32_t i = 0; i < n; i++)
        if (key_len[i] > 17) memcpy(tails.data() + toff[i], key_bytes + key_off[i] + 17, key_len[i] - 17);
    const uint32_t tstride = out_stride > 17 ? ((out_stride - 17 + 7) & ~7u) : 8;
    uint64_t *dhi = nullptr, *dlo = nullptr, *dout = nullptr;
    uint32_t* dmeta = nullptr;
    const uint8_t** dtp = nullptr;
    uint8_t *dtails = nullptr, *douttail = nullptr;
    int64_t* dsteps = nullptr;
    int r = FDBCS_OK;
    auto cleanup = [&]() {
        dfree(dhi); dfree(dlo); dfree(dmeta); dfree(dtp); dfree(dtails); dfree(dsteps); dfree(dout); dfree(douttail);
    };
    if ((r = dalloc(dhi, n)) || (r = dalloc(dlo, n)) || (r = dalloc(dmeta, n)) || (r = dalloc(dtp, n)) ||
        (r = dalloc(dtails, (int64_t)tbytes + 8)) || (r = dalloc(dsteps, n)) || (r = dalloc(dout, 3 * (int64_t)n)) ||
        (r = dalloc(douttail, (int64_t)n * tstride))) {
        cleanup();
        return r;
    }
    std::vector<const uint8_t*> tp(n, nullptr);
    for (int32_t i = 0; i < n; i++)
        if (key_len[i] > 17) tp[i] = dtails + toff[i];
    hipError_t e = hipSuccess;
    auto cp = [&](void* d, const void* h, size_t b) {
        if (e == hipSuccess) e = hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, s);
    };
    cp(dhi, hi.data(), (size_t)n * 8);
    cp(dlo, lo.data(), (size_t)n * 8);
    cp(dmeta, meta.data(), (size_t)n * 4);
    cp(dtp, tp.data(), (size_t)n * 8);
    cp(dtails, tails.data(), tails.size());
    cp(dsteps, steps, (size_t)n * 8);
    NthArgs a{};
    a.n = n; a.qhi = dhi; a.qlo = dlo; a.qmeta = dmeta; a.qtail = dtp; a.steps = dsteps;
    a.out = dout; a.out_tail = douttail; a.tail_stride = tstride;
    launch_nth_after(cs->h, cs->cur, cs->sc, a, s);  // (after every batch already on the stream)
    std::vector<uint64_t> res(3 * (size_t)n);
    std::vector<uint8_t> rtail((size_t)n * tstride);
    if (e == hipSuccess) e = hipMemcpyAsync(res.data(), dout, res.size() * 8, hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipMemcpyAsync(rtail.data(), douttail, rtail.size(), hipMemcpyDeviceToHost, s);
    if (e == hipSuccess) e = hipStreamSynchronize(s);
    cleanup();
    if (e != hipSuccess) {
        last_hip_error() = e;
        return FDBCS_E_HIP;
    }
    for (int32_t i = 0; i < n; i++) {
        const uint64_t m = res[3 * (size_t)i + 2];
        if (m == ~0ull) {
            out_len[i] = -1;
            continue;
        }
        const std::vector<uint8_t> k = decode_key(res[3 * (size_t)i], res[3 * (size_t)i + 1], (uint32_t)m,
                                                  rtail.data() + (size_t)i * tstride);
        if (k.size() > out_stride) {
            out_len[i] = (int32_t)k.size();  // (too long for out_stride: not copied)
            continue;
        }
        memcpy(out + (size_t)i * out_stride, k.data(), k.size());
        out_len[i] = (int32_t)k.size();
    }
    return FDBCS_OK;
}
