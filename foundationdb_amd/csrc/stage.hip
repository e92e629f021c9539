// stage.hip -- host staging of the per-transaction path (see stage.h).
#include "stage.h"
#include "stage_pack.h"

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace fdbcs_dev {

namespace {

// The record stream and offsets: host-mapped and coherent while small enough
// for live ingest (which reads them while they are written); a stream grown
// past LIVE_STREAM_MAX (large batches, which never go live) is default
// pinned memory -- coherent allocations of ~10^6-transaction streams left
// later whole-batch staging out of memory.
constexpr uint64_t LIVE_STREAM_MAX = 256ull << 20;
#ifdef FDBCS_STAGE_NONCOHERENT  // (A/B of the adds' cost)
unsigned stream_flags(uint64_t) { return hipHostMallocDefault; }
#else
unsigned stream_flags(uint64_t bytes) {
    return bytes <= LIVE_STREAM_MAX ? hipHostMallocMapped | hipHostMallocCoherent : hipHostMallocDefault;
}
#endif

using fdbcs_pack::put_ranges;

}  // namespace

// ---- borrowed batches ----------------------------------------------------------
// finish() of a borrowed batch: the records the adds would have written, made
// on host threads from the caller's range arrays (still valid: the caller
// keeps them until detectConflicts returns, as the reference's arena).  One
// parallel region over N workers (the caller's thread is worker 0):
//   1. every piece of the batch is checked (FDBCS_E_KEY / FDBCS_E_RANGE as
//      the add would refuse it) and measured: record bytes, reads, writes, key
//      bytes;
//   2. worker 0 places the pieces (a prefix over them) and sizes the stream;
//   3. each worker writes its pieces' records and offset entries, the offsets
//      straight after the records.
// The pieces are round-major (round c = pieces c*N .. c*N + N - 1, one
// contiguous part of the stream), and worker 0 sends each round on the copy
// stream as soon as its last piece is written, so the copies of the first
// rounds overlap the packing of the later ones.  A refused batch changes
// nothing (FDBCS_E_KEY / FDBCS_E_RANGE from detectConflicts; the reference
// would ASSERT in detectConflicts, SkipList.cpp:1117, 1127).  Point ranges
// share their end's bytes whatever the key length (SHARE_ABOVE 0): no jump of
// the caller's add loop to mispredict here, and fewer PCIe bytes.
//
// The workers are a pool kept by the stage and blocked on a condition
// variable between batches: spinning helper threads made the caller's own add
// loop 3x slower ("Measured and dropped" (ii)), and creating
// threads per batch costs more than a config-2 batch's whole pack.
class HostPool {
   public:
    explicit HostPool(int n) : n_(n) {
        for (int w = 1; w < n_; w++) th_.emplace_back([this, w] { loop(w); });
    }
    ~HostPool() {
        {
            std::lock_guard<std::mutex> g(mu_);
            quit_ = true;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int size() const { return n_; }
    // f(worker) on every worker, the caller's thread as worker 0
    void run(const std::function<void(int)>& f) {
        start(&f, n_);
        f(0);
        wait();
    }
    // f(w) on workers 1 .. n-1, returning at once (*f must outlive wait())
    void start(const std::function<void(int)>* f, int n) {
        left_.store(n - 1, std::memory_order_relaxed);
        {
            std::lock_guard<std::mutex> g(mu_);
            f_ = f;
            active_ = n;
            gen_.fetch_add(1, std::memory_order_release);
        }
        cv_.notify_all();
    }
    void wait() {
        while (left_.load(std::memory_order_acquire) > 0) _mm_pause();
    }

   private:
    // A worker that just finished polls for the next job for a while before
    // it sleeps: a Resolver's batches follow each other closely, and a
    // sleeping thread's wake-up took longer than the adds it should overlap
    // (config 2: ~25 us of adds; FDBCS_POOL_SPIN_US, default 2000).
    static int64_t spin_ns() {
        static const int64_t ns = 1000 * (getenv("FDBCS_POOL_SPIN_US") ? atoll(getenv("FDBCS_POOL_SPIN_US")) : 2000);
        return ns;
    }
    void loop(int w) {
        uint64_t seen = 0;
        bool worked = false;  // (only the workers of the last job poll: the others sleep at once)
        for (;;) {
            const std::function<void(int)>* f;
            int active;
            if (worked) {
                const auto t0 = std::chrono::steady_clock::now();
                for (int it = 1; gen_.load(std::memory_order_acquire) == seen; it++) {
                    _mm_pause();
                    if ((it & 1023) == 0 && std::chrono::duration_cast<std::chrono::nanoseconds>(
                                                std::chrono::steady_clock::now() - t0).count() > spin_ns())
                        break;
                }
            }
            {
                std::unique_lock<std::mutex> g(mu_);
                cv_.wait(g, [&] { return gen_.load(std::memory_order_relaxed) != seen; });
                seen = gen_.load(std::memory_order_relaxed);
                if (quit_) return;
                f = f_;
                active = active_;
            }
            worked = w < active;
            if (!worked) continue;
            (*f)(w);
            left_.fetch_sub(1, std::memory_order_acq_rel);
        }
    }
    int n_;
    std::vector<std::thread> th_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::atomic<uint64_t> gen_{0};
    bool quit_ = false;
    int active_ = 0;
    const std::function<void(int)>* f_ = nullptr;
    std::atomic<int> left_{0};
};

namespace {
int host_threads() {
    static const int n = [] {
        const char* e = getenv("FDBCS_HOST_THREADS");
        const int hw = (int)std::max(1u, std::thread::hardware_concurrency());
        return std::max(1, e ? atoi(e) : std::min(16, hw));
    }();
    return n;
}
// transactions per worker below which fewer workers pack (FDBCS_BORROW_GRAIN)
int64_t borrow_grain() {
    static const int64_t g = getenv("FDBCS_BORROW_GRAIN") ? std::max(1LL, atoll(getenv("FDBCS_BORROW_GRAIN"))) : 512;
    return g;
}
}  // namespace

// ---- live borrowed batches -------------------------------------------------------
namespace {
constexpr int64_t LB_CHUNK = 64;  // transactions a helper packs and publishes at once
// (copy mode) bytes per H2D copy of the finished prefix (FDBCS_LB_COPY, default 128 KiB)
uint64_t lb_copy_min() {
    static const uint64_t n = getenv("FDBCS_LB_COPY") ? std::max(4096ULL, strtoull(getenv("FDBCS_LB_COPY"), nullptr, 0))
                                                       : (512ull << 10);  // (A/B: profiles/r06_ab_lb_copy.txt)
    return n;
}
int lb_helpers() {  // FDBCS_LB_HELPERS (default 4: 4, 8 and 12 gave the same config-2 window)
    static const int n = getenv("FDBCS_LB_HELPERS") ? std::max(1, atoi(getenv("FDBCS_LB_HELPERS"))) : 4;
    return n;
}
// The caller's batch arrays are cold (a Resolver request arrives from the
// network): the range entries of transaction t + 8 and the keys of t + 4 are
// requested ahead, as the copying add does for its own keys.
inline void lb_prefetch_ranges(const fdbcs_range* r, int n) {
    for (int i = 0; i < n; i += 2) __builtin_prefetch(r + i);
}
inline void lb_prefetch_keys(const fdbcs_range* r, int n) {
    for (int i = 0; i < n; i++) {
        __builtin_prefetch(r[i].begin);
        __builtin_prefetch(r[i].end);
    }
}
}  // namespace

struct TxnStage::LbShared {
    alignas(64) std::atomic<int64_t> added{0};  // transactions added (the caller publishes whole chunks)
    alignas(64) std::atomic<int> fin{0};        // the caller is in finish(): `added` is final
    alignas(64) std::atomic<int64_t> next{0};   // the next chunk a helper takes
    alignas(64) std::atomic<int64_t> ticket{0}; // the chunk whose stream bytes are reserved next
    uint64_t cursor = 0;                        // stream bytes reserved (the ticket's holder only)
    alignas(64) std::atomic<int> stop{0};       // refused, over a capacity, or abandoned: helpers leave
    std::atomic<int> broken{0};                 // over the stream or key-byte capacity (finish repacks)
    std::atomic<int64_t> bad{INT64_MAX};        // the first refused transaction
    std::atomic<int> code{FDBCS_OK};
    std::atomic<uint64_t> keys{0};
    std::mutex pub_mu;
    int64_t pub = 0;                            // chunks published (pub_mu)
    int64_t nchunks = 0;
    std::unique_ptr<std::atomic<uint8_t>[]> done;
    std::vector<uint64_t> end;                  // per chunk: its reserved bytes' end (a fresh line after)
    std::vector<int64_t> tend;                  // per chunk: its last transaction + 1
    std::vector<int64_t> ro, wo;                // per chunk: reads / writes before it (the caller writes these)
    std::function<void(int)> fn;
    void reset(int64_t n) {
        added.store(0);
        fin.store(0);
        next.store(0);
        ticket.store(0);
        cursor = 0;
        stop.store(0);
        broken.store(0);
        bad.store(INT64_MAX);
        code.store(FDBCS_OK);
        keys.store(0);
        pub = 0;
        if (n > nchunks) {
            done.reset(new std::atomic<uint8_t>[(size_t)n]);
            end.resize((size_t)n);
            tend.resize((size_t)n);
            ro.resize((size_t)n);
            wo.resize((size_t)n);
            nchunks = n;
        }
        for (int64_t k = 0; k < nchunks; k++) done[k].store(0, std::memory_order_relaxed);
    }
};

// One helper: chunks in the order taken; each measured (and checked), its
// stream bytes reserved in chunk order (so the published bytes stay a
// prefix, each chunk starting on a fresh 128-byte line: pad_published's rule),
// packed, then the prefix of finished chunks published.
void TxnStage::lb_work() {
    LbShared& S = *lbs_;
    const BorrowRec* br = brec_;
    for (;;) {
        const int64_t k = S.next.fetch_add(1, std::memory_order_relaxed);
        const int64_t t0 = k * LB_CHUNK;
        int64_t t1;
        for (;;) {  // until the chunk is whole (or the batch ends inside it)
            if (S.stop.load(std::memory_order_acquire)) return;
            const int64_t a = S.added.load(std::memory_order_acquire);
            if (a >= t0 + LB_CHUNK) {
                t1 = t0 + LB_CHUNK;
                break;
            }
            if (S.fin.load(std::memory_order_acquire)) {
                t1 = std::min(t0 + LB_CHUNK, S.added.load(std::memory_order_acquire));
                break;
            }
            _mm_pause();
        }
        if (t1 <= t0 || k >= S.nchunks) return;  // (past the batch's end)
        uint64_t bytes = 0, keys = 0;
        for (int64_t t = t0; t < std::min(t1, t0 + 8); t++) {
            lb_prefetch_ranges(br[t].rd, br[t].nr);
            lb_prefetch_ranges(br[t].wr, br[t].nw);
        }
        for (int64_t t = t0; t < t1; t++) {
            if (t + 8 < t1) {
                lb_prefetch_ranges(br[t + 8].rd, br[t + 8].nr);
                lb_prefetch_ranges(br[t + 8].wr, br[t + 8].nw);
            }
            if (t + 4 < t1) {
                lb_prefetch_keys(br[t + 4].rd, br[t + 4].nr);
                lb_prefetch_keys(br[t + 4].wr, br[t + 4].nw);
            }
            const BorrowRec& x = br[t];
            if (x.nr + x.nw == 0) continue;
            int st;
            const uint64_t kb = fdbcs_pack::ranges_bytes<0>(x.rd, x.nr, x.wr, x.nw, st);
            if (st != FDBCS_OK) {
                int64_t b = S.bad.load();
                while (t < b && !S.bad.compare_exchange_weak(b, t)) {
                }
                if (S.bad.load() == t) S.code.store(st);
                S.stop.store(1, std::memory_order_release);
                return;
            }
            for (int i = 0; i < x.nr; i++) keys += (uint64_t)x.rd[i].begin_len + x.rd[i].end_len;
            for (int i = 0; i < x.nw; i++) keys += (uint64_t)x.wr[i].begin_len + x.wr[i].end_len;
            bytes += (sizeof(StageHdr) + 8 * (uint64_t)(x.nr + x.nw) + kb + 7) & ~uint64_t(7);
        }
        while (S.ticket.load(std::memory_order_acquire) != k) {
            if (S.stop.load(std::memory_order_acquire)) return;
            _mm_pause();
        }
        const uint64_t off = S.cursor;
        const uint64_t nxt = (off + bytes + 16 + 127) & ~uint64_t(127);
        const bool over = nxt + 8 * ((uint64_t)lcaps_.T + 1) + 16 > cap_ ||
                          S.keys.fetch_add(keys, std::memory_order_relaxed) + keys > lcaps_.key_bytes;
        if (over) {
            S.broken.store(1);
            S.stop.store(1, std::memory_order_release);
            return;
        }
        S.cursor = nxt;
        S.end[k] = nxt;
        S.tend[k] = t1;
        S.ticket.store(k + 1, std::memory_order_release);
        uint64_t o = off;
        int64_t R = S.ro[k], W = S.wo[k];
        for (int64_t t = t0; t < t1; t++) {
            const BorrowRec& x = br[t];
            if (x.nr + x.nw == 0) {
                toff_[t] = STAGE_EMPTY | ((uint64_t)W << 32) | (uint64_t)R;
                continue;
            }
            uint8_t* p = pin_ + o;
            StageRange* ent = reinterpret_cast<StageRange*>(p + sizeof(StageHdr));
            uint8_t* kp = p + sizeof(StageHdr) + sizeof(StageRange) * (size_t)(x.nr + x.nw);
            fdbcs_pack::put_ranges<StageRange, STAGE_SHARED, 0>(x.rd, x.nr, ent, p, kp);
            fdbcs_pack::put_ranges<StageRange, STAGE_SHARED, 0>(x.wr, x.nw, ent + x.nr, p, kp);
            const StageHdr h{x.snap, (int32_t)R, (int32_t)W, x.nr, x.nw};
            memcpy(p, &h, sizeof h);
            toff_[t] = o;
            o += ((uint64_t)(kp - p) + 7) & ~uint64_t(7);
            R += x.nr;
            W += x.nw;
        }
        S.done[k].store(1, std::memory_order_release);
        std::lock_guard<std::mutex> g(S.pub_mu);  // the finished prefix to the live kernel (publish()'s word)
        int64_t p = S.pub;
        while (p < S.nchunks && S.done[p].load(std::memory_order_acquire)) p++;
        if (p > S.pub) {
            S.pub = p;
            if (lb_live_) {  // to the live kernel
                if (bar_) _mm_sfence();
                __atomic_store_n(&prog_[0], S.end[p - 1] << 20 | (uint64_t)S.tend[p - 1], __ATOMIC_RELEASE);
            } else if (S.end[p - 1] - sent_ >= lb_copy_min()) {  // to the device, on the copy stream
                if (hipMemcpyAsync(dev_ + sent_, pin_ + sent_, S.end[p - 1] - sent_, hipMemcpyHostToDevice, copy_) !=
                    hipSuccess) {
                    S.broken.store(1);
                    S.stop.store(1, std::memory_order_release);
                    return;
                }
                sent_ = S.end[p - 1];
            }
        }
    }
}

void TxnStage::lb_abandon() {
    if (!lb_) return;
    lbs_->stop.store(1, std::memory_order_release);
    pool_->wait();
    lb_ = false;
    live_cancel();
}

int TxnStage::grow_brec(int64_t need) {
    static_assert(sizeof(BorrowRec) == 32 && offsetof(BorrowRec, rd) == 8 && offsetof(BorrowRec, wr) == 16 &&
                      offsetof(BorrowRec, nr) == 24 && offsetof(BorrowRec, nw) == 28,
                  "the adds store a record as two 16-byte halves");
    const int64_t nc = (std::max<int64_t>(need, std::max<int64_t>(4096, 2 * brec_cap_)) + 1) & ~int64_t(1);  // (64-byte multiple)
    BorrowRec* n = static_cast<BorrowRec*>(aligned_alloc(64, (size_t)nc * sizeof(BorrowRec)));
    if (!n) return FDBCS_E_NOMEM;
    _mm_sfence();
    if (T_) memcpy(n, brec_, (size_t)T_ * sizeof(BorrowRec));
    free(brec_);
    brec_ = n;
    brec_cap_ = nc;
    return FDBCS_OK;
}

void TxnStage::drop_pool() {
    if (lb_) lb_abandon();
    delete pool_;
    pool_ = nullptr;
    delete lbs_;
    lbs_ = nullptr;
}

int TxnStage::pack_borrowed() {
    const int64_t T = T_;
    if (!pool_ && T >= 2 * borrow_grain() && host_threads() > 1) pool_ = new HostPool(host_threads());
    const int N = pool_ ? (int)std::max<int64_t>(1, std::min<int64_t>(pool_->size(), T / borrow_grain())) : 1;
    // rounds: one H2D copy each, the first ones overlapping the later packing
    const int C = T >= (1 << 17) ? 8 : (T >= 4096 ? 2 : 1);
    const int P = C * N;
    struct Piece {
        int64_t t0, t1;
        uint64_t bytes = 0, keys = 0;
        int64_t reads = 0, writes = 0;
        int64_t bad = -1;
        int code = FDBCS_OK;
        uint64_t off = 0;
        int64_t ro = 0, wo = 0;
    };
    std::vector<Piece> pc((size_t)P);
    for (int p = 0; p < P; p++) {
        pc[p].t0 = T * p / P;
        pc[p].t1 = T * (p + 1) / P;
    }
    const BorrowRec* br = brec_;
    auto measure = [&](Piece& q) {
        for (int64_t t = q.t0; t < q.t1; t++) {
            const BorrowRec& x = br[t];
            q.reads += x.nr;
            q.writes += x.nw;
            if (x.nr + x.nw == 0) continue;
            int st;
            const uint64_t kb = fdbcs_pack::ranges_bytes<0>(x.rd, x.nr, x.wr, x.nw, st);
            if (st != FDBCS_OK) {
                q.bad = t;
                q.code = st;
                return;
            }
            for (int i = 0; i < x.nr; i++) q.keys += (uint64_t)x.rd[i].begin_len + x.rd[i].end_len;
            for (int i = 0; i < x.nw; i++) q.keys += (uint64_t)x.wr[i].begin_len + x.wr[i].end_len;
            q.bytes += (sizeof(StageHdr) + 8 * (uint64_t)(x.nr + x.nw) + kb + 7) & ~uint64_t(7);
        }
    };
    auto pack = [&](const Piece& q, uint64_t* toff) {
        uint64_t o = q.off;
        int64_t R = q.ro, W = q.wo;
        for (int64_t t = q.t0; t < q.t1; t++) {
            const BorrowRec& x = br[t];
            if (x.nr + x.nw == 0) {
                toff[t] = STAGE_EMPTY | ((uint64_t)W << 32) | (uint64_t)R;
                continue;
            }
            uint8_t* p = pin_ + o;
            StageRange* ent = reinterpret_cast<StageRange*>(p + sizeof(StageHdr));
            uint8_t* kp = p + sizeof(StageHdr) + sizeof(StageRange) * (size_t)(x.nr + x.nw);
            fdbcs_pack::put_ranges<StageRange, STAGE_SHARED, 0>(x.rd, x.nr, ent, p, kp);
            fdbcs_pack::put_ranges<StageRange, STAGE_SHARED, 0>(x.wr, x.nw, ent + x.nr, p, kp);
            const StageHdr h{x.snap, (int32_t)R, (int32_t)W, x.nr, x.nw};
            memcpy(p, &h, sizeof h);
            toff[t] = o;
            o += ((uint64_t)(kp - p) + 7) & ~uint64_t(7);
            R += x.nr;
            W += x.nw;
        }
    };
    // (phase flags: worker 0 publishes the placement, or an abort, once every
    // worker has measured; the workers spin only inside this one region)
    std::atomic<int> measured{0}, phase{0};  // phase: 1 placed, 2 abort
    std::vector<std::atomic<int>> done((size_t)C);
    for (auto& d : done) d.store(0, std::memory_order_relaxed);
    int status = FDBCS_OK;
    uint64_t total = 0, keys = 0;
    auto body = [&](int w) {
        if (w < N)
            for (int c = 0; c < C; c++) measure(pc[(size_t)c * N + w]);
        measured.fetch_add(1, std::memory_order_acq_rel);
        if (w != 0) {
            int ph;
            while ((ph = phase.load(std::memory_order_acquire)) == 0) _mm_pause();
            if (ph != 1 || w >= N) return;
        } else {
            const int all = pool_ ? pool_->size() : 1;
            while (measured.load(std::memory_order_acquire) < all) _mm_pause();
            uint64_t off = 0;
            int64_t ro = 0, wo = 0;
            for (Piece& q : pc) {
                if (q.bad >= 0) {  // (the first refused transaction, in batch order)
                    bad_txn_ = q.bad;
                    status = q.code;
                    break;
                }
                q.off = off;
                q.ro = ro;
                q.wo = wo;
                off += q.bytes;
                keys += q.keys;
                ro += q.reads;
                wo += q.writes;
            }
            // (the record offsets after the records: finish() sends them with
            // the rest.  An eighth more than this batch needs, so that the next
            // batch of about this size does not re-pin the stream: pinning
            // ~300 MB again put 40 ms batches into config 5's timed region)
            const uint64_t need = off + 8 * (uint64_t)(T + 1) + 16;
            if (status == FDBCS_OK && (need > cap_ || T + 1 > toff_cap_))
                status = grow(T + 1 + T / 8, need + need / 8);
            if (status != FDBCS_OK) {
                phase.store(2, std::memory_order_release);
                return;
            }
            total = off;
            phase.store(1, std::memory_order_release);
        }
        for (int c = 0; c < C; c++) {
            pack(pc[(size_t)c * N + w], reinterpret_cast<uint64_t*>(pin_ + total));  // (offsets after the records)
            done[c].fetch_add(1, std::memory_order_acq_rel);
            if (w != 0) continue;
            // worker 0: this round to the device once every piece of it is written
            while (done[c].load(std::memory_order_acquire) < N) _mm_pause();
            const uint64_t a = pc[(size_t)c * N].off, b = c + 1 < C ? pc[(size_t)(c + 1) * N].off : total;
            if (b > a && hipMemcpyAsync(dev_ + a, pin_ + a, b - a, hipMemcpyHostToDevice, copy_) != hipSuccess)
                status = FDBCS_E_HIP;
        }
    };
    if (pool_) pool_->run(body);
    else body(0);
    if (status != FDBCS_OK) return status;
    used_ = total;
    sent_ = total;  // (finish() sends the offsets and makes the engine's stream wait for the copies)
    K_ = keys;
    toff_in_stream_ = true;
    return FDBCS_OK;
}

void TxnStage::sync() {
    if (copy_) hipStreamSynchronize(copy_);
    if (stream_) hipStreamSynchronize(stream_);
}

void TxnStage::release() {
    live_cancel();  // (a live kernel waiting for this batch leaves: the syncs below return)
    sync();
    drop_pool();
    free(brec_);
    brec_ = nullptr;
    brec_cap_ = 0;
    auto free_host_or_dev = [this](void* p) {
        if (!p) return;
        if (bar_) hipFree(p);
        else hipHostFree(p);
    };
    free_host_or_dev(pin_);
    if (dev_ && dev_ != pin_) hipFree(dev_);
    if (view_) hipFree(view_);
    if (copied_) hipEventDestroy(copied_);
    free_host_or_dev(toff_);
    free_host_or_dev(prog_);
    pin_ = dev_ = view_ = nullptr;
    toff_ = toff_dev_ = nullptr;
    prog_ = prog_dev_ = nullptr;
    live_ = false;
    copied_ = nullptr;
    cap_ = view_cap_ = 0;
    toff_cap_ = 0;
    stream_ = copy_ = nullptr;
    open_ = false;
}

int TxnStage::configure(hipStream_t stream, hipStream_t copy, uint64_t chunk) {
    stream_ = stream;
    copy_ = copy;
    chunk_ = std::max<uint64_t>(4096, chunk);
    if (const char* e = getenv("FDBCS_STAGE_EARLY")) early_ = strtoull(e, nullptr, 0);
    if (const char* e = getenv("FDBCS_LIVE_PUB")) pub_every_ = std::max<int64_t>(8, strtoll(e, nullptr, 0));  // (default 16)
    if (!copied_ && hipEventCreateWithFlags(&copied_, hipEventDisableTiming) != hipSuccess) return FDBCS_E_HIP;
    if (!prog_) {
        // FDBCS_STAGE_BAR=1 (A/B): the stream in device memory the host writes
        // through the large BAR (fine-grained, uncached on the device): the
        // kernels read it from HBM, no copies.  Measured at config 2: detect
        // ~6 us shorter, but the adds' small write-combined stores over PCIe
        // took 245-270 us per batch against 192 into pinned host memory, so
        // the default stays pinned host memory (chunk copies / live reads).
        const bool bar = getenv("FDBCS_STAGE_BAR") && atoi(getenv("FDBCS_STAGE_BAR"));
        bar_ = bar && hipExtMallocWithFlags((void**)&prog_, 64, hipDeviceMallocUncached) == hipSuccess;
        if (bar_) {
            volatile uint64_t* w = prog_;
            for (int i = 0; i < 8; i++) w[i] = 0;  // (the host's store through the BAR: it works or faults here)
            _mm_sfence();
            prog_dev_ = prog_;
        } else {
            if (hipHostMalloc((void**)&prog_, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess)
                return FDBCS_E_NOMEM;
            memset(prog_, 0, 64);
            if (hipHostGetDevicePointer((void**)&prog_dev_, prog_, 0) != hipSuccess) return FDBCS_E_HIP;
        }
    }
    return FDBCS_OK;
}

int TxnStage::begin(bool borrow) {
    live_cancel();  // (a batch begun and never detected)
    if (lb_) lb_abandon();  // (a live borrowed batch begun and never detected)
    borrow_ = borrow;
    bad_txn_ = -1;
    began_live_ = false;
    toff_in_stream_ = false;
    T_ = R_ = W_ = 0;
    K_ = 0;
    used_ = sent_ = 0;
    chunk_sent_ = false;
    live_ = live_broken_ = false;
    if (!pin_) {
        int r = grow(8192, 4 << 20);
        if (r) return r;
    }
    open_ = true;
    return FDBCS_OK;
}

// Grow the offsets and / or the stream.  Chunks already sent went to the old
// device buffer: the whole stream is sent again (sent_ = 0).
int TxnStage::grow(int64_t need_txns, uint64_t need_bytes) {
    if (need_txns > toff_cap_ || need_bytes > cap_) {
        live_cancel();  // (the live kernel reads the old buffers: it leaves first)
        sync();         // copies in flight read the old buffers
    }
    if (bar_) return grow_bar(need_txns, need_bytes);
    if (need_txns > toff_cap_) {
        const int64_t nc = std::max<int64_t>(need_txns, 2 * toff_cap_);
        uint64_t* nt = nullptr;
        if (hipHostMalloc((void**)&nt, (size_t)nc * 8, stream_flags((uint64_t)nc * 8)) != hipSuccess)
            return FDBCS_E_NOMEM;
        toff_live_ = (uint64_t)nc * 8 <= LIVE_STREAM_MAX;
        // (the entries written so far: a borrowed batch's adds write none --
        // its T_ counts transactions whose entries pack_borrowed writes later)
        if (T_ && !borrow_) memcpy(nt, toff_, (size_t)T_ * 8);
        if (toff_) hipHostFree(toff_);
        toff_ = nt;
        toff_cap_ = nc;
        if (hipHostGetDevicePointer((void**)&toff_dev_, toff_, 0) != hipSuccess) return FDBCS_E_HIP;
    }
    if (need_bytes > cap_) {
        const uint64_t nc = std::max<uint64_t>(need_bytes, 2 * cap_);
        uint8_t* np = nullptr;
        // (coherent: the live kernel reads the records over PCIe as they are
        // written, which a device-cached line of a half-written record would break)
        if (hipHostMalloc((void**)&np, nc, stream_flags(nc)) != hipSuccess)
            return FDBCS_E_NOMEM;
        pin_live_ = nc <= LIVE_STREAM_MAX;
        if (used_) memcpy(np, pin_, used_);
        if (pin_) hipHostFree(pin_);
        pin_ = np;
        if (hipHostGetDevicePointer((void**)&pin_dev_, pin_, 0) != hipSuccess) return FDBCS_E_HIP;
        if (dev_) hipFree(dev_);
        dev_ = nullptr;
        cap_ = 0;
        if (hipMalloc((void**)&dev_, nc) != hipSuccess) return FDBCS_E_NOMEM;
        cap_ = nc;
        sent_ = 0;
    }
    return FDBCS_OK;
}

// The BAR stream: device memory, grown by a device-to-device copy (the host
// never reads it back: reads through the BAR are uncached PCIe round trips).
int TxnStage::grow_bar(int64_t need_txns, uint64_t need_bytes) {
    if (need_txns > toff_cap_) {
        const int64_t nc = std::max<int64_t>(need_txns, 2 * toff_cap_);
        uint64_t* nt = nullptr;
        if (hipExtMallocWithFlags((void**)&nt, (size_t)nc * 8, hipDeviceMallocUncached) != hipSuccess)
            return FDBCS_E_NOMEM;
        if (T_ && !borrow_) {  // (see grow: a borrowed batch's adds wrote no entries)
            _mm_sfence();
            if (hipMemcpy(nt, toff_, (size_t)T_ * 8, hipMemcpyDeviceToDevice) != hipSuccess) return FDBCS_E_HIP;
        }
        if (toff_) hipFree(toff_);
        toff_ = toff_dev_ = nt;
        toff_cap_ = nc;
        toff_live_ = true;
    }
    if (need_bytes > cap_) {
        const uint64_t nc = std::max<uint64_t>(need_bytes, 2 * cap_);
        uint8_t* np = nullptr;
        if (hipExtMallocWithFlags((void**)&np, nc, hipDeviceMallocUncached) != hipSuccess) return FDBCS_E_NOMEM;
        if (used_) {
            _mm_sfence();
            if (hipMemcpy(np, pin_, used_, hipMemcpyDeviceToDevice) != hipSuccess) return FDBCS_E_HIP;
        }
        if (pin_) hipFree(pin_);
        pin_ = pin_dev_ = dev_ = np;
        cap_ = nc;
        pin_live_ = true;
    }
    return FDBCS_OK;
}

int TxnStage::add(int64_t snap, const fdbcs_range* reads, int32_t nr, const fdbcs_range* writes, int32_t nw) {
    if (!open_) return FDBCS_E_STATE;
    if (nr < 0 || nw < 0 || (nr && !reads) || (nw && !writes)) return FDBCS_E_ARG;
    if (T_ >= MAX_T || R_ + nr > INT32_MAX / 2 || W_ + nw > INT32_MAX / 2) return FDBCS_E_CAPACITY;
    if (lb_ && (T_ + 1 > lcaps_.T || R_ + nr > lcaps_.R || W_ + nw > lcaps_.W)) lb_abandon();  // (live caps)
    if (lb_) {  // live borrowed: the helpers take whole chunks (lb_work)
        if ((T_ & (LB_CHUNK - 1)) == 0) {
            lbs_->ro[T_ / LB_CHUNK] = R_;
            lbs_->wo[T_ / LB_CHUNK] = W_;
        }
        brec_[T_] = BorrowRec{snap, reads, writes, nr, nw};
        T_++;
        R_ += nr;
        W_ += nw;
        if ((T_ & (LB_CHUNK - 1)) == 0) lbs_->added.store(T_, std::memory_order_release);
        return FDBCS_OK;
    }
    if (borrow_) {  // (checked and packed at finish: pack_borrowed)
        if (T_ >= brec_cap_) {
            const int r = grow_brec(T_ + 1);
            if (r) return r;
        }
        __m128i* d = reinterpret_cast<__m128i*>(brec_ + T_);
        _mm_stream_si128(d, _mm_set_epi64x((long long)(uintptr_t)reads, (long long)snap));
        _mm_stream_si128(d + 1, _mm_set_epi64x((long long)(((uint64_t)(uint32_t)nw << 32) | (uint32_t)nr),
                                               (long long)(uintptr_t)writes));
        T_++;
        R_ += nr;
        W_ += nw;
        return FDBCS_OK;
    }
    const int n = nr + nw;
    if (n == 0) {  // no record: the offset entry says so (kernels.h STAGE_EMPTY)
        if (T_ + 1 > toff_cap_ || used_ + 8 * (uint64_t)(T_ + 1) + 16 > cap_) {
            int r = grow(T_ + 1, used_ + 8 * (uint64_t)(T_ + 1) + 16);
            if (r) return r;
        }
        toff_[T_++] = STAGE_EMPTY | ((uint64_t)W_ << 32) | (uint64_t)R_;
        return FDBCS_OK;
    }
    uint64_t kbytes = 0;
    uint32_t longest = 0;
    // (the keys are requested here, all at once, and read in the copy pass)
    for (int i = 0; i < nr; i++) {
        kbytes += (uint64_t)reads[i].begin_len + reads[i].end_len;
        longest = std::max({longest, reads[i].begin_len, reads[i].end_len});
        __builtin_prefetch(reads[i].begin);
        __builtin_prefetch(reads[i].end);
    }
    for (int i = 0; i < nw; i++) {
        kbytes += (uint64_t)writes[i].begin_len + writes[i].end_len;
        longest = std::max({longest, writes[i].begin_len, writes[i].end_len});
        __builtin_prefetch(writes[i].begin);
        __builtin_prefetch(writes[i].end);
    }
    if (longest > FDBCS_MAX_KEY) return FDBCS_E_KEY;
    const uint64_t rec = (sizeof(StageHdr) + 8 * (uint64_t)n + kbytes + 7) & ~uint64_t(7);
    // (room for the record offsets appended at finish)
    const uint64_t need = used_ + rec + 8 * (uint64_t)(T_ + 1) + 16;
    if (T_ + 1 > toff_cap_ || need > cap_) {
        int r = grow(T_ + 1, need);
        if (r) return r;
    }
    // one pass: check begin < end and copy, reads then writes
    uint8_t* p = pin_ + used_;
    StageRange* ent = reinterpret_cast<StageRange*>(p + sizeof(StageHdr));
    uint8_t* kp = p + sizeof(StageHdr) + sizeof(StageRange) * (size_t)n;
    bool bad = put_ranges<StageRange, STAGE_SHARED>(reads, nr, ent, p, kp);
    bad |= put_ranges<StageRange, STAGE_SHARED>(writes, nw, ent + nr, p, kp);
    if (bad) return FDBCS_E_RANGE;  // (the record is not committed: used_ stays)
    const uint64_t rec_used = ((uint64_t)(kp - p) + 7) & ~uint64_t(7);  // (<= rec: point ranges share bytes)
    const StageHdr h{snap, (int32_t)R_, (int32_t)W_, nr, nw};
    memcpy(p, &h, sizeof h);
    toff_[T_] = used_;
    used_ += rec_used;
    T_++;
    K_ += kbytes;
    R_ += nr;
    W_ += nw;
    if (live_) {
        live_check();
        if (!live_broken_) return FDBCS_OK;  // (no chunk copies: the live kernel reads the stream itself)
    }
    if (bar_) return FDBCS_OK;  // (the stream is in device memory already)
    // a chunk every chunk_ bytes, and one more `early_` bytes before where the
    // previous batch ended (batches are alike): detectConflicts then sends
    // only that much and the record offsets
    if (used_ - sent_ >= chunk_ || (used_ >= early_at_ && sent_ < early_at_)) {
        if (hipMemcpyAsync(dev_ + sent_, pin_ + sent_, used_ - sent_, hipMemcpyHostToDevice, copy_) != hipSuccess)
            return FDBCS_E_HIP;
        sent_ = used_;
        chunk_sent_ = true;
        if (pull_rest() && hipEventRecord(copied_, copy_) != hipSuccess) return FDBCS_E_HIP;
    }
    return FDBCS_OK;
}

// FDBCS_PULL_REST=1: finish() has the engine's queue read the stream's rest
// from the mapped pinned buffer (launch_pull) instead of a last SDMA copy and
// a cross-queue event behind it (A/B knob: ~5 us per batch, within the
// run-to-run spread; off by default)
bool TxnStage::pull_rest() {
    static const bool on = getenv("FDBCS_PULL_REST") && atoi(getenv("FDBCS_PULL_REST"));
    return on;
}

int TxnStage::skip(int32_t n) {
    if (!open_) return FDBCS_E_STATE;
    if (n < 0) return FDBCS_E_ARG;
    if (T_ + n > MAX_T) return FDBCS_E_CAPACITY;
    lb_abandon();  // (runs of empty transactions: a plain borrowed batch from here)
    if (borrow_) {
        if (T_ + n > brec_cap_) {
            const int r = grow_brec(T_ + n);
            if (r) return r;
        }
        std::fill(brec_ + T_, brec_ + T_ + n, BorrowRec{0, nullptr, nullptr, 0, 0});
        T_ += n;
        return FDBCS_OK;
    }
    const uint64_t need = used_ + 8 * (uint64_t)(T_ + n) + 16;
    if (T_ + n > toff_cap_ || need > cap_) {
        int r = grow(T_ + n, need);
        if (r) return r;
    }
    const uint64_t e = STAGE_EMPTY | ((uint64_t)W_ << 32) | (uint64_t)R_;
    std::fill(toff_ + T_, toff_ + T_ + n, e);
    T_ += n;
    if (live_) live_check();
    return FDBCS_OK;
}

// ---- live ingest --------------------------------------------------------------
// The published bytes end on a 128-byte line (an L2 line) at least 16 bytes
// past the last record: the next record starts on a fresh line, so the live
// kernel, which reads only below the published end, never caches a line the
// host writes again (k_live_ingest), and a key's aligned 8-byte reads stay
// below it.  Records are located by their offsets; the gap is never read.
bool TxnStage::pad_published() {
    const uint64_t p = (used_ + 16 + 127) & ~uint64_t(127);
    if (p + 8 * ((uint64_t)T_ + 1) + 16 > cap_) return false;  // (no room: the batch falls back)
    used_ = p;
    return true;
}

void TxnStage::publish() {
    if (!pad_published()) {
        live_cancel();
        return;
    }
    // one word, T (< 2^20: live batches have T <= LARGE_T) and the bytes
    // written whole, after the records and their offsets (through the BAR the
    // stores are write-combined: the fence drains them first)
    if (bar_) _mm_sfence();
    __atomic_store_n(&prog_[0], (uint64_t)used_ << 20 | (uint64_t)T_, __ATOMIC_RELEASE);
    next_pub_ = T_ + pub_every_;
}

void TxnStage::live_check() {
    if (live_broken_) return;
    if (T_ > lcaps_.T || R_ > lcaps_.R || W_ > lcaps_.W || K_ > lcaps_.key_bytes) {
        live_cancel();
        return;
    }
    if (T_ >= next_pub_) publish();
}

void TxnStage::live_cancel() {
    if (!live_ || live_broken_ || !prog_) return;
    live_broken_ = true;
    if (bar_) _mm_sfence();
    __atomic_store_n(&prog_[2], (uint64_t)LV_CANCEL, __ATOMIC_RELEASE);
}

// records (header <= 24 B + 7 B of alignment, 8 B range entries, keys) and
// the padding of every publish (< 144 B each: one per pub_every_
// transactions, one more at the final word, pad_published)
uint64_t TxnStage::live_stream_bound(const LiveCaps& caps) const {
    const uint64_t slots = 2 * ((uint64_t)caps.R + (uint64_t)caps.W);
    return 32 * (uint64_t)caps.T + 4 * slots + caps.key_bytes + 64 +
           160 * ((uint64_t)caps.T / (uint64_t)pub_every_ + 2);
}

int TxnStage::begin_live(const LiveCaps& caps) {
    if (!open_ || T_ || live_) return FDBCS_E_STATE;
    // the records and, should the batch fall back, the offsets appended at finish
    const uint64_t need = live_stream_bound(caps) + 8 * ((uint64_t)caps.T + 1);
    const uint64_t slots = 2 * ((uint64_t)caps.R + (uint64_t)caps.W);
    int r;
    if ((r = grow(caps.T + 1, need))) return r;
    if (!pin_live_ || !toff_live_) return FDBCS_E_STATE;  // (grown past the live size: not coherent)
    auto al = [](uint64_t x) { return (x + 15) & ~uint64_t(15); };
    const uint64_t o_ro = al(8 * (uint64_t)caps.T), o_wo = al(o_ro + 4 * ((uint64_t)caps.T + 1)),
                   o_ko = al(o_wo + 4 * ((uint64_t)caps.T + 1)), o_kl = al(o_ko + 8 * slots),
                   total = al(o_kl + 4 * slots) + 16;
    if (total > view_cap_) {
        if (view_) {
            sync();
            hipFree(view_);
            view_ = nullptr;
        }
        const uint64_t nc = std::max<uint64_t>(total, 2 * view_cap_);
        view_cap_ = 0;
        if (hipMalloc((void**)&view_, nc) != hipSuccess) return FDBCS_E_NOMEM;
        view_cap_ = nc;
    }
    lview_ = UnpackOut{(int64_t*)view_, (int32_t*)(view_ + o_ro), (int32_t*)(view_ + o_wo),
                       (uint64_t*)(view_ + o_ko), (uint32_t*)(view_ + o_kl)};
    for (int i = 0; i < 8; i++) prog_[i] = 0;  // LV_RUNNING, nothing published (read by the kernel launched next)
    __atomic_thread_fence(__ATOMIC_SEQ_CST);
    if (bar_) _mm_sfence();
    lcaps_ = caps;
    next_pub_ = pub_every_;
    if (borrow_ && (r = start_helpers(true))) return r;  // (the caps above size the helpers' buffers)  // live borrowed: the helpers publish to the kernel
    live_ = true;
    live_broken_ = false;
    began_live_ = true;
    return FDBCS_OK;
}

// The helpers of a borrowed batch (lb_work), spinning until the first chunk
// is added.  live: they publish to the live kernel; else they send the
// finished prefix to the device on the copy stream, every LB_COPY_MIN bytes,
// and detectConflicts ingests the batch whole from device memory (the live
// kernel's reads of the records over PCIe were slower than these copies
// once the adds no longer paced it).
int TxnStage::start_helpers(bool live) {
    if (!pool_ && host_threads() > 1) pool_ = new HostPool(host_threads());
    if (!pool_) return FDBCS_E_STATE;
    int r;
    if ((r = grow_brec((int64_t)lcaps_.T + LB_CHUNK))) return r;
    if (!lbs_) lbs_ = new LbShared();
    lbs_->reset((int64_t)lcaps_.T / LB_CHUNK + 2);
    lbs_->fn = [this](int) { lb_work(); };
    lb_live_ = live;
    sent_ = 0;
    pool_->start(&lbs_->fn, 1 + std::min(lb_helpers(), pool_->size() - 1));
    lb_ = true;
    return FDBCS_OK;
}

int TxnStage::begin_helpers(const LiveCaps& caps) {
    if (!open_ || T_ || live_ || !borrow_) return FDBCS_E_STATE;
    int r;
    if ((r = grow(caps.T + 1, live_stream_bound(caps) + 8 * ((uint64_t)caps.T + 1)))) return r;
    lcaps_ = caps;
    return start_helpers(false);
}

int TxnStage::finish(fdbcs_batch_view& dv, StagedBatch* staged) {
    if (!open_) return FDBCS_E_STATE;
    open_ = false;
    if (lb_) {  // live borrowed: the last chunks, then the batch is live, refused, or repacked whole
        LbShared& S = *lbs_;
        S.added.store(T_, std::memory_order_release);
        S.fin.store(1, std::memory_order_release);
        pool_->wait();
        lb_ = false;
        if (S.bad.load() != INT64_MAX) {
            bad_txn_ = S.bad.load();
            live_cancel();
            return S.code.load();
        }
        if (S.stop.load()) {  // (over a capacity: repacked below, and ingested whole)
            live_cancel();
            _mm_sfence();
            if (hipStreamSynchronize(copy_) != hipSuccess) return FDBCS_E_HIP;  // (helpers' copies read the stream)
            sent_ = 0;
        } else {
            used_ = S.cursor;
            K_ = S.keys.load();
            borrow_ = false;  // (the stream and the offsets are complete: finish as a copied batch)
        }
    }
    if (borrow_) {
        _mm_sfence();  // (the adds' non-temporal stores, before the workers read them)
        const int r = pack_borrowed();
        if (r) return r;
    }
    bool go_live = false;
    // (the detect sizes nothing anew for a live batch: run_batch refuses one
    // whose stream or key bytes outgrew what live_begin sized its buffers
    // for.  live_check keeps every add within the capacities and the bound
    // counts every publish's padding, so this cannot trip; should it, the
    // batch falls back to the whole-stream ingest here instead -- ADVICE r05)
    if (live_ && !live_broken_ &&
        std::max<uint64_t>(used_ + 144, key_total()) > std::max<uint64_t>(lcaps_.key_bytes, live_stream_bound(lcaps_)))
        live_cancel();
    if (live_ && !live_broken_ && staged && pad_published()) {
        // the final word: the kernel finishes the last groups and leaves
        prog_[3] = (uint64_t)T_;
        prog_[4] = (uint64_t)R_;
        prog_[5] = (uint64_t)W_;
        prog_[1] = used_;
        if (bar_) _mm_sfence();
        // the published word itself says final (LV_FINAL_BIT): the kernel's
        // poller sees the last T and bytes in the one word it polls, a PCIe
        // round trip sooner than by reading [3] and [1] after the state
        __atomic_store_n(&prog_[0], LV_FINAL_BIT | (uint64_t)used_ << 20 | (uint64_t)T_, __ATOMIC_RELEASE);
        __atomic_store_n(&prog_[2], (uint64_t)LV_FINAL, __ATOMIC_RELEASE);
        // Did the kernel give up first (its timeout: e.g. an add phase stalled
        // for seconds behind another engine's hipFree)?  Store, full fence,
        // load here; mark, fence, load in the poller (k_live_ingest): one of
        // the two sees the other.  Marked: ingest the whole stream below (its
        // k_live_reset undoes whatever the kernel did).
        __atomic_thread_fence(__ATOMIC_SEQ_CST);
        if (__atomic_load_n(&prog_[6], __ATOMIC_ACQUIRE)) {
            timeouts_++;
            live_broken_ = true;
        } else {
            go_live = true;
        }
    }
    if (go_live) {
        live_ = false;
        dv = fdbcs_batch_view{};
        dv.txn_count = (int32_t)T_;
        dv.read_count = (int32_t)R_;
        dv.write_count = (int32_t)W_;
        dv.snapshot = lview_.snap;
        dv.read_off = lview_.ro;
        dv.write_off = lview_.wo;
        dv.key_off = lview_.koff;
        dv.key_len = lview_.klen;
        dv.key_bytes = pin_dev_;  // (the stream itself, host-mapped: only the rare view readers go there)
        dv.key_bytes_len = used_;
        *staged = StagedBatch{};
        staged->stream = pin_dev_;
        staged->toff = toff_dev_;
        staged->view = lview_;
        staged->live = true;
        return FDBCS_OK;
    }
    const bool failed = live_;  // (a live batch cancelled on the way: ingested whole below)
    live_cancel();
    live_ = false;
    const uint64_t* dtoff = toff_;
    if (bar_) {
        // the records and offsets are in device memory already: drain the
        // write-combined stores before the launches that read them
        _mm_sfence();
    } else {
    // the record offsets go after the records (8-byte aligned: records are),
    // and the rest of the stream in one copy
    const uint64_t o_toff = used_;
    dtoff = reinterpret_cast<const uint64_t*>(dev_ + o_toff);
    early_at_ = early_ && used_ > early_ ? used_ - early_ : ~0ull;  // (the next batch's extra chunk)
    if (T_ && !toff_in_stream_) memcpy(pin_ + o_toff, toff_, (size_t)T_ * 8);
    const uint64_t end = o_toff + 8 * (uint64_t)T_;
    if (pull_rest()) {
        // the chunks already sent: their last copy's event (recorded at the
        // copy, long complete by now); the rest: read by the engine's queue
        if (chunk_sent_ && hipStreamWaitEvent(stream_, copied_, 0) != hipSuccess) return FDBCS_E_HIP;
        if (end > sent_) launch_pull(pin_dev_ + sent_, dev_ + sent_, end - sent_, stream_);
        sent_ = end;
    } else {
        // (measured and kept: the rest on the copy stream too -- sending it on the
        // conflict set's stream, right before the kernels, was ~12 us slower)
        if (end > sent_ &&
            hipMemcpyAsync(dev_ + sent_, pin_ + sent_, end - sent_, hipMemcpyHostToDevice, copy_) != hipSuccess)
            return FDBCS_E_HIP;
        sent_ = end;
        if (hipEventRecord(copied_, copy_) != hipSuccess || hipStreamWaitEvent(stream_, copied_, 0) != hipSuccess)
            return FDBCS_E_HIP;
    }
    }
    // the view's arrays: snapshot [T] | read_off [T+1] | write_off [T+1] | key_off [2R+2W] | key_len [2R+2W]
    auto al = [](uint64_t x) { return (x + 15) & ~uint64_t(15); };
    const int64_t slots = 2 * (R_ + W_);
    const uint64_t o_ro = al(8 * T_), o_wo = al(o_ro + 4 * (T_ + 1)), o_ko = al(o_wo + 4 * (T_ + 1)),
                   o_kl = al(o_ko + 8 * slots), total = al(o_kl + 4 * slots) + 16;
    if (total > view_cap_) {
        if (view_) {
            sync();
            hipFree(view_);
            view_ = nullptr;
        }
        const uint64_t nc = std::max<uint64_t>(total, 2 * view_cap_);
        view_cap_ = 0;
        if (hipMalloc((void**)&view_, nc) != hipSuccess) return FDBCS_E_NOMEM;
        view_cap_ = nc;
    }
    dv = fdbcs_batch_view{};
    dv.txn_count = (int32_t)T_;
    dv.read_count = (int32_t)R_;
    dv.write_count = (int32_t)W_;
    dv.snapshot = (const int64_t*)view_;
    dv.read_off = (const int32_t*)(view_ + o_ro);
    dv.write_off = (const int32_t*)(view_ + o_wo);
    dv.key_off = (const uint64_t*)(view_ + o_ko);
    dv.key_len = (const uint32_t*)(view_ + o_kl);
    dv.key_bytes = dev_;
    dv.key_bytes_len = used_;
    const UnpackOut out{(int64_t*)dv.snapshot, (int32_t*)dv.read_off, (int32_t*)dv.write_off, (uint64_t*)dv.key_off,
                        (uint32_t*)dv.key_len};
    static const bool separate = getenv("FDBCS_SEPARATE_UNPACK") != nullptr;  // (A/B measurements)
    if (staged && !separate) {
        *staged = StagedBatch{dev_, dtoff, out};
        staged->live_failed = failed;
        return FDBCS_OK;
    }
    if (staged) {
        *staged = StagedBatch{};
        staged->live_failed = failed;
    }
    launch_unpack(dev_, dtoff, (int)T_, (int)R_, (int)W_, out, stream_);
    return FDBCS_OK;
}

}  // namespace fdbcs_dev
