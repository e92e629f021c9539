/*
 * ConflictSetShim.cpp -- drop-in replacement for fdbserver/SkipList.cpp.
 *
 * Implements the unchanged fdbserver/ConflictSet.h surface on the MI355X
 * conflict set behind include/fdbcs.h (libfdbcs.so), so that
 * fdbserver/Resolver.actor.cpp (:47 newConflictSet, :51 destroyConflictSet,
 * :140-153 ConflictBatch per batch) links against the GPU engine with no
 * other change.  fdbserver.actor.cpp:481,1349 calls skipListTest(), which
 * SkipList.cpp defined; this TU defines it too.  See INTEGRATION.md.
 *
 * One Resolver over G GPUs: with FDBCS_SHARDS=G (G > 1) newConflictSet()
 * builds one exact conflict set over G GPUs (include/fdbcs.h fdbcs_sharded_*,
 * SURVEY.md §8e) -- one worker thread per rank, each driving its GPU -- so
 * Resolver.actor.cpp:140-153 gets one resolver's verdicts from G GPUs with no
 * other change.  addTransaction checks the ranges (and throws, as with one
 * GPU) and publishes the transaction; the workers add it to their ranks while
 * the Resolver's loop goes on (under protocol B each keeps only the ranges on
 * its keys), so at detectConflicts only the last few adds and the detect
 * remain.  FDBCS_SHARD_PROTOCOL=a|b (default b); FDBCS_SHARD_COMM=host
 * exchanges through in-process host collectives (every rank may then share
 * one GPU: tests), else RCCL; FDBCS_SHARD_DEVICES lists the ranks' devices
 * (default 0..G-1); FDBCS_SHARD_BOUNDS lists the G-1 strictly increasing
 * split keys in hex (default: the first two key bytes split uniformly).
 *
 * A rank that fails mid-batch does not leave the others waiting in a
 * collective: the caller's thread sees its status, aborts every rank
 * (fdbcs_sharded_abort / the host barrier's abort flag) and throws, as the
 * reference's ASSERT ends the resolver role.
 *
 * ConflictSet.h leaves KeyInfo, TransactionInfo and ReadConflictRange
 * incomplete and names five private methods; they are defined here only as
 * far as the header's members need them (the batch lives in the engine's
 * pinned staging buffer, not in `points`).
 */
#include "fdbserver/ConflictSet.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <random>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "fdbcs.h"

struct KeyInfo {};
struct TransactionInfo {};
struct ReadConflictRange {};

namespace {
struct MultiGpu;
}

struct ConflictSet {
    fdbcs* h = nullptr;        // one GPU
    MultiGpu* multi = nullptr;  // or G GPUs as one resolver (FDBCS_SHARDS)
    std::vector<uint8_t> verdict;  // last batch (GetTooOldTransactions)
    // One GPU, borrowed batches (FDBCS_BORROW_ALWAYS; FDBCS_SHIM_BORROW=0
    // copies instead): the batch's ranges as fdbcs_range, kept until
    // detectConflicts returns (a ChunkLog never moves an entry)
    bool borrow = false;
    void* ranges = nullptr;  // ChunkLog<fdbcs_range>
    std::vector<std::unique_ptr<fdbcs_range[]>> big;
};

namespace {

// ASSERT -> internal_error() in the reference (flow/Error.h:86-90, code
// 4100 in flow/error_definitions.h:201); the resolver role dies on it and its
// trace names that code.  Inside fdbserver, ConflictSet.h's includes
// (fdbclient/CommitTransaction.h -> flow) define the internal_error() macro,
// so the shim throws the reference's own Error; a non-Error exception would
// reach the actor wrappers as unknown_error.  The stand-alone test build
// (tests/shim/stub, no flow) throws std::runtime_error instead.
[[noreturn]] void fail_internal(const std::string& msg) {
    fprintf(stderr, "fdbcs: %s\n", msg.c_str());
#ifdef internal_error
    throw internal_error();
#else
    throw std::runtime_error(msg);
#endif
}

void ok_or_throw(int status, const char* what) {
    if (status != FDBCS_OK) fail_internal(std::string(what) + " failed: " + fdbcs_strerror(status));
}

fdbcs_range to_range(const KeyRangeRef& r) {
    return fdbcs_range{r.begin.begin(), (uint32_t)r.begin.size(), r.end.begin(), (uint32_t)r.end.size()};
}

int keycmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {  // SkipList.cpp:113-120
    const int c = std::min(al, bl) ? memcmp(a, b, std::min(al, bl)) : 0;
    if (c) return c < 0 ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

// fdbcs_batch_add's per-transaction checks (include/fdbcs.h), on the caller's
// thread: the G-GPU mode refuses the same transactions, with the same
// exception, as one GPU does
int check_ranges(const fdbcs_range* r, int n) {
    for (int i = 0; i < n; i++)
        if (r[i].begin_len > FDBCS_MAX_KEY || r[i].end_len > FDBCS_MAX_KEY) return FDBCS_E_KEY;
    for (int i = 0; i < n; i++)
        if (keycmp(r[i].begin, r[i].begin_len, r[i].end, r[i].end_len) >= 0) return FDBCS_E_RANGE;
    return FDBCS_OK;
}

// Append-only storage whose elements never move (workers read published
// entries while the caller appends): fixed-size chunks behind a directory
// sized once.
template <class X>
struct ChunkLog {
    static constexpr size_t CH = 1 << 13, MAXCH = 1 << 14;  // up to 2^27 entries
    std::vector<std::unique_ptr<X[]>> ch;
    size_t n = 0;
    ChunkLog() : ch(MAXCH) {}
    X& operator[](size_t i) { return ch[i / CH][i % CH]; }
    const X& operator[](size_t i) const { return ch[i / CH][i % CH]; }
    // k contiguous free entries (k <= CH), moving to the next chunk if needed
    X* reserve(size_t k) {
        if (n % CH + k > CH) n = (n / CH + 1) * CH;
        if (n / CH >= MAXCH) fail_internal("fdbcs: batch too large for the shim's log");
        std::unique_ptr<X[]>& c = ch[n / CH];
        if (!c) c.reset(new X[CH]);
        X* p = &c[n % CH];
        n += k;
        return p;
    }
};

// the one-GPU set's range log (ConflictSet::ranges)
ChunkLog<fdbcs_range>& range_log(ConflictSet* cs) { return *static_cast<ChunkLog<fdbcs_range>*>(cs->ranges); }

// ---- G GPUs as one resolver ------------------------------------------------
// Rank g lives on worker thread g (its device context, its RCCL rank).  Jobs
// are started on every worker and waited for separately, so that a batch job
// (ConflictBatch construction .. detectConflicts) runs beside the caller's
// addTransaction calls.
struct TxnRec {
    int64_t snap;
    int32_t nr, nw;
    const fdbcs_range* rg;  // nr reads, then nw writes (borrowed keys, as the reference borrows them)
};

struct MultiGpu {
    int G = 0;
    int proto = FDBCS_PROTOCOL_B;
    bool host = false;
    std::vector<fdbcs_sharded*> sh;
    std::vector<std::thread> th;
    std::mutex m;
    std::condition_variable cv_job, cv_done;
    std::function<int(int)> job;
    uint64_t seq = 0;
    int pending = 0;
    bool quit = false;
    bool broken = false;  // a rank failed mid-batch and every rank was aborted
    std::vector<int> status;
    // the batch being published
    ChunkLog<TxnRec> txns;
    ChunkLog<fdbcs_range> ranges;
    std::vector<std::unique_ptr<fdbcs_range[]>> big;  // transactions with more ranges than a chunk
    std::atomic<int64_t> published{0};
    std::atomic<bool> closed{false}, cancel{false};
    int64_t now = 0, new_oldest = 0;
    bool open = false;  // a batch job is running
    std::vector<std::vector<uint8_t>> verd;  // per rank
    // in-process host collectives (FDBCS_SHARD_COMM=host)
    std::atomic<int> bar_count{0};
    std::atomic<int> bar_gen{0};
    std::atomic<bool> aborted{false};
    std::vector<const uint8_t*> pub;
    std::vector<std::vector<uint8_t>> tmp;
    void* comm_ctx = nullptr;  // HostComm[G] (the ranks' fdbcs_comm_ops contexts)

    // false: aborted while waiting (the collective then fails)
    bool barrier() {
        const int gen = bar_gen.load(std::memory_order_acquire);
        if (bar_count.fetch_add(1, std::memory_order_acq_rel) == G - 1) {
            bar_count.store(0, std::memory_order_relaxed);
            bar_gen.store(gen + 1, std::memory_order_release);
            return !aborted.load(std::memory_order_acquire);
        }
        for (int i = 0; bar_gen.load(std::memory_order_acquire) == gen; i++) {
            if (aborted.load(std::memory_order_acquire)) return false;
            if (i > 1000) std::this_thread::yield();
        }
        return !aborted.load(std::memory_order_acquire);
    }

    void start(std::function<int(int)> f) {
        {
            std::unique_lock<std::mutex> lk(m);
            job = std::move(f);
            pending = G;
            seq++;
            std::fill(status.begin(), status.end(), 0);
        }
        cv_job.notify_all();
    }

    // Wait for the job on every worker; the first nonzero status.  When a
    // rank has failed and the others are still running after a grace period,
    // they are waiting for it in a collective: abort every rank.
    int wait() {
        std::unique_lock<std::mutex> lk(m);
        auto failed = [&] {
            for (int g = 0; g < G; g++)
                if (status[g]) return true;
            return false;
        };
        while (pending) {
            cv_done.wait_for(lk, std::chrono::milliseconds(50), [&] { return pending == 0 || failed(); });
            if (pending && failed()) {
                if (!cv_done.wait_for(lk, std::chrono::milliseconds(200), [&] { return pending == 0; })) {
                    lk.unlock();
                    abort_all();
                    lk.lock();
                    cv_done.wait(lk, [&] { return pending == 0; });
                }
            }
        }
        for (int g = 0; g < G; g++)
            if (status[g]) return status[g];
        return FDBCS_OK;
    }

    int run(std::function<int(int)> f) {
        start(std::move(f));
        return wait();
    }

    // (a rank blocked in RCCL waits on an event behind the collective, which
    // ncclCommAbort ends; the host collectives' barrier sees `aborted`)
    void abort_all() {
        aborted.store(true, std::memory_order_release);
        cancel.store(true, std::memory_order_release);
        for (fdbcs_sharded* s : sh)
            if (s) fdbcs_sharded_abort(s);
        broken = true;
    }

    void worker(int g) {
        uint64_t seen = 0;
        for (;;) {
            std::function<int(int)> f;
            {
                std::unique_lock<std::mutex> lk(m);
                cv_job.wait(lk, [&] { return quit || seq != seen; });
                if (quit) return;
                seen = seq;
                f = job;
            }
            const int st = f(g);
            std::lock_guard<std::mutex> lk(m);
            status[g] = st;
            if (--pending == 0 || st) cv_done.notify_one();
        }
    }

    // ConflictBatch on every rank: add what the caller publishes until
    // detectConflicts closes the batch, then detect
    int batch_job(int g) {
        fdbcs_sharded* s = sh[g];
        int r = fdbcs_sharded_batch_begin(s);
        int64_t done = 0;
        for (int spins = 0; r == FDBCS_OK;) {
            const int64_t p = published.load(std::memory_order_acquire);
            if (done < p) {
                for (; r == FDBCS_OK && done < p; done++) {
                    const TxnRec& x = txns[(size_t)done];
                    r = fdbcs_sharded_batch_add(s, x.snap, x.rg, x.nr, x.rg + x.nr, x.nw);
                }
                spins = 0;
                continue;
            }
            if (cancel.load(std::memory_order_acquire)) return FDBCS_E_STATE;
            if (closed.load(std::memory_order_acquire) && done == published.load(std::memory_order_acquire)) break;
            if (++spins > 2000) std::this_thread::yield();
        }
        if (r) return r;
        verd[g].assign((size_t)done + 1, 0);
        if (inject_failure(g)) return FDBCS_E_NOMEM;
        return fdbcs_sharded_batch_detect(s, now, new_oldest, verd[g].data());
    }
    static bool inject_failure(int g);
};

// test hook (tests/test_shim.py): rank FDBCS_TEST_FAIL_RANK fails the
// FDBCS_TEST_FAIL_BATCH-th detectConflicts (0-based) without running it, as a
// rank whose allocation failed would, while the others enter the exchanges
bool MultiGpu::inject_failure(int g) {
    static const int rank = getenv("FDBCS_TEST_FAIL_RANK") ? atoi(getenv("FDBCS_TEST_FAIL_RANK")) : -1;
    static const int batch = getenv("FDBCS_TEST_FAIL_BATCH") ? atoi(getenv("FDBCS_TEST_FAIL_BATCH")) : 0;
    static std::atomic<int> seen{0};
    if (rank < 0 || g != rank) return false;
    return seen.fetch_add(1) == batch;
}

struct HostComm {
    MultiGpu* mg;
    int rank;
};

int host_allreduce_max(void* ctx, uint8_t* buf, uint64_t n) {
    HostComm* c = static_cast<HostComm*>(ctx);
    MultiGpu& mg = *c->mg;
    mg.pub[c->rank] = buf;
    if (!mg.barrier()) return 1;
    std::vector<uint8_t>& t = mg.tmp[c->rank];
    t.assign(buf, buf + n);
    for (int r = 0; r < mg.G; r++)
        for (uint64_t i = 0; i < n; i++) t[i] = std::max(t[i], mg.pub[r][i]);
    if (!mg.barrier()) return 1;  // every rank has read every buffer
    memcpy(buf, t.data(), n);
    return 0;
}

int host_allgather(void* ctx, const uint8_t* send, uint8_t* recv, uint64_t n) {
    HostComm* c = static_cast<HostComm*>(ctx);
    MultiGpu& mg = *c->mg;
    mg.pub[c->rank] = send;
    if (!mg.barrier()) return 1;
    for (int r = 0; r < mg.G; r++) memcpy(recv + r * n, mg.pub[r], n);
    return mg.barrier() ? 0 : 1;
}

std::vector<std::string> split_list(const char* s) {
    std::vector<std::string> out;
    std::string cur;
    for (const char* p = s; *p; p++) {
        if (*p == ',') {
            out.push_back(cur);
            cur.clear();
        } else {
            cur += *p;
        }
    }
    out.push_back(cur);
    return out;
}

std::vector<uint8_t> from_hex(const std::string& h) {
    auto nib = [&](char c) -> int {
        if (c >= '0' && c <= '9') return c - '0';
        if (c >= 'a' && c <= 'f') return c - 'a' + 10;
        if (c >= 'A' && c <= 'F') return c - 'A' + 10;
        fail_internal("FDBCS_SHARD_BOUNDS: '" + h + "' is not hex");
    };
    if (h.size() % 2) fail_internal("FDBCS_SHARD_BOUNDS: '" + h + "' has an odd number of hex digits");
    std::vector<uint8_t> out;
    for (size_t i = 0; i < h.size(); i += 2) out.push_back((uint8_t)(nib(h[i]) << 4 | nib(h[i + 1])));
    return out;
}

int device_ordinal() {
    // one Resolver process per GPU: FDBCS_DEVICE picks it (default: current device)
    const char* d = getenv("FDBCS_DEVICE");
    return d ? atoi(d) : -1;
}

// stop and join the workers, destroy the ranks, free mg (every exit path)
void free_multi(MultiGpu* mg) {
    if (!mg) return;
    if (!mg->th.empty()) {
        if (mg->open) {  // a batch job still running (its ConflictBatch never detected)
            mg->cancel.store(true, std::memory_order_release);
            mg->wait();
            mg->open = false;
        }
        mg->run([mg](int g) {
            fdbcs_sharded_destroy(mg->sh[g]);
            mg->sh[g] = nullptr;
            return 0;
        });
        {
            std::lock_guard<std::mutex> lk(mg->m);
            mg->quit = true;
        }
        mg->cv_job.notify_all();
        for (auto& t : mg->th) t.join();
    }
    delete[] static_cast<HostComm*>(mg->comm_ctx);
    delete mg;
}

MultiGpu* make_multi(int G) {
    std::unique_ptr<MultiGpu, void (*)(MultiGpu*)> mg(new MultiGpu, free_multi);
    mg->G = G;
    mg->sh.assign(G, nullptr);
    mg->status.assign(G, 0);
    mg->pub.assign(G, nullptr);
    mg->tmp.resize(G);
    mg->verd.resize(G);
    if (const char* p = getenv("FDBCS_SHARD_PROTOCOL")) {
        if (!strcmp(p, "a")) mg->proto = FDBCS_PROTOCOL_A;
        else if (!strcmp(p, "b")) mg->proto = FDBCS_PROTOCOL_B;
        else fail_internal("FDBCS_SHARD_PROTOCOL: a or b");
    }
    // split keys: G-1, strictly increasing (the header's requirement)
    std::vector<std::vector<uint8_t>> bounds;
    if (const char* b = getenv("FDBCS_SHARD_BOUNDS")) {
        for (const std::string& h : split_list(b)) bounds.push_back(from_hex(h));
    } else {
        for (int g = 1; g < G; g++) {
            const uint32_t v = (uint32_t)((uint64_t)g * 65536 / G);
            bounds.push_back({(uint8_t)(v >> 8), (uint8_t)v});
        }
    }
    if ((int)bounds.size() != G - 1) fail_internal("FDBCS_SHARD_BOUNDS: need G-1 keys");
    for (int g = 1; g + 1 < G; g++)
        if (keycmp(bounds[g - 1].data(), (uint32_t)bounds[g - 1].size(), bounds[g].data(), (uint32_t)bounds[g].size()) >= 0)
            fail_internal("FDBCS_SHARD_BOUNDS: split keys must increase strictly");
    std::vector<uint8_t> bb;
    std::vector<uint64_t> bo;
    std::vector<uint32_t> bl;
    for (auto& k : bounds) {
        bo.push_back(bb.size());
        bl.push_back((uint32_t)k.size());
        bb.insert(bb.end(), k.begin(), k.end());
    }
    bb.push_back(0);
    std::vector<int> dev(G);
    for (int g = 0; g < G; g++) dev[g] = g;
    if (const char* d = getenv("FDBCS_SHARD_DEVICES")) {
        const auto v = split_list(d);
        for (int g = 0; g < G; g++) dev[g] = atoi(v[g % v.size()].c_str());
    }
    const char* cm = getenv("FDBCS_SHARD_COMM");
    mg->host = cm && !strcmp(cm, "host");
    HostComm* hc = new HostComm[G];
    for (int g = 0; g < G; g++) hc[g] = HostComm{mg.get(), g};
    mg->comm_ctx = hc;
    MultiGpu* raw = mg.get();
    for (int g = 0; g < G; g++) mg->th.emplace_back([raw, g] { raw->worker(g); });
    // 1: every rank's engine (RCCL joined only once all of them exist, so a
    // rank that fails here leaves nobody waiting in ncclCommInitRank)
    const bool host = mg->host;
    const int proto = mg->proto;
    int st = mg->run([&, hc, raw](int g) {
        fdbcs_config cfg{};
        cfg.device = dev[g];
        fdbcs_comm_ops ops{&hc[g], host_allreduce_max, host_allgather};
        int r = fdbcs_sharded_create(&raw->sh[g], g, G, bb.data(), bo.data(), bl.data(), 0, &cfg, nullptr,
                                     host ? &ops : nullptr);
        if (r == FDBCS_OK) r = fdbcs_sharded_set_protocol(raw->sh[g], proto, 0);
        return r;
    });
    ok_or_throw(st, "newConflictSet (sharded)");
    if (!host) {  // 2: the RCCL communicator, every rank at once
        uint8_t id[FDBCS_COMM_ID_BYTES] = {};
        ok_or_throw(fdbcs_comm_unique_id(id), "newConflictSet (RCCL id)");
        st = mg->run([raw, &id](int g) { return fdbcs_sharded_comm_init(raw->sh[g], id); });
        ok_or_throw(st, "newConflictSet (RCCL init)");
    }
    return mg.release();
}

int shard_count() {
    const char* s = getenv("FDBCS_SHARDS");
    return s ? std::max(1, atoi(s)) : 1;
}

MultiGpu* usable(MultiGpu* mg) {
    if (mg->broken) fail_internal("fdbcs: a shard failed earlier; the conflict set is unusable");
    return mg;
}

}  // namespace

// The engine behind a ConflictSet, for the Resolver's load-metrics binding
// (fdbcs_sample_add_batch rolls the batch this conflict set last resolved, on
// that engine's device).  Not part of ConflictSet.h:
// Resolver.actor.cpp declares it next to its iopsSample.  G-GPU mode: rank
// 0's engine, which under protocol A holds the whole batch and under B its
// share (the sample then covers rank 0's keys).
fdbcs* conflictSetDevice(ConflictSet* cs) {
    if (!cs) return nullptr;
    return cs->multi ? fdbcs_sharded_local(cs->multi->sh[0]) : cs->h;
}

// newConflictSet() -- SkipList.cpp:956
ConflictSet* newConflictSet() {
    std::unique_ptr<ConflictSet> cs(new ConflictSet);
    if (const int G = shard_count(); G > 1) {
        cs->multi = make_multi(G);
        return cs.release();
    }
    fdbcs_config cfg{};
    cfg.device = device_ordinal();
    // FDBCS_SHIM_BORROW=1: the Resolver keeps a request's transactions until
    // detectConflicts returns (the reference's addTransaction borrows their
    // KeyRefs, SkipList.cpp:993-1004), so the engine may record pointers at
    // each add and pack the batch on helper threads (include/fdbcs.h
    // FDBCS_BORROW_ALWAYS).  Off by default here: skipListTest's 2,500-txn
    // batches measured slower borrowed (verdicts-only rate 15.7 against 25.4 M
    // txn/s copied) -- each detect then waits for the pack and its copy, where
    // the copied form's live ingest has encoded the batch during the adds.
    const char* b = getenv("FDBCS_SHIM_BORROW");
    cs->borrow = b && atoi(b);
    if (cs->borrow) {
        cfg.flags = FDBCS_BORROW_ALWAYS;
        cs->ranges = new ChunkLog<fdbcs_range>();
    }
    ok_or_throw(fdbcs_create(&cs->h, 0, &cfg), "newConflictSet");
    return cs.release();
}

// clearConflictSet() -- SkipList.cpp:957-959 (oldestVersion, removalKey kept)
void clearConflictSet(ConflictSet* cs, Version v) {
    if (MultiGpu* mg = cs->multi) {
        usable(mg);
        ok_or_throw(mg->run([mg, v](int g) { return fdbcs_sharded_clear(mg->sh[g], v); }), "clearConflictSet");
        return;
    }
    ok_or_throw(fdbcs_clear(cs->h, v), "clearConflictSet");
}

// destroyConflictSet() -- SkipList.cpp:960-962
void destroyConflictSet(ConflictSet* cs) {
    if (cs->multi) free_multi(cs->multi);
    else fdbcs_destroy(cs->h);
    delete static_cast<ChunkLog<fdbcs_range>*>(cs->ranges);
    delete cs;
}

// ConflictBatch ctor/dtor -- SkipList.cpp:964-971
ConflictBatch::ConflictBatch(ConflictSet* cs)
    : cs(cs), transactionCount(0), transactionConflictStatus(nullptr) {
    if (MultiGpu* mg = cs->multi) {
        usable(mg);
        if (mg->open) {  // (an earlier ConflictBatch never reached detectConflicts)
            mg->cancel.store(true, std::memory_order_release);
            mg->wait();
        }
        mg->txns.n = 0;
        mg->ranges.n = 0;
        mg->big.clear();
        mg->published.store(0, std::memory_order_relaxed);
        mg->closed.store(false, std::memory_order_relaxed);
        mg->cancel.store(false, std::memory_order_relaxed);
        mg->open = true;
        mg->start([mg](int g) { return mg->batch_job(g); });  // the ranks add as transactions arrive
        return;
    }
    if (cs->borrow) {
        range_log(cs).n = 0;
        cs->big.clear();
    }
    ok_or_throw(fdbcs_batch_begin(cs->h), "ConflictBatch");
}

// A batch dropped before detectConflicts (an exception in the Resolver's
// loop): the ranks stop adding before the borrowed keys go away.
ConflictBatch::~ConflictBatch() {
    MultiGpu* mg = cs->multi;
    if (mg && mg->open && mg->closed.load(std::memory_order_acquire) == false) {
        mg->cancel.store(true, std::memory_order_release);
        mg->wait();
        mg->open = false;
    }
}

// addTransaction -- SkipList.cpp:979-1008.  One GPU: the keys are copied into
// pinned staging now (the reference borrows them until detectConflicts).  G
// GPUs: the ranges are checked here (a bad one throws, as with one GPU, and
// the transaction is not part of the batch), then published; each rank's
// worker adds the transaction (its ranges on that rank's keys, protocol B)
// while this loop goes on.  The keys stay borrowed until detectConflicts.
void ConflictBatch::addTransaction(const CommitTransactionRef& tr) {
    const int nr = tr.read_conflict_ranges.size(), nw = tr.write_conflict_ranges.size();
    if (MultiGpu* mg = cs->multi) {
        fdbcs_range* rg;
        if ((size_t)(nr + nw) <= ChunkLog<fdbcs_range>::CH) {
            rg = mg->ranges.reserve((size_t)(nr + nw));
        } else {
            mg->big.emplace_back(new fdbcs_range[(size_t)(nr + nw)]);
            rg = mg->big.back().get();
        }
        int k = 0;
        for (const auto& r : tr.read_conflict_ranges) rg[k++] = to_range(r);
        for (const auto& w : tr.write_conflict_ranges) rg[k++] = to_range(w);
        ok_or_throw(check_ranges(rg, nr + nw), "addTransaction");
        const int64_t t = mg->published.load(std::memory_order_relaxed);
        *mg->txns.reserve(1) = TxnRec{tr.read_snapshot, nr, nw, rg};
        mg->published.store(t + 1, std::memory_order_release);
        transactionCount++;
        return;
    }
    if (cs->borrow) {  // the ranges into the batch's log, checked here (a bad one throws, as when copied)
        fdbcs_range* rg;
        if ((size_t)(nr + nw) <= ChunkLog<fdbcs_range>::CH) {
            rg = range_log(cs).reserve((size_t)std::max(nr + nw, 1));
        } else {
            cs->big.emplace_back(new fdbcs_range[(size_t)(nr + nw)]);
            rg = cs->big.back().get();
        }
        int k = 0;
        for (const auto& r : tr.read_conflict_ranges) rg[k++] = to_range(r);
        for (const auto& w : tr.write_conflict_ranges) rg[k++] = to_range(w);
        ok_or_throw(check_ranges(rg, nr + nw), "addTransaction");
        ok_or_throw(fdbcs_batch_add(cs->h, tr.read_snapshot, rg, nr, rg + nr, nw), "addTransaction");
        transactionCount++;
        return;
    }
    static thread_local std::vector<fdbcs_range> rr, wr;
    rr.clear();
    wr.clear();
    for (const auto& r : tr.read_conflict_ranges) rr.push_back(to_range(r));
    for (const auto& w : tr.write_conflict_ranges) wr.push_back(to_range(w));
    ok_or_throw(fdbcs_batch_add(cs->h, tr.read_snapshot, rr.data(), (int32_t)rr.size(), wr.data(),
                                (int32_t)wr.size()),
                "addTransaction");
    transactionCount++;
}

// detectConflicts -- SkipList.cpp:1163-1208.  Appends, like the reference,
// the ascending indices of committed transactions to nonConflicting and of
// tooOld ones to *tooOldTransactions.
void ConflictBatch::detectConflicts(Version now, Version newOldestVersion, vector<int>& nonConflicting,
                                    vector<int>* tooOldTransactions) {
    cs->verdict.assign((size_t)transactionCount, 0);
    if (MultiGpu* mg = cs->multi) {
        usable(mg);
        if (!mg->open) fail_internal("fdbcs: detectConflicts without an open ConflictBatch");
        mg->now = now;
        mg->new_oldest = newOldestVersion;
        mg->closed.store(true, std::memory_order_release);  // (now / new_oldest published with it)
        const int st = mg->wait();
        mg->open = false;
        ok_or_throw(st, "detectConflicts");
        memcpy(cs->verdict.data(), mg->verd[0].data(), (size_t)transactionCount);  // (identical on every rank)
    } else {
        ok_or_throw(fdbcs_batch_detect(cs->h, now, newOldestVersion, cs->verdict.data()), "detectConflicts");
    }
    for (int t = 0; t < transactionCount; t++) {
        if (cs->verdict[t] == FDBCS_COMMITTED) nonConflicting.push_back(t);
        else if (cs->verdict[t] == FDBCS_TOO_OLD && tooOldTransactions) tooOldTransactions->push_back(t);
    }
}

// GetTooOldTransactions -- SkipList.cpp:1155-1161 (no callers in the reference)
void ConflictBatch::GetTooOldTransactions(vector<int>& tooOldTransactions) {
    for (int t = 0; t < (int)cs->verdict.size(); t++)
        if (cs->verdict[t] == FDBCS_TOO_OLD) tooOldTransactions.push_back(t);
}

// `fdbserver -r skiplisttest` (fdbserver.actor.cpp:1348-1349) on the GPU
// conflict set, in the reference's shape (SkipList.cpp:1412-1507): 500
// batches of 5,000 ranges [setK(k), setK(k + 1 + U[0,10])) with k ~ U[0, 2e7)
// generated first (setK = 12 x '.' + the int big-endian, :909-922); then,
// timed, per batch: the transactions built (1 read + 1 write each, the keys
// copied into the batch's buffer, read_snapshot i -- the reference's
// g_buildTest), ConflictBatch + addTransaction x 2,500 (g_add),
// detectConflicts(i + 50, i) (g_detectConflicts).  "New conflict set" is the
// whole loop, as in the reference; "Detect only" the reference's detect time
// (history update included, from the stage-timed run), "Verdicts only" this
// build's early-returning detectConflicts.  "Skiplist only" and the per-stage
// counters (the reference's D.CheckRead + D.MergeWrite and PerfDoubleCounters,
// :91-111) come from the engine's per-stage HIP events in a second run of the
// same batches on a fresh conflict set (stage timing waits for each whole
// batch, which the first run's overlap of history update and next adds does
// not).  The reference's miniConflictSetTest (:1394-1410) checks its bitset;
// this build has none, so it is not repeated here.
void skipListTest() {
    printf("Skip list test (fdbcs, MI355X)\n");
    std::mt19937_64 rng(1);
    const int batches = 500, ranges = 5000;
    std::vector<uint8_t> keys((size_t)batches * ranges * 32);
    auto setK = [](uint8_t* p, uint32_t k) {
        memset(p, '.', 12);
        for (int i = 0; i < 4; i++) p[12 + i] = (uint8_t)(k >> (24 - 8 * i));
    };
    for (int i = 0; i < batches; i++) {
        for (int j = 0; j < ranges; j++) {
            uint8_t* p = &keys[((size_t)i * ranges + j) * 32];
            const uint32_t k = (uint32_t)(rng() % 20000000u), k2 = k + 1 + (uint32_t)(rng() % 11);
            setK(p, k);
            setK(p + 16, k2);
        }
    }
    printf("Test data generated\n  %d batches, %d/batch\nRunning\n", batches, ranges);
    using clk = std::chrono::steady_clock;
    auto secs = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
    // one pass of the reference's timed loop; stage: per-stage device time sums (or null)
    struct Pass {
        double total = 0, build = 0, add = 0, detect = 0;
        long accepted = 0, tcount = 0, cranges = 0;
        double stage[7] = {0, 0, 0, 0, 0, 0, 0};
        long long hist = 0;
    };
    auto run = [&](bool stage_timing) {
        Pass P;
        ConflictSet* cs = newConflictSet();
        if (stage_timing && cs->h) fdbcs_enable_stage_timing(cs->h, 1);
        const int readCount = 1, writeCount = 1;
        const auto start = clk::now();
        for (int i = 0; i < batches; i++) {
            auto t = clk::now();
            Arena buf;
            std::vector<uint8_t> kb((size_t)ranges * 32);  // the batch's own copy of its keys (KeyRangeRef(buf, r))
            std::vector<CommitTransactionRef> trs;
            for (int j = 0; j + readCount + writeCount <= ranges; j += readCount + writeCount) {
                CommitTransactionRef tr;
                for (int k = 0; k < readCount + writeCount; k++) {
                    const uint8_t* src = &keys[((size_t)i * ranges + j + k) * 32];
                    uint8_t* dst = &kb[(size_t)(j + k) * 32];
                    memcpy(dst, src, 32);
                    const KeyRangeRef r(StringRef(dst, 16), StringRef(dst + 16, 16));
                    if (k < readCount) tr.read_conflict_ranges.push_back(buf, r);
                    else tr.write_conflict_ranges.push_back(buf, r);
                }
                P.cranges += readCount + writeCount;
                tr.read_snapshot = i;
                trs.push_back(tr);
            }
            P.tcount += (long)trs.size();
            auto t1 = clk::now();
            P.build += secs(t, t1);
            std::vector<int> nonConflict;
            {
                ConflictBatch batch(cs);
                for (size_t j = 0; j < trs.size(); j++) batch.addTransaction(trs[j]);
                auto t2 = clk::now();
                P.add += secs(t1, t2);
                batch.detectConflicts(i + 50, i, nonConflict);
                P.detect += secs(t2, clk::now());
            }
            P.accepted += (long)nonConflict.size();
            if (stage_timing && cs->h) {
                double us[7];
                if (fdbcs_stage_times(cs->h, us, 7) == 7)
                    for (int s = 0; s < 7; s++) P.stage[s] += us[s] * 1e-6;
            }
        }
        P.total = secs(start, clk::now());
        if (MultiGpu* mg = cs->multi) {
            std::vector<long long> part(mg->G);
            mg->run([mg, &part](int g) {
                part[g] = (long long)fdbcs_history_size(fdbcs_sharded_local(mg->sh[g]));
                return 0;
            });
            for (long long x : part) P.hist += x;
        } else {
            P.hist = (long long)fdbcs_history_size(cs->h);
        }
        destroyConflictSet(cs);
        return P;
    };
    const Pass P = run(false);
    auto rate = [&](const char* name, double sec) {
        printf("%-18s%0.3f sec\n                  %0.3f Mtransactions/sec\n                  %0.3f Mkeys/sec\n", name,
               sec, P.tcount / sec / 1e6, P.cranges * 2 / sec / 1e6);
    };
    rate("New conflict set: ", P.total);
    const bool multi = shard_count() > 1;
    if (!multi) {  // per-stage device times: a second, stage-timed run on a fresh conflict set
        const Pass S = run(true);
        // "Detect only" is the reference's quantity (SkipList.cpp:1485-1487):
        // detectConflicts through mergeWriteConflictRanges and removeBefore
        // (:1184-1206) -- the stage-timed run waits for each whole batch.
        // "Verdicts only": detectConflicts as this build returns it to the
        // Resolver, at the verdicts, the history update running on behind them.
        rate("Detect only:      ", S.detect);
        rate("Verdicts only:    ", P.detect);
        rate("Skiplist only:    ", S.stage[1] + S.stage[4]);
        printf("Performance counters:\n");
        const char* names[] = {"Build", "Add", "Detect", "D.Sort", "D.CheckRead", "D.CheckIntraBatch",
                               "D.Combine", "D.MergeWrite", "D.RemoveBefore"};
        // (fdbcs_stage_times: [0] encode/sort, [1] read check, [2] intra-batch, [3] combine,
        // [4] merge, [5] compaction; the first three from the timed run)
        const double vals[] = {P.build, P.add, P.detect, S.stage[0], S.stage[1], S.stage[2], S.stage[3], S.stage[4],
                               S.stage[5]};
        for (int c = 0; c < 9; c++) printf("%20s: %0.6f\n", names[c], vals[c]);
        printf("(D.* : device time from HIP events, stage-timed second run; Build / Add / Detect: host time)\n");
    } else {
        rate("Verdicts only:    ", P.detect);  // (no stage-timed run across ranks: no "Detect only")
        printf("(%d GPUs as one resolver)\n", shard_count());
    }
    printf("%ld transactions accepted\n%lld entries in version history\n", P.accepted, P.hist);
}
