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
 * SURVEY.md §8e protocol A) -- one worker thread per rank, each driving its
 * GPU -- so Resolver.actor.cpp:140-153 gets one resolver's verdicts from G
 * GPUs with no other change.  FDBCS_SHARD_COMM=host exchanges through
 * in-process host collectives (every rank may then share one GPU: tests),
 * else RCCL; FDBCS_SHARD_DEVICES lists the ranks' devices (default 0..G-1);
 * FDBCS_SHARD_BOUNDS lists the G-1 split keys in hex (default: the first two
 * key bytes split uniformly).
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
};

namespace {

// ---- G GPUs as one resolver ------------------------------------------------
// Rank g lives on worker thread g (its device context, its RCCL rank).  The
// batch is recorded on the caller's thread (the ranges are borrowed until
// detectConflicts, as the reference borrows them, SkipList.cpp:979-1008) and
// every rank replays it at detectConflicts, in parallel.
struct MultiGpu {
    int G = 0;
    std::vector<fdbcs_sharded*> sh;
    std::vector<std::thread> th;
    // the job all workers run (one per call), and its completion
    std::mutex m;
    std::condition_variable cv_job, cv_done;
    std::function<int(int)> job;
    uint64_t seq = 0;
    int pending = 0;
    bool quit = false;
    std::vector<int> status;
    // the batch being recorded
    std::vector<int64_t> snap;
    std::vector<int32_t> nr, nw;
    std::vector<fdbcs_range> ranges;  // per txn: its reads, then its writes
    std::vector<std::vector<uint8_t>> verd;  // per rank
    // in-process host collectives (FDBCS_SHARD_COMM=host)
    std::atomic<int> bar_count{0};
    std::atomic<int> bar_gen{0};
    std::vector<const uint8_t*> pub;
    std::vector<std::vector<uint8_t>> tmp;
    void* comm_ctx = nullptr;  // HostComm[G] (the ranks' fdbcs_comm_ops contexts)

    void barrier() {
        const int gen = bar_gen.load(std::memory_order_acquire);
        if (bar_count.fetch_add(1, std::memory_order_acq_rel) == G - 1) {
            bar_count.store(0, std::memory_order_relaxed);
            bar_gen.store(gen + 1, std::memory_order_release);
            return;
        }
        for (int i = 0; bar_gen.load(std::memory_order_acquire) == gen; i++)
            if (i > 1000) std::this_thread::yield();
    }

    // run f(rank) on every worker; the first nonzero status
    int run(std::function<int(int)> f) {
        {
            std::unique_lock<std::mutex> lk(m);
            job = std::move(f);
            pending = G;
            seq++;
        }
        cv_job.notify_all();
        std::unique_lock<std::mutex> lk(m);
        cv_done.wait(lk, [&] { return pending == 0; });
        for (int g = 0; g < G; g++)
            if (status[g]) return status[g];
        return FDBCS_OK;
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
            if (--pending == 0) cv_done.notify_one();
        }
    }
};

struct HostComm {
    MultiGpu* mg;
    int rank;
};

int host_allreduce_max(void* ctx, uint8_t* buf, uint64_t n) {
    HostComm* c = static_cast<HostComm*>(ctx);
    MultiGpu& mg = *c->mg;
    mg.pub[c->rank] = buf;
    mg.barrier();
    std::vector<uint8_t>& t = mg.tmp[c->rank];
    t.assign(buf, buf + n);
    for (int r = 0; r < mg.G; r++)
        for (uint64_t i = 0; i < n; i++) t[i] = std::max(t[i], mg.pub[r][i]);
    mg.barrier();  // every rank has read every buffer
    memcpy(buf, t.data(), n);
    return 0;
}

int host_allgather(void* ctx, const uint8_t* send, uint8_t* recv, uint64_t n) {
    HostComm* c = static_cast<HostComm*>(ctx);
    MultiGpu& mg = *c->mg;
    mg.pub[c->rank] = send;
    mg.barrier();
    for (int r = 0; r < mg.G; r++) memcpy(recv + r * n, mg.pub[r], n);
    mg.barrier();
    return 0;
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
    std::vector<uint8_t> out;
    for (size_t i = 0; i + 1 < h.size(); i += 2) out.push_back((uint8_t)strtoul(h.substr(i, 2).c_str(), nullptr, 16));
    return out;
}

// ASSERT -> internal_error in the reference (flow/Error.h:86); the resolver
// role dies on it.  The shim throws so that the caller's error path runs.
void ok_or_throw(int status, const char* what) {
    if (status != FDBCS_OK) {
        fprintf(stderr, "fdbcs: %s failed: %s\n", what, fdbcs_strerror(status));
        throw std::runtime_error(fdbcs_strerror(status));
    }
}

fdbcs_range to_range(const KeyRangeRef& r) {
    return fdbcs_range{r.begin.begin(), (uint32_t)r.begin.size(), r.end.begin(), (uint32_t)r.end.size()};
}

int device_ordinal() {
    // one Resolver process per GPU: FDBCS_DEVICE picks it (default: current device)
    const char* d = getenv("FDBCS_DEVICE");
    return d ? atoi(d) : -1;
}

MultiGpu* make_multi(int G) {
    MultiGpu* mg = new MultiGpu;
    mg->G = G;
    mg->sh.assign(G, nullptr);
    mg->status.assign(G, 0);
    mg->pub.assign(G, nullptr);
    mg->tmp.resize(G);
    mg->verd.resize(G);
    // split keys
    std::vector<std::vector<uint8_t>> bounds;
    if (const char* b = getenv("FDBCS_SHARD_BOUNDS")) {
        for (const std::string& h : split_list(b)) bounds.push_back(from_hex(h));
    } else {
        for (int g = 1; g < G; g++) {
            const uint32_t v = (uint32_t)((uint64_t)g * 65536 / G);
            bounds.push_back({(uint8_t)(v >> 8), (uint8_t)v});
        }
    }
    if ((int)bounds.size() != G - 1) throw std::runtime_error("FDBCS_SHARD_BOUNDS: need G-1 keys");
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
    const bool host = cm && !strcmp(cm, "host");
    uint8_t id[FDBCS_COMM_ID_BYTES] = {};
    if (!host) ok_or_throw(fdbcs_comm_unique_id(id), "newConflictSet (RCCL id)");
    HostComm* hc = new HostComm[G];
    for (int g = 0; g < G; g++) hc[g] = HostComm{mg, g};
    mg->comm_ctx = hc;
    for (int g = 0; g < G; g++) mg->th.emplace_back([mg, g] { mg->worker(g); });
    // every rank joins at once (ncclCommInitRank blocks until all have)
    const int st = mg->run([&, hc](int g) {
        fdbcs_config cfg{};
        cfg.device = dev[g];
        fdbcs_comm_ops ops{&hc[g], host_allreduce_max, host_allgather};
        return fdbcs_sharded_create(&mg->sh[g], g, G, bb.data(), bo.data(), bl.data(), 0, &cfg, host ? nullptr : id,
                                    host ? &ops : nullptr);
    });
    ok_or_throw(st, "newConflictSet (sharded)");
    return mg;
}

void free_multi(MultiGpu* mg) {
    mg->run([mg](int g) {
        fdbcs_sharded_destroy(mg->sh[g]);
        return 0;
    });
    {
        std::lock_guard<std::mutex> lk(mg->m);
        mg->quit = true;
    }
    mg->cv_job.notify_all();
    for (auto& t : mg->th) t.join();
    delete[] static_cast<HostComm*>(mg->comm_ctx);
    delete mg;
}

int shard_count() {
    const char* s = getenv("FDBCS_SHARDS");
    return s ? std::max(1, atoi(s)) : 1;
}

}  // namespace

// The engine behind a ConflictSet, for the Resolver's load-metrics binding
// (fdbcs_sample_add_batch rolls the batch this conflict set last resolved;
// INTEGRATION.md §4.3).  Not part of ConflictSet.h: Resolver.actor.cpp
// declares it next to its iopsSample.
fdbcs* conflictSetDevice(ConflictSet* cs) {
    if (!cs) return nullptr;
    return cs->multi ? fdbcs_sharded_local(cs->multi->sh[0]) : cs->h;  // (every rank holds the whole batch)
}

// newConflictSet() -- SkipList.cpp:956
ConflictSet* newConflictSet() {
    ConflictSet* cs = new ConflictSet;
    if (const int G = shard_count(); G > 1) {
        cs->multi = make_multi(G);
        return cs;
    }
    fdbcs_config cfg{};
    cfg.device = device_ordinal();
    ok_or_throw(fdbcs_create(&cs->h, 0, &cfg), "newConflictSet");
    return cs;
}

// clearConflictSet() -- SkipList.cpp:957-959 (oldestVersion, removalKey kept)
void clearConflictSet(ConflictSet* cs, Version v) {
    if (MultiGpu* mg = cs->multi) {
        ok_or_throw(mg->run([mg, v](int g) { return fdbcs_sharded_clear(mg->sh[g], v); }), "clearConflictSet");
        return;
    }
    ok_or_throw(fdbcs_clear(cs->h, v), "clearConflictSet");
}

// destroyConflictSet() -- SkipList.cpp:960-962
void destroyConflictSet(ConflictSet* cs) {
    if (cs->multi) free_multi(cs->multi);
    else fdbcs_destroy(cs->h);
    delete cs;
}

// ConflictBatch ctor/dtor -- SkipList.cpp:964-971
ConflictBatch::ConflictBatch(ConflictSet* cs)
    : cs(cs), transactionCount(0), transactionConflictStatus(nullptr) {
    if (MultiGpu* mg = cs->multi) {
        mg->snap.clear();
        mg->nr.clear();
        mg->nw.clear();
        mg->ranges.clear();
        return;
    }
    ok_or_throw(fdbcs_batch_begin(cs->h), "ConflictBatch");
}

ConflictBatch::~ConflictBatch() {}

// addTransaction -- SkipList.cpp:979-1008.  Keys are copied into pinned
// staging now (the reference borrows them until detectConflicts).
void ConflictBatch::addTransaction(const CommitTransactionRef& tr) {
    if (MultiGpu* mg = cs->multi) {  // recorded; every rank replays it at detectConflicts
        for (const auto& r : tr.read_conflict_ranges) mg->ranges.push_back(to_range(r));
        for (const auto& w : tr.write_conflict_ranges) mg->ranges.push_back(to_range(w));
        mg->snap.push_back(tr.read_snapshot);
        mg->nr.push_back((int32_t)tr.read_conflict_ranges.size());
        mg->nw.push_back((int32_t)tr.write_conflict_ranges.size());
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
        const int T = transactionCount;
        const int st = mg->run([mg, T, now, newOldestVersion](int g) {
            fdbcs_sharded* sh = mg->sh[g];
            int r = fdbcs_sharded_batch_begin(sh);
            size_t o = 0;
            for (int t = 0; r == FDBCS_OK && t < T; t++) {
                const fdbcs_range* rd = mg->ranges.data() + o;
                r = fdbcs_sharded_batch_add(sh, mg->snap[t], rd, mg->nr[t], rd + mg->nr[t], mg->nw[t]);
                o += (size_t)mg->nr[t] + mg->nw[t];
            }
            mg->verd[g].assign((size_t)T + 1, 0);
            if (r == FDBCS_OK) r = fdbcs_sharded_batch_detect(sh, now, newOldestVersion, mg->verd[g].data());
            return r;
        });
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
// conflict set, in the reference's shape (SkipList.cpp:1412-1551): 500
// batches of 5,000 ranges [setK(k), setK(k + 1 + U[0,10])) with k ~ U[0, 2e7),
// setK = 12 x '.' + the int big-endian (:909-922); each batch is 2,500
// transactions of 1 read + 1 write with read_snapshot i, then
// ConflictBatch + addTransaction x 2,500 + detectConflicts(i + 50, i).  The
// transactions are built outside the timed part (the reference's g_buildTest
// is inside its "New conflict set" figure; "Detect only" matches this one).
// The reference's miniConflictSetTest (:1394-1410) checks its bitset; this
// build has none, so it is not repeated here.
void skipListTest() {
    printf("Skip list test (fdbcs, MI355X)\n");
    ConflictSet* cs = newConflictSet();
    std::mt19937_64 rng(1);
    const int batches = 500, ranges = 5000, txns = ranges / 2;
    std::vector<uint8_t> keys((size_t)batches * ranges * 32);
    auto setK = [](uint8_t* p, uint32_t k) {
        memset(p, '.', 12);
        for (int i = 0; i < 4; i++) p[12 + i] = (uint8_t)(k >> (24 - 8 * i));
    };
    Arena arena;
    std::vector<CommitTransactionRef> trs((size_t)batches * txns);
    for (int i = 0; i < batches; i++) {
        for (int j = 0; j < ranges; j++) {
            uint8_t* p = &keys[((size_t)i * ranges + j) * 32];
            const uint32_t k = (uint32_t)(rng() % 20000000u), k2 = k + 1 + (uint32_t)(rng() % 11);
            setK(p, k);
            setK(p + 16, k2);
        }
        for (int t = 0; t < txns; t++) {
            const uint8_t* rd = &keys[((size_t)i * ranges + 2 * t) * 32];
            const uint8_t* wr = rd + 32;
            CommitTransactionRef& tr = trs[(size_t)i * txns + t];
            tr.read_conflict_ranges.push_back(arena, KeyRangeRef(StringRef(rd, 16), StringRef(rd + 16, 16)));
            tr.write_conflict_ranges.push_back(arena, KeyRangeRef(StringRef(wr, 16), StringRef(wr + 16, 16)));
            tr.read_snapshot = i;
        }
    }
    printf("Test data generated\n  %d batches, %d/batch\nRunning\n", batches, ranges);
    double add = 0, detect = 0;
    long accepted = 0;
    for (int i = 0; i < batches; i++) {
        std::vector<int> nonConflict;
        const auto t0 = std::chrono::steady_clock::now();
        ConflictBatch batch(cs);
        for (int t = 0; t < txns; t++) batch.addTransaction(trs[(size_t)i * txns + t]);
        const auto t1 = std::chrono::steady_clock::now();
        batch.detectConflicts(i + 50, i, nonConflict);
        const auto t2 = std::chrono::steady_clock::now();
        add += std::chrono::duration<double>(t1 - t0).count();
        detect += std::chrono::duration<double>(t2 - t1).count();
        accepted += (long)nonConflict.size();
    }
    const double tcount = (double)batches * txns, keys2 = tcount * 4;
    printf("New conflict set: %0.3f sec\n                  %0.3f Mtransactions/sec\n                  %0.3f Mkeys/sec\n",
           add + detect, tcount / (add + detect) / 1e6, keys2 / (add + detect) / 1e6);
    printf("Detect only:      %0.3f sec\n                  %0.3f Mtransactions/sec\n                  %0.3f Mkeys/sec\n",
           detect, tcount / detect / 1e6, keys2 / detect / 1e6);
    long long hist = 0;
    if (MultiGpu* mg = cs->multi) {
        std::vector<long long> part(mg->G);
        mg->run([mg, &part](int g) {
            part[g] = (long long)fdbcs_history_size(fdbcs_sharded_local(mg->sh[g]));
            return 0;
        });
        for (long long x : part) hist += x;
        printf("(%d GPUs as one resolver)\n", mg->G);
    } else {
        hist = (long long)fdbcs_history_size(cs->h);
    }
    printf("%ld transactions accepted\n%lld entries in version history\n", accepted, hist);
    destroyConflictSet(cs);
}
