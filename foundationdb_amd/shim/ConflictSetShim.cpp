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
 * ConflictSet.h leaves KeyInfo, TransactionInfo and ReadConflictRange
 * incomplete and names five private methods; they are defined here only as
 * far as the header's members need them (the batch lives in the engine's
 * pinned staging buffer, not in `points`).
 */
#include "fdbserver/ConflictSet.h"

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <stdexcept>

#include "fdbcs.h"

struct KeyInfo {};
struct TransactionInfo {};
struct ReadConflictRange {};

struct ConflictSet {
    fdbcs* h = nullptr;
    std::vector<uint8_t> verdict;  // last batch (GetTooOldTransactions)
};

namespace {

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

}  // namespace

// The engine behind a ConflictSet, for the Resolver's load-metrics binding
// (fdbcs_sample_add_batch rolls the batch this conflict set last resolved;
// INTEGRATION.md §4.3).  Not part of ConflictSet.h: Resolver.actor.cpp
// declares it next to its iopsSample.
fdbcs* conflictSetDevice(ConflictSet* cs) { return cs ? cs->h : nullptr; }

// newConflictSet() -- SkipList.cpp:956
ConflictSet* newConflictSet() {
    ConflictSet* cs = new ConflictSet;
    fdbcs_config cfg{};
    cfg.device = device_ordinal();
    ok_or_throw(fdbcs_create(&cs->h, 0, &cfg), "newConflictSet");
    return cs;
}

// clearConflictSet() -- SkipList.cpp:957-959 (oldestVersion, removalKey kept)
void clearConflictSet(ConflictSet* cs, Version v) { ok_or_throw(fdbcs_clear(cs->h, v), "clearConflictSet"); }

// destroyConflictSet() -- SkipList.cpp:960-962
void destroyConflictSet(ConflictSet* cs) {
    fdbcs_destroy(cs->h);
    delete cs;
}

// ConflictBatch ctor/dtor -- SkipList.cpp:964-971
ConflictBatch::ConflictBatch(ConflictSet* cs)
    : cs(cs), transactionCount(0), transactionConflictStatus(nullptr) {
    ok_or_throw(fdbcs_batch_begin(cs->h), "ConflictBatch");
}

ConflictBatch::~ConflictBatch() {}

// addTransaction -- SkipList.cpp:979-1008.  Keys are copied into pinned
// staging now (the reference borrows them until detectConflicts).
void ConflictBatch::addTransaction(const CommitTransactionRef& tr) {
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
    ok_or_throw(fdbcs_batch_detect(cs->h, now, newOldestVersion, cs->verdict.data()), "detectConflicts");
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

// `fdbserver -r skiplisttest` (fdbserver.actor.cpp:1348-1349): the
// reference's micro-benchmark shape (SkipList.cpp:1412-1551: batches of 2,500
// transactions, one read and one write of 16-byte keys each) on the GPU
// conflict set.
void skipListTest() {
    ConflictSet* cs = newConflictSet();
    std::mt19937_64 rng(1);
    const int batches = 500, txns = 2500;
    std::vector<uint8_t> keys(4 * 16 * (size_t)txns);
    std::vector<fdbcs_range> rr(txns), wr(txns);
    std::vector<uint8_t> verdict(txns);
    double secs = 0;
    long committed = 0;
    for (int b = 0; b < batches; b++) {
        ok_or_throw(fdbcs_batch_begin(cs->h), "ConflictBatch");
        for (int t = 0; t < txns; t++) {
            uint8_t* k = &keys[(size_t)t * 64];
            for (int q = 0; q < 4; q++) {
                memset(k + 16 * q, '.', 12);
                const uint32_t v = (uint32_t)(rng() % 20000000u) + (q & 1) * (1 + (uint32_t)(rng() % 11));
                for (int i = 0; i < 4; i++) k[16 * q + 12 + i] = (uint8_t)(v >> (24 - 8 * i));
            }
            if (memcmp(k, k + 16, 16) >= 0) std::swap_ranges(k, k + 16, k + 16);
            if (memcmp(k + 32, k + 48, 16) >= 0) std::swap_ranges(k + 32, k + 48, k + 48);
            rr[t] = fdbcs_range{k, 16, k + 16, 16};
            wr[t] = fdbcs_range{k + 32, 16, k + 48, 16};
        }
        const auto t0 = std::chrono::steady_clock::now();
        for (int t = 0; t < txns; t++) ok_or_throw(fdbcs_batch_add(cs->h, b, &rr[t], 1, &wr[t], 1), "add");
        ok_or_throw(fdbcs_batch_detect(cs->h, b + 50, b, verdict.data()), "detect");
        secs += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        for (uint8_t v : verdict) committed += v == FDBCS_COMMITTED;
    }
    printf("fdbcs skipListTest: %d batches x %d txns: %.3f Mtxn/s, %ld committed, history %lld boundaries\n",
           batches, txns, batches * (double)txns / secs / 1e6, committed, (long long)fdbcs_history_size(cs->h));
    destroyConflictSet(cs);
}
