// Drives the ConflictSet.h drop-in (ConflictSetShim.cpp) exactly as
// Resolver.actor.cpp:140-153 does: per batch, construct a ConflictBatch,
// addTransaction x T, detectConflicts(now, newOldest, commitList, &tooOldList).
// Input/output are flat binary files written / read by tests/test_shim.py.
//   in : i32 nbatch; per batch: i64 now, i64 new_oldest, i32 T; per txn:
//        i64 snapshot, i32 nreads, i32 nwrites, then each range as
//        u32 len, bytes (begin) and u32 len, bytes (end)
//   out: per batch: i32 n, n x i32 (nonConflicting); i32 m, m x i32 (tooOld)
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <string>
#include <vector>

#include "fdbserver/ConflictSet.h"
#include "fdbcs.h"

void skipListTest();
fdbcs* conflictSetDevice(ConflictSet* cs);  // ConflictSetShim.cpp (the Resolver's load-metrics binding)

template <class T>
static T rd(FILE* f) {
    T x;
    if (fread(&x, sizeof x, 1, f) != 1) exit(3);
    return x;
}

static KeyRangeRef kr(const std::string& b, const std::string& e) {
    return KeyRangeRef(KeyRef((const uint8_t*)b.data(), (int)b.size()), KeyRef((const uint8_t*)e.data(), (int)e.size()));
}

// "errors": a batch whose middle transaction has begin >= end, then one with
// a key over FDBCS_MAX_KEY: addTransaction throws for it (with one GPU and
// with G), the others resolve
static int errors_mode() {
    ConflictSet* cs = newConflictSet();
    static const std::string a = "a", b = "b", c = "c", d = "d", e = "e", f = "f", big(30002, 'x');
    for (int round = 0; round < 2; round++) {
        CommitTransactionRef t0, bad, t2;
        t0.read_conflict_ranges.push_back(kr(a, b));
        t0.write_conflict_ranges.push_back(kr(c, d));
        t0.read_snapshot = 5;
        if (round == 0) bad.read_conflict_ranges.push_back(kr(b, b));
        else bad.write_conflict_ranges.push_back(kr(a, big));
        t2.write_conflict_ranges.push_back(kr(e, f));
        std::vector<int> nc;
        ConflictBatch batch(cs);
        batch.addTransaction(t0);
        try {
            batch.addTransaction(bad);
            printf("accepted\n");
        } catch (const std::exception& x) {
            printf("refused: %s\n", x.what());
        }
        batch.addTransaction(t2);
        batch.detectConflicts(10 + round, 0, nc);
        printf("committed:");
        for (int i : nc) printf(" %d", i);
        printf("\n");
    }
    destroyConflictSet(cs);
    return 0;
}

// "rankfail": batches until detectConflicts throws (a shard made to fail by
// FDBCS_TEST_FAIL_RANK / _BATCH), then the set must refuse further batches
static int rankfail_mode() {
    ConflictSet* cs = newConflictSet();
    std::vector<std::string> keys, ends;  // (alive while the batches borrow them)
    for (int i = 0; i < 400; i++) {
        keys.push_back(std::string(1, (char)('a' + i % 26)) + std::to_string(i));
        ends.push_back(keys.back() + "~");
    }
    for (int i = 0; i < 5; i++) {
        try {
            std::vector<CommitTransactionRef> trs(100);
            for (int t = 0; t < 100; t++) {
                trs[t].read_conflict_ranges.push_back(kr(keys[4 * t], ends[4 * t]));
                trs[t].write_conflict_ranges.push_back(kr(keys[4 * t + 1], ends[4 * t + 1]));
                trs[t].read_snapshot = 100 * i;
            }
            std::vector<int> nc;
            ConflictBatch batch(cs);
            for (auto& t : trs) batch.addTransaction(t);
            batch.detectConflicts(100 * i + 50, 0, nc);
            printf("batch %d ok (%zu committed)\n", i, nc.size());
        } catch (const std::exception& x) {
            printf("threw at batch %d: %s\n", i, x.what());
            break;
        }
    }
    try {
        ConflictBatch again(cs);
        printf("usable\n");
    } catch (const std::exception& x) {
        printf("unusable: %s\n", x.what());
    }
    fflush(stdout);
    destroyConflictSet(cs);
    return 0;
}

// "sample IN OUT UNITS SEED": the resolve loop of main() with the Resolver's
// iopsSample bound as INTEGRATION.md §4.3 binds it (fdbcs_sample_attach to
// conflictSetDevice once, fdbcs_sample_add_batch after each detectConflicts,
// a poll every third batch); OUT (text): every sample entry (hex key,
// metric), the queue size, getEstimate(allKeys) and two splitEstimates
static int sample_mode(const char* inp, const char* outp, long units, unsigned long seed) {
    FILE* in = fopen(inp, "rb");
    FILE* out = fopen(outp, "w");
    if (!in || !out) return 2;
    ConflictSet* cs = newConflictSet();
    fdbcs_sample* s = nullptr;
    if (fdbcs_sample_create(&s, units, seed) || fdbcs_sample_attach(s, conflictSetDevice(cs), 100)) return 4;
    const int nb = rd<int32_t>(in);
    for (int b = 0; b < nb; b++) {
        const int64_t now = rd<int64_t>(in), nold = rd<int64_t>(in);
        const int T = rd<int32_t>(in);
        std::vector<std::vector<uint8_t>> keep;
        std::vector<CommitTransactionRef> trs(T);
        for (int t = 0; t < T; t++) {
            trs[t].read_snapshot = rd<int64_t>(in);
            const int nr = rd<int32_t>(in), nw = rd<int32_t>(in);
            for (int k = 0; k < nr + nw; k++) {
                KeyRef ends[2];
                for (int q = 0; q < 2; q++) {
                    const uint32_t n = rd<uint32_t>(in);
                    keep.emplace_back(n + 1);
                    if (n && fread(keep.back().data(), 1, n, in) != n) return 3;
                    ends[q] = KeyRef(keep.back().data(), (int)n);
                }
                (k < nr ? trs[t].read_conflict_ranges : trs[t].write_conflict_ranges)
                    .push_back(KeyRangeRef(ends[0], ends[1]));
            }
        }
        std::vector<int> commitList, tooOldList;
        {
            ConflictBatch batch(cs);
            for (int t = 0; t < T; t++) batch.addTransaction(trs[t]);
            batch.detectConflicts(now, nold, commitList, &tooOldList);
        }
        if (fdbcs_sample_add_batch(s, conflictSetDevice(cs), nullptr, 100, 0.5 * b + 1.0, nullptr)) return 5;
        if (b % 3 == 2 && fdbcs_sample_poll(s, 0.5 * b)) return 6;
    }
    std::vector<uint8_t> k(70000);
    const int64_t n = fdbcs_sample_size(s);
    for (int64_t i = 0; i < n; i++) {
        int64_t m = 0;
        const int32_t len = fdbcs_sample_entry(s, i, k.data(), (uint32_t)k.size(), &m);
        if (len < 0) return 7;
        for (int32_t j = 0; j < len; j++) fprintf(out, "%02x", k[j]);
        fprintf(out, " %lld\n", (long long)m);
    }
    const uint8_t hi[2] = {0xff, 0xff};
    const int64_t total = fdbcs_sample_estimate(s, nullptr, 0, hi, 2);
    fprintf(out, "queue %lld\nestimate %lld\n", (long long)fdbcs_sample_queue_size(s), (long long)total);
    for (int front = 0; front < 2; front++) {
        const int32_t len = fdbcs_sample_split(s, nullptr, 0, hi, 2, total / 3, front, k.data(), (uint32_t)k.size());
        if (len < 0) return 8;
        fprintf(out, "split%d ", front);
        for (int32_t j = 0; j < len; j++) fprintf(out, "%02x", k[j]);
        fprintf(out, "\n");
    }
    destroyConflictSet(cs);  // (before its sample, as ~Resolver does)
    fdbcs_sample_destroy(s);
    fclose(out);
    fclose(in);
    return 0;
}

int main(int argc, char** argv) {
    if (argc == 6 && std::string(argv[1]) == "sample") return sample_mode(argv[2], argv[3], atol(argv[4]), strtoul(argv[5], nullptr, 0));
    if (argc == 2 && std::string(argv[1]) == "skiplisttest") {
        skipListTest();
        return 0;
    }
    if (argc == 2 && std::string(argv[1]) == "errors") return errors_mode();
    if (argc == 2 && std::string(argv[1]) == "rankfail") return rankfail_mode();
    if (argc != 3) return 2;
    FILE* in = fopen(argv[1], "rb");
    FILE* out = fopen(argv[2], "wb");
    if (!in || !out) return 2;
    ConflictSet* cs = newConflictSet();
    const int nb = rd<int32_t>(in);
    for (int b = 0; b < nb; b++) {
        const int64_t now = rd<int64_t>(in), nold = rd<int64_t>(in);
        const int T = rd<int32_t>(in);
        std::vector<std::vector<uint8_t>> keep;  // keys stay alive until detectConflicts returns
        std::vector<CommitTransactionRef> trs(T);
        for (int t = 0; t < T; t++) {
            trs[t].read_snapshot = rd<int64_t>(in);
            const int nr = rd<int32_t>(in), nw = rd<int32_t>(in);
            for (int k = 0; k < nr + nw; k++) {
                KeyRef ends[2];
                for (int q = 0; q < 2; q++) {
                    const uint32_t n = rd<uint32_t>(in);
                    keep.emplace_back(n + 1);
                    if (n && fread(keep.back().data(), 1, n, in) != n) return 3;
                    ends[q] = KeyRef(keep.back().data(), (int)n);
                }
                (k < nr ? trs[t].read_conflict_ranges : trs[t].write_conflict_ranges)
                    .push_back(KeyRangeRef(ends[0], ends[1]));
            }
        }
        std::vector<int> commitList, tooOldList;
        {
            ConflictBatch batch(cs);
            for (int t = 0; t < T; t++) batch.addTransaction(trs[t]);
            batch.detectConflicts(now, nold, commitList, &tooOldList);
        }
        const int32_t n = (int32_t)commitList.size(), m = (int32_t)tooOldList.size();
        fwrite(&n, 4, 1, out);
        fwrite(commitList.data(), 4, n, out);
        fwrite(&m, 4, 1, out);
        fwrite(tooOldList.data(), 4, m, out);
    }
    destroyConflictSet(cs);
    fclose(out);
    fclose(in);
    return 0;
}
