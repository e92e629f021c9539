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
#include <string>
#include <vector>

#include "fdbserver/ConflictSet.h"

void skipListTest();

template <class T>
static T rd(FILE* f) {
    T x;
    if (fread(&x, sizeof x, 1, f) != 1) exit(3);
    return x;
}

int main(int argc, char** argv) {
    if (argc == 2 && std::string(argv[1]) == "skiplisttest") {
        skipListTest();
        return 0;
    }
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
