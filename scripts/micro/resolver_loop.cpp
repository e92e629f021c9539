// resolver_loop.cpp -- the bench's Resolver window (fdbwl_run_resolver) in a
// bare process (no Python, no torch), to separate the library's host cost
// from the interpreter's environment.
//   g++ -O2 -I include -o scripts/micro/resolver_loop scripts/micro/resolver_loop.cpp \
//       -L foundationdb_amd -lfdbcs -lfdbcs_workload -Wl,-rpath,$PWD/foundationdb_amd
#include <chrono>
#include <cstdio>
#include <cstring>
#include <cstdlib>
#include <vector>

#include "../../foundationdb_amd/csrc/workload.h"

int main(int argc, char** argv) {
    const int prefill = argc > 1 ? atoi(argv[1]) : 300, steps = argc > 2 ? atoi(argv[2]) : 60;
    const int cfg = argc > 3 ? atoi(argv[3]) : 2;
    const bool add_only = argc > 4 && atoi(argv[4]);  // time fdbcs_batch_add alone (no detect)
    fdbcs* cs = nullptr;
    fdbcs_config c{};
    c.device = 0;
    c.max_history = 30000000;
    if (fdbcs_create(&cs, 0, &c)) return 1;
    fdbwl* g = fdbwl_create(cfg, 0, 0);
    if (fdbwl_prefill(g, cs, 0, prefill)) return 2;
    if (argc > 5 && atoi(argv[5]) >= 2) {  // add_micro's synthetic point ranges through fdbcs_batch_add
        // (mode 3: one read in five a short range [k, k + 1..16), as config 2's)
        const bool mixed = atoi(argv[5]) == 3;
        const int T = 5000;
        std::vector<uint8_t> bytes((size_t)T * 7 * 34);
        std::vector<fdbcs_range> rd(T * 5), wr(T * 2);
        uint64_t x = 88172645463325252ull;
        for (int r = 0; r < T * 7; r++) {
            uint8_t* p = &bytes[(size_t)r * 34];
            for (int k = 0; k < 2; k++) {
                x ^= x << 13; x ^= x >> 7; x ^= x << 17;
                memcpy(p + 8 * k, &x, 8);
            }
            memcpy(p + 17, p, 16);
            p[33] = 0;
            fdbcs_range rg{p, 16, p + 17, 17};
            if (mixed && r < T * 5 && (x >> 40) % 5 == 0 && p[15] < 0xF0) {
                p[17 + 15] = (uint8_t)(p[15] + 1 + (x >> 50) % 15);
                rg.end_len = 16;
            }
            if (r < T * 5) rd[r] = rg; else wr[r - T * 5] = rg;
        }
        double a = 0;
        for (int i = 0; i < steps; i++) {
            const auto t0 = std::chrono::steady_clock::now();
            int st = fdbcs_batch_begin(cs);
            for (int t = 0; st == 0 && t < T; t++) st = fdbcs_batch_add(cs, 0, &rd[5 * t], 5, &wr[2 * t], 2);
            if (st) return 4;
            if (i >= 5) a += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        }
        printf("synthetic %s via fdbcs_batch_add: %.1f us\n", mixed ? "points + 1/5 short reads" : "points", a / (steps - 5));
        return 0;
    }
    if (argc > 5 && atoi(argv[5])) {  // the same batch over and over (warm caches and TLB)
        fdbwl_run* r = fdbwl_run_prepare(g, prefill, 1);
        double a = 0, x = 0;
        for (int i = 0; i < steps; i++) {
            if (fdbwl_run_adds(r, cs, &x)) return 3;
            if (i >= 5) a += x;
        }
        printf("same batch: add %.1f us\n", a / (steps - 5));
        return 0;
    }
    for (int rep = 0; rep < 3; rep++) {
        fdbwl_run* r = fdbwl_run_prepare(g, prefill + rep * steps, steps);
        std::vector<double> us(steps), add(steps);
        if (add_only) {
            if (fdbwl_run_adds(r, cs, add.data())) return 3;
        } else if (fdbwl_run_resolver(r, cs, us.data(), add.data(), nullptr)) {
            return 3;
        }
        double a = 0, b = 0;
        for (int i = 0; i < steps; i++) a += us[i], b += add[i];
        printf("rep %d: %.1f us per batch, add %.1f us, H %lld\n", rep, a / steps, b / steps,
               (long long)fdbcs_history_size(cs));
        fdbwl_run_destroy(r);
    }
    fdbcs_destroy(cs);
    return 0;
}
