// resolver_loop.cpp -- the bench's Resolver window (fdbwl_run_resolver) in a
// bare process (no Python, no torch), to separate the library's host cost
// from the interpreter's environment.
//   g++ -O2 -I include -o scripts/micro/resolver_loop scripts/micro/resolver_loop.cpp \
//       -L foundationdb_amd -lfdbcs -lfdbcs_workload -Wl,-rpath,$PWD/foundationdb_amd
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "../../foundationdb_amd/csrc/workload.h"

int main(int argc, char** argv) {
    const int prefill = argc > 1 ? atoi(argv[1]) : 300, steps = argc > 2 ? atoi(argv[2]) : 60;
    const int cfg = argc > 3 ? atoi(argv[3]) : 2;
    fdbcs* cs = nullptr;
    fdbcs_config c{};
    c.device = 0;
    c.max_history = 30000000;
    if (fdbcs_create(&cs, 0, &c)) return 1;
    fdbwl* g = fdbwl_create(cfg, 0, 0);
    if (fdbwl_prefill(g, cs, 0, prefill)) return 2;
    for (int rep = 0; rep < 3; rep++) {
        fdbwl_run* r = fdbwl_run_prepare(g, prefill + rep * steps, steps);
        std::vector<double> us(steps), add(steps);
        if (fdbwl_run_resolver(r, cs, us.data(), add.data(), nullptr)) return 3;
        double a = 0, b = 0;
        for (int i = 0; i < steps; i++) a += us[i], b += add[i];
        printf("rep %d: %.1f us per batch, add %.1f us, H %lld\n", rep, a / steps, b / steps,
               (long long)fdbcs_history_size(cs));
        fdbwl_run_destroy(r);
    }
    fdbcs_destroy(cs);
    return 0;
}
