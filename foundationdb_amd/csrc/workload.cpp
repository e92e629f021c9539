// workload.cpp -- deterministic synthetic batch generators (see workload.h).
#include "workload.h"

#include <dlfcn.h>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <thread>
#include <vector>

namespace {

struct Rng {  // xoshiro256**
    uint64_t s[4];
    static uint64_t splitmix(uint64_t& x) {
        uint64_t z = (x += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    explicit Rng(uint64_t seed) {
        for (auto& x : s) x = splitmix(seed);
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9;
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return r;
    }
    uint64_t uniform(uint64_t n) { return n ? next() % n : 0; }           // [0, n)
    int64_t range(int64_t a, int64_t b) { return a + (int64_t)uniform((uint64_t)(b - a + 1)); }  // [a, b]
    double u01() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
};

inline void put_be64(uint8_t* p, uint64_t x) {
    for (int i = 0; i < 8; i++) p[i] = (uint8_t)(x >> (56 - 8 * i));
}
inline void put_be32(uint8_t* p, uint32_t x) {
    for (int i = 0; i < 4; i++) p[i] = (uint8_t)(x >> (24 - 8 * i));
}

struct Shape {
    int reads, writes, stride;  // stride = bytes reserved per key slot
};

const int CHUNK = 1024;

}  // namespace

struct fdbwl {
    int config = 2;
    int T = 5000;
    int threads = 1;
    Shape shape{5, 2, 17};
    std::vector<double> zipf_cdf;
    // batch storage
    std::vector<int64_t> snap;
    std::vector<int32_t> roff, woff;
    std::vector<uint64_t> koff;
    std::vector<uint32_t> klen;
    std::vector<uint8_t> bytes;
    // config 4: the wide read ends at the S-th boundary after its begin in the
    // current history, answered by `succ` (the engine's
    // fdbcs_nth_after, or the oracle's); without it, a log-uniform fraction
    // of the tenant's key space
    fdbwl_succ_fn succ = nullptr;
    void* succ_ctx = nullptr;
    std::vector<int64_t> wide_step;  // per txn: S (0: no query)
};

namespace {

static const uint8_t kPath[56] = {
    '/', 'a', 'p', 'p', '/', 't', 'e', 'n', 'a', 'n', 't', 's', '/', 'o', 'r', 'd', 'e', 'r', 's', '/',
    'b', 'y', '-', 'c', 'u', 's', 't', 'o', 'm', 'e', 'r', '/', 'r', 'e', 'g', 'i', 'o', 'n', '/', 'e',
    'u', '-', 'w', 'e', 's', 't', '/', 'i', 'n', 'd', 'e', 'x', '/', 'v', '1', '/'};

// key slot s of the batch: bytes at s * stride
struct Writer {
    fdbwl* g;
    uint8_t* key(int64_t slot) { return g->bytes.data() + slot * g->shape.stride; }
    void set(int64_t slot, uint32_t len) {
        g->koff[slot] = (uint64_t)slot * g->shape.stride;
        g->klen[slot] = len;
    }
};

// 16-byte big-endian integer helpers for short reads [k, k + d]
void add128(uint8_t* k, uint64_t d) {
    for (int i = 15; i >= 0 && d; i--) {
        uint64_t x = (uint64_t)k[i] + (d & 0xFF);
        k[i] = (uint8_t)x;
        d = (d >> 8) + (x >> 8);
    }
}

void gen_chunk(fdbwl* g, int64_t index, int c0, int c1) {
    const int cfg = g->config;
    Rng rng(0x5EED0000ull + (uint64_t)(cfg == 50 ? 5 : cfg) * 1000ull + (uint64_t)index * 0x100000001B3ull +
            (uint64_t)(c0 / CHUNK) * 0x9E3779B97F4A7C15ull);
    Writer w{g};
    const int R = g->T * g->shape.reads;
    const int64_t now = cfg == 1 ? index + 50 : (cfg == 50 ? 100000 * (index + 1) : 10000000 + index * 10000);
    for (int t = c0; t < c1; t++) {
        // snapshot
        if (cfg == 1) g->snap[t] = index;
        else if (cfg == 50) g->snap[t] = 0;
        else if (rng.uniform(1000) == 0) g->snap[t] = now - 5000000 - 20000;
        else g->snap[t] = now - rng.range(10000, 200000);
        for (int k = 0; k < g->shape.reads + g->shape.writes; k++) {
            const bool is_read = k < g->shape.reads;
            const int64_t r = is_read ? (int64_t)t * g->shape.reads + k
                                      : (int64_t)R + (int64_t)t * g->shape.writes + (k - g->shape.reads);
            const int64_t sb = 2 * r, se = 2 * r + 1;
            uint8_t* b = w.key(sb);
            uint8_t* e = w.key(se);
            if (cfg == 1) {
                // skipListTest: setK(key), setK(key + 1 + U[0,10]) (SkipList.cpp:909-922, 1436-1447)
                const uint32_t key = (uint32_t)rng.uniform(20000000);
                const uint32_t key2 = key + 1 + (uint32_t)rng.uniform(11);
                memset(b, '.', 12); put_be32(b + 12, key);
                memset(e, '.', 12); put_be32(e + 12, key2);
                w.set(sb, 16);
                w.set(se, 16);
                continue;
            }
            if (cfg == 4) {
                const uint64_t tenant = rng.uniform(16);
                put_be64(b, tenant);
                memcpy(b + 8, kPath, 56);
                if (is_read && k == g->shape.reads - 1 && g->succ) {
                    // wide read [b, the S-th boundary after b), S ~ logU[1e3, 1e5]:
                    // the begin here, the end from g->succ once the batch is generated
                    const uint32_t n = (uint32_t)rng.range(4, 36);
                    for (uint32_t i = 0; i < n; i++) b[64 + i] = (uint8_t)rng.next();
                    w.set(sb, 64 + n);
                    g->wide_step[t] = (int64_t)std::exp(std::log(1e3) + rng.u01() * (std::log(1e5) - std::log(1e3)));
                    continue;
                }
                if (is_read && k == g->shape.reads - 1) {
                    // wide read over a log-uniform fraction of the tenant's space
                    const double f = std::exp(std::log(1e-3) + rng.u01() * (std::log(1e-1) - std::log(1e-3)));
                    const uint64_t x = rng.next();
                    const double span = f * 18446744073709551616.0;
                    uint64_t y = (double)(~x) < span ? ~0ull : x + (uint64_t)span;
                    if (y == x) y = x + 1;
                    put_be64(b + 64, x);
                    memcpy(e, b, 64);
                    put_be64(e + 64, y);
                    w.set(sb, 72);
                    w.set(se, 72);
                    if (y < x || y == ~0ull) {  // span clipped at the top: end past every key of the tenant
                        put_be64(e + 64, ~0ull);
                        e[72] = 0xFF;
                        w.set(se, 73);
                    }
                } else {
                    const uint32_t n = (uint32_t)rng.range(4, 36);
                    for (uint32_t i = 0; i < n; i++) b[64 + i] = (uint8_t)rng.next();
                    memcpy(e, b, 64 + n);
                    e[64 + n] = 0;
                    w.set(sb, 64 + n);
                    w.set(se, 65 + n);
                }
                continue;
            }
            // configs 2, 3, 5, 50: 16-byte keys
            if (cfg == 3) {
                const double u = rng.u01();
                const auto& cdf = g->zipf_cdf;
                const uint64_t rank = (uint64_t)(std::lower_bound(cdf.begin(), cdf.end(), u) - cdf.begin());
                put_be64(b, rank * 0x9E3779B97F4A7C15ull);
                memcpy(b + 8, "zzzzzzzz", 8);
            } else {
                put_be64(b, rng.next());
                put_be64(b + 8, rng.next());
            }
            memcpy(e, b, 16);
            if (is_read && rng.uniform(5) == 0) {
                add128(e, 1 + rng.uniform(16));
                bool wrapped = memcmp(e, b, 16) <= 0;
                if (!wrapped) {
                    w.set(sb, 16);
                    w.set(se, 16);
                    continue;
                }
                memcpy(e, b, 16);
            }
            e[16] = 0;  // point range [k, k\0) (fdbclient/FDBTypes.h:288-291)
            w.set(sb, 16);
            w.set(se, 17);
        }
    }
}

}  // namespace

extern "C" {

fdbwl* fdbwl_create(int32_t config, int32_t txns, int32_t threads) {
    fdbwl* g = new fdbwl();
    g->config = config;
    switch (config) {
        case 1: g->T = 2500; g->shape = {1, 1, 16}; break;
        case 2: g->T = 5000; g->shape = {5, 2, 17}; break;
        case 3: g->T = 5000; g->shape = {5, 2, 17}; break;
        case 4: g->T = 5000; g->shape = {5, 2, 104}; break;
        case 5: g->T = 1000000; g->shape = {5, 2, 17}; break;
        case 50: g->T = 1000000; g->shape = {0, 1, 17}; break;
        default: delete g; return nullptr;
    }
    if (txns > 0) g->T = txns;
    if (config == 3) {
        const int n = 1000000;
        g->zipf_cdf.resize(n);
        double s = 0;
        for (int i = 0; i < n; i++) s += 1.0 / std::pow((double)(i + 1), 0.99);
        double acc = 0;
        for (int i = 0; i < n; i++) {
            acc += 1.0 / std::pow((double)(i + 1), 0.99) / s;
            g->zipf_cdf[i] = acc;
        }
        g->zipf_cdf[n - 1] = 1.0;
    }
    int hw = (int)std::thread::hardware_concurrency();
    g->threads = threads > 0 ? threads : std::max(1, std::min(16, hw));
    const int64_t T = g->T, R = T * g->shape.reads, W = T * g->shape.writes, slots = 2 * (R + W);
    g->snap.resize(T);
    g->roff.resize(T + 1);
    g->woff.resize(T + 1);
    for (int64_t t = 0; t <= T; t++) {
        g->roff[t] = (int32_t)(t * g->shape.reads);
        g->woff[t] = (int32_t)(t * g->shape.writes);
    }
    g->koff.resize(slots);
    g->klen.resize(slots);
    g->bytes.assign((size_t)slots * g->shape.stride, 0);
    return g;
}

void fdbwl_destroy(fdbwl* g) { delete g; }

int fdbwl_generate(fdbwl* g, int64_t index, fdbcs_batch_view* v, int64_t* now, int64_t* new_oldest) {
    if (!g || !v) return FDBCS_E_ARG;
    const int T = g->T;
    const int nchunks = (T + CHUNK - 1) / CHUNK;
    const int nth = std::min(g->threads, nchunks);
    if (nth <= 1) {
        for (int c = 0; c < nchunks; c++) gen_chunk(g, index, c * CHUNK, std::min(T, (c + 1) * CHUNK));
    } else {
        std::vector<std::thread> th;
        for (int k = 0; k < nth; k++)
            th.emplace_back([=]() {
                for (int c = k; c < nchunks; c += nth) gen_chunk(g, index, c * CHUNK, std::min(T, (c + 1) * CHUNK));
            });
        for (auto& x : th) x.join();
    }
    const int cfg = g->config;
    if (cfg == 4 && g->succ) {  // the wide reads' ends: one batched query of the history
        const int nr = g->shape.reads;
        std::vector<uint64_t> qoff(T);
        std::vector<uint32_t> qlen(T);
        std::vector<int32_t> olen(T);
        const uint32_t stride = g->shape.stride;
        std::vector<uint8_t> out((size_t)T * stride);
        for (int t = 0; t < T; t++) {
            const int64_t sb = 2 * ((int64_t)t * nr + nr - 1);
            qoff[t] = g->koff[sb];
            qlen[t] = g->klen[sb];
        }
        const int r = g->succ(g->succ_ctx, T, g->bytes.data(), qoff.data(), qlen.data(), g->wide_step.data(),
                              out.data(), stride, olen.data());
        if (r) return r;
        for (int t = 0; t < T; t++) {
            const int64_t se = 2 * ((int64_t)t * nr + nr - 1) + 1;
            uint8_t* e = g->bytes.data() + (uint64_t)se * stride;
            if (olen[t] < 0 || (uint32_t)olen[t] > stride) {  // past the last boundary: to the end of the key space
                e[0] = 0xFF;
                e[1] = 0xFF;
                g->koff[se] = (uint64_t)se * stride;
                g->klen[se] = 2;
            } else {
                memcpy(e, out.data() + (size_t)t * stride, (size_t)olen[t]);
                g->koff[se] = (uint64_t)se * stride;
                g->klen[se] = (uint32_t)olen[t];
            }
        }
    }
    const int64_t nw = cfg == 1 ? index + 50 : (cfg == 50 ? 100000 * (index + 1) : 10000000 + index * 10000);
    if (now) *now = nw;
    if (new_oldest) *new_oldest = cfg == 1 ? index : (cfg == 50 ? 0 : nw - 5000000);
    memset(v, 0, sizeof(*v));
    v->txn_count = T;
    v->read_count = T * g->shape.reads;
    v->write_count = T * g->shape.writes;
    v->snapshot = g->snap.data();
    v->read_off = g->roff.data();
    v->write_off = g->woff.data();
    v->key_off = g->koff.data();
    v->key_len = g->klen.data();
    v->key_bytes = g->bytes.data();
    v->key_bytes_len = g->bytes.size();
    return FDBCS_OK;
}

}  // extern "C"

// ---- bench drivers ----------------------------------------------------------------

struct fdbwl_run {
    struct Batch {
        std::vector<uint8_t> bytes;        // key arena (the proxy request's)
        std::vector<fdbcs_range> reads, writes;
        std::vector<int64_t> snap;
        std::vector<int32_t> roff, woff;   // per transaction: its first read / write
        std::vector<int32_t> gidx;         // split runs: the batch index of each transaction kept
        int64_t now = 0, nold = 0;
    };
    std::vector<Batch> b;
    int32_t T = 0;
};

extern "C" {

void fdbwl_set_successor(fdbwl* g, fdbwl_succ_fn fn, void* ctx) {
    if (!g) return;
    g->succ = fn;
    g->succ_ctx = ctx;
    g->wide_step.assign(g->T, 0);
}

int fdbwl_succ_engine(void* cs, int32_t n, const uint8_t* key_bytes, const uint64_t* key_off, const uint32_t* key_len,
                      const int64_t* steps, uint8_t* out, uint32_t out_stride, int32_t* out_len) {
    return fdbcs_nth_after((fdbcs*)cs, n, key_bytes, key_off, key_len, steps, out, out_stride, out_len);
}

fdbwl_run* fdbwl_run_prepare(fdbwl* g, int64_t first, int32_t n) {
    if (!g || n < 0) return nullptr;
    fdbwl_run* r = new fdbwl_run();
    r->b.resize(n);
    r->T = g->T;
    for (int32_t i = 0; i < n; i++) {
        fdbcs_batch_view v;
        fdbwl_run::Batch& B = r->b[i];
        fdbwl_generate(g, first + i, &v, &B.now, &B.nold);
        B.bytes.assign(v.key_bytes, v.key_bytes + v.key_bytes_len);
        B.snap.assign(v.snapshot, v.snapshot + v.txn_count);
        B.roff.assign(v.read_off, v.read_off + v.txn_count + 1);
        B.woff.assign(v.write_off, v.write_off + v.txn_count + 1);
        const uint8_t* base = B.bytes.data();
        auto rng = [&](int64_t s) {
            return fdbcs_range{base + v.key_off[s], v.key_len[s], base + v.key_off[s + 1], v.key_len[s + 1]};
        };
        B.reads.resize(v.read_count);
        B.writes.resize(v.write_count);
        for (int64_t k = 0; k < v.read_count; k++) B.reads[k] = rng(2 * k);
        for (int64_t k = 0; k < v.write_count; k++) B.writes[k] = rng(2 * ((int64_t)v.read_count + k));
    }
    return r;
}

// As fdbwl_run_prepare, each batch reduced to one rank's protocol-B input:
// every transaction (global indices) with only the ranges intersecting the
// rank's keys and the writes ending at its first key -- the proxy's
// per-resolver split (fdbcs_split_batch_keep_all, MasterProxyServer.actor.cpp:
// 267-307), done here before the clock as the proxy does it before the
// request reaches the resolver.
fdbwl_run* fdbwl_run_prepare_split(fdbwl* g, int64_t first, int32_t n, int32_t nres, const uint8_t* bound_bytes,
                                   const uint64_t* bound_off, const uint32_t* bound_len, int32_t resolver) {
    if (!g || n < 0 || nres < 1 || resolver < 0 || resolver >= nres) return nullptr;
    fdbwl_run* r = new fdbwl_run();
    r->b.resize(n);
    r->T = g->T;
    std::vector<int64_t> snap;
    std::vector<int32_t> ro, wo, idx;
    std::vector<uint64_t> ko;
    std::vector<uint32_t> kl;
    for (int32_t i = 0; i < n; i++) {
        fdbcs_batch_view v, sv;
        fdbwl_run::Batch& B = r->b[i];
        fdbwl_generate(g, first + i, &v, &B.now, &B.nold);
        snap.resize(v.txn_count);
        ro.resize(v.txn_count + 1);
        wo.resize(v.txn_count + 1);
        idx.resize(v.txn_count);
        ko.resize(2 * ((size_t)v.read_count + v.write_count));
        kl.resize(ko.size());
        if (fdbcs_split_batch_keep_all(&v, nres, bound_bytes, bound_off, bound_len, resolver, &sv, snap.data(),
                                       ro.data(), wo.data(), ko.data(), kl.data(), idx.data()) != FDBCS_OK) {
            delete r;
            return nullptr;
        }
        // the share's keys only, in one arena (the request this resolver receives)
        std::vector<uint64_t> nk(2 * ((size_t)sv.read_count + sv.write_count));
        uint64_t nb = 0;
        for (size_t s = 0; s < nk.size(); s++) nb += sv.key_len[s];
        B.bytes.resize(nb);
        nb = 0;
        for (size_t s = 0; s < nk.size(); s++) {
            memcpy(B.bytes.data() + nb, sv.key_bytes + sv.key_off[s], sv.key_len[s]);
            nk[s] = nb;
            nb += sv.key_len[s];
        }
        // the transactions with a range here, at their batch indices (the
        // others reach the rank as runs of fdbcs_sharded_batch_skip)
        B.roff.assign(1, 0);
        B.woff.assign(1, 0);
        for (int32_t t = 0; t < sv.txn_count; t++) {
            if (sv.read_off[t + 1] == sv.read_off[t] && sv.write_off[t + 1] == sv.write_off[t]) continue;
            B.gidx.push_back(t);
            B.snap.push_back(sv.snapshot[t]);
            B.roff.push_back(sv.read_off[t + 1]);
            B.woff.push_back(sv.write_off[t + 1]);
        }
        const uint8_t* base = B.bytes.data();
        auto rng = [&](int64_t s) { return fdbcs_range{base + nk[s], sv.key_len[s], base + nk[s + 1], sv.key_len[s + 1]}; };
        B.reads.resize(sv.read_count);
        B.writes.resize(sv.write_count);
        for (int64_t k = 0; k < sv.read_count; k++) B.reads[k] = rng(2 * k);
        for (int64_t k = 0; k < sv.write_count; k++) B.writes[k] = rng(2 * ((int64_t)sv.read_count + k));
    }
    return r;
}

void fdbwl_run_destroy(fdbwl_run* r) { delete r; }

int32_t fdbwl_run_txns(const fdbwl_run* r) { return r ? r->T : 0; }

uint64_t fdbwl_run_key_bytes(const fdbwl_run* r, int32_t i) {
    if (!r || i < 0 || (size_t)i >= r->b.size()) return 0;
    uint64_t n = 0;
    for (const fdbcs_range& x : r->b[i].reads) n += (uint64_t)x.begin_len + x.end_len;
    for (const fdbcs_range& x : r->b[i].writes) n += (uint64_t)x.begin_len + x.end_len;
    return n;
}

// FDBWL_MARK=1 (measurement): a no-op HIP API call at the window's start, at
// the end of the adds and at detectConflicts' return, so that a rocprofv3
// --hip-runtime-trace aligns the host phases with the device timeline
// (scripts/api_timeline.py).  Resolved at run time: this library does not
// link the HIP runtime.
static void trace_mark() {
    using fn = int (*)();
    static const fn f = getenv("FDBWL_MARK") ? (fn)dlsym(RTLD_DEFAULT, "hipPeekAtLastError") : nullptr;
    if (f) f();
}

int fdbwl_run_resolver(fdbwl_run* r, fdbcs* cs, double* batch_us, double* add_us, uint8_t* verdicts) {
    return fdbwl_run_resolver_sampled(r, cs, nullptr, 0, 0.0, 0.0, batch_us, add_us, verdicts);
}

int fdbwl_run_resolver_sampled(fdbwl_run* r, fdbcs* cs, void* sample, int64_t offset_per_key, double expire0,
                               double expire_step, double* batch_us, double* add_us, uint8_t* verdicts) {
    if (!r || !cs) return FDBCS_E_ARG;
    fdbcs_sample* smp = static_cast<fdbcs_sample*>(sample);
    std::vector<uint8_t> scratch(std::max<int32_t>(r->T, 1));
    for (size_t i = 0; i < r->b.size(); i++) {
        const fdbwl_run::Batch& B = r->b[i];
        uint8_t* out = verdicts ? verdicts + i * (size_t)r->T : scratch.data();
        static const int warm = getenv("FDBWL_WARM") ? atoi(getenv("FDBWL_WARM")) : 0;
        if (warm) {  // (experiment: the request as just received, in cache)
            volatile uint64_t acc = 0;
            for (size_t k = 0; k < B.bytes.size(); k += 64) acc += B.bytes[k];
            for (size_t k = 0; k < B.reads.size(); k += 2) acc += B.reads[k].begin_len;
            for (size_t k = 0; k < B.writes.size(); k += 2) acc += B.writes[k].begin_len;
        }
        trace_mark();
        const auto t0 = std::chrono::steady_clock::now();
        int st = fdbcs_batch_begin(cs);  // ConflictBatch conflictBatch(self->conflictSet)
        const int T = (int)B.snap.size();
        for (int t = 0; st == FDBCS_OK && t < T; t++)  // conflictBatch.addTransaction(req.transactions[t])
            st = fdbcs_batch_add(cs, B.snap[t], B.reads.data() + B.roff[t], B.roff[t + 1] - B.roff[t],
                                 B.writes.data() + B.woff[t], B.woff[t + 1] - B.woff[t]);
        const auto ta = std::chrono::steady_clock::now();
        trace_mark();
        if (st == FDBCS_OK) st = fdbcs_batch_detect(cs, B.now, B.nold, out);  // detectConflicts(...)
        if (st == FDBCS_OK && smp)  // if (self->resolverCount > 1): the batch's iopsSample adds
            st = fdbcs_sample_add_batch(smp, cs, nullptr, offset_per_key, expire0 + (double)i * expire_step, nullptr);
        const auto t1 = std::chrono::steady_clock::now();
        trace_mark();
        if (st != FDBCS_OK) return st;
        if (batch_us) batch_us[i] = std::chrono::duration<double, std::micro>(t1 - t0).count();
        if (add_us) add_us[i] = std::chrono::duration<double, std::micro>(ta - t0).count();
    }
    return FDBCS_OK;
}

// The same loop over one rank of an exact sharded resolver (fdbcs_sharded_*).
int fdbwl_run_resolver_sharded(fdbwl_run* r, fdbcs_sharded* sh, double* batch_us, double* add_us,
                               uint8_t* verdicts) {
    if (!r || !sh) return FDBCS_E_ARG;
    std::vector<uint8_t> scratch(std::max<int32_t>(r->T, 1));
    for (size_t i = 0; i < r->b.size(); i++) {
        const fdbwl_run::Batch& B = r->b[i];
        uint8_t* out = verdicts ? verdicts + i * (size_t)r->T : scratch.data();
        trace_mark();
        const auto t0 = std::chrono::steady_clock::now();
        int st = fdbcs_sharded_batch_begin(sh);
        const int n = (int)B.snap.size();
        int32_t next = 0;  // batch index of the next transaction
        for (int k = 0; st == FDBCS_OK && k < n; k++) {
            const int32_t t = B.gidx.empty() ? k : B.gidx[k];
            if (t > next) st = fdbcs_sharded_batch_skip(sh, t - next);
            if (st == FDBCS_OK)
                st = fdbcs_sharded_batch_add(sh, B.snap[k], B.reads.data() + B.roff[k], B.roff[k + 1] - B.roff[k],
                                             B.writes.data() + B.woff[k], B.woff[k + 1] - B.woff[k]);
            next = t + 1;
        }
        if (st == FDBCS_OK && r->T > next) st = fdbcs_sharded_batch_skip(sh, r->T - next);
        const auto ta = std::chrono::steady_clock::now();
        trace_mark();
        if (st == FDBCS_OK) st = fdbcs_sharded_batch_detect(sh, B.now, B.nold, out);
        const auto t1 = std::chrono::steady_clock::now();
        trace_mark();
        if (st != FDBCS_OK) return st;
        if (batch_us) batch_us[i] = std::chrono::duration<double, std::micro>(t1 - t0).count();
        if (add_us) add_us[i] = std::chrono::duration<double, std::micro>(ta - t0).count();
    }
    return FDBCS_OK;
}

int fdbwl_run_adds(fdbwl_run* r, fdbcs* cs, double* add_us) {
    if (!r || !cs) return FDBCS_E_ARG;
    for (size_t i = 0; i < r->b.size(); i++) {
        const fdbwl_run::Batch& B = r->b[i];
        const auto t0 = std::chrono::steady_clock::now();
        int st = fdbcs_batch_begin(cs);
        const int T = (int)B.snap.size();
        for (int t = 0; st == FDBCS_OK && t < T; t++)
            st = fdbcs_batch_add(cs, B.snap[t], B.reads.data() + B.roff[t], B.roff[t + 1] - B.roff[t],
                                 B.writes.data() + B.woff[t], B.woff[t + 1] - B.woff[t]);
        const auto ta = std::chrono::steady_clock::now();
        if (st != FDBCS_OK) return st;
        if (add_us) add_us[i] = std::chrono::duration<double, std::micro>(ta - t0).count();
    }
    return FDBCS_OK;
}

int fdbwl_prefill(fdbwl* g, fdbcs* cs, int64_t first, int32_t n) {
    if (!g || !cs || n < 0) return FDBCS_E_ARG;
    std::vector<uint8_t> verdict(std::max(g->T, 1));
    int inflight = 0;
    for (int32_t i = 0; i < n; i++) {
        fdbcs_batch_view v;
        int64_t now, nold;
        fdbwl_generate(g, first + i, &v, &now, &nold);  // (overlaps the batch in flight)
        if (inflight == 2) {
            int st = fdbcs_batch_wait(cs, verdict.data());
            if (st != FDBCS_OK) return st;
            inflight--;
        }
        int st = fdbcs_batch_submit_packed(cs, &v, now, nold);  // (copies v into pinned staging)
        if (st != FDBCS_OK) return st;
        inflight++;
    }
    while (inflight--) {
        int st = fdbcs_batch_wait(cs, verdict.data());
        if (st != FDBCS_OK) return st;
    }
    return FDBCS_OK;
}

}  // extern "C"
