// load_metrics.hip -- the Resolver's load metrics.
//
// The reference Resolver keeps `iopsSample`, a TransientStorageMetricSample
// (fdbserver/StorageMetrics.actor.h:98-182) over the begin keys of every
// range it resolves (Resolver.actor.cpp:146-151, only when resolverCount > 1):
//
//   for each transaction t, in batch order:
//     for each write range w of t:  addAndExpire(w.begin, SAMPLE_OFFSET_PER_KEY + |w.begin|, expire)
//     for each read range r of t:   addAndExpire(r.begin, SAMPLE_OFFSET_PER_KEY + |r.begin|, expire)
//
// and answers the master's ResolutionMetricsRequest with getEstimate(allKeys)
// and ResolutionSplitRequest with splitEstimate (Resolver.actor.cpp:276-284;
// the caller is resolutionBalancing, masterserver.actor.cpp:964-1020).
//
// Split of the work here:
//   device  the per-range roll over the whole batch (R + W ranges, the part
//           that grows with the batch): one thread per range in the
//           Resolver's add order, an ordered stream compaction of the sampled
//           ranges (count -> scan -> emit) and a gather of their begin-key
//           bytes.  Inputs are the batch already resident in HBM.
//   host    the sample itself (a sorted key -> metric set with prefix sums
//           and the expiry queue): at KEY_BYTES_PER_SAMPLE = 2e4 it holds
//           ~0.6 % of the keys of the last SAMPLE_EXPIRATION_TIME second,
//           tens of thousands of entries, queried a few times per second.
//
// The roll.  The reference draws g_random->random01() < metric / units
// (StorageMetrics.actor.h:103-105), an unseeded global stream.  Here draw k of
// a sample (batch sequence number `seq`, position `pos` in the add order
// above) is the integer h = mix64(seed + seq * C1 + pos * C2) and the key is
// sampled iff h mod units < metric: the same probability metric / units
// (to within 2^-49), a counter-based draw every thread computes alone, and a
// definition the oracle (oracle/load_sample.py) restates bit for bit.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <deque>
#include <cstdint>
#include <string>
#include <vector>

#include "../../include/fdbcs.h"
#include "kernels.h"

namespace {

#define LM_HIPOK(x)                                      \
    do {                                                 \
        if ((x) != hipSuccess) return FDBCS_E_HIP;       \
    } while (0)

constexpr int RB = 256;  // ranges per workgroup (4 wavefronts)

using fdbcs_dev::roll_amount;  // (common.h: the draw and the add decision, shared with the ingest's roll)
using fdbcs_dev::roll_hash;

struct RollArgs {
    const int32_t* read_off;   // [T+1]
    const int32_t* write_off;  // [T+1]
    const uint64_t* key_off;
    const uint32_t* key_len;
    const uint8_t* key_bytes;
    int32_t T, R, W;
    uint64_t seed, seq;
    int64_t offset_per_key, units;
};

// Position pos of the Resolver's add order -> begin key slot.  Transaction t
// starts at read_off[t] + write_off[t]; its writes come first.
__device__ inline uint32_t pos_slot(const RollArgs& a, int64_t pos) {
    int lo = 0, hi = a.T - 1;  // last t with read_off[t] + write_off[t] <= pos
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if ((int64_t)a.read_off[mid] + a.write_off[mid] <= pos) lo = mid;
        else hi = mid - 1;
    }
    const int64_t base = (int64_t)a.read_off[lo] + a.write_off[lo];
    const int64_t nw = a.write_off[lo + 1] - a.write_off[lo];
    const int64_t k = pos - base;
    if (k < nw) return (uint32_t)(2 * (int64_t)a.R + 2 * ((int64_t)a.write_off[lo] + k));
    return (uint32_t)(2 * ((int64_t)a.read_off[lo] + (k - nw)));
}

__device__ inline int64_t pos_amount(const RollArgs& a, int64_t pos, uint32_t& slot, uint32_t& len) {
    slot = pos_slot(a, pos);
    len = a.key_len[slot];
    return roll_amount(roll_hash(a.seed, a.seq, (uint64_t)pos), a.offset_per_key + (int64_t)len, a.units);
}

// Workgroup-wide exclusive scan of two counters (one per thread); returns the
// totals through tot_*.
__device__ inline void block_scan2(uint32_t c, uint32_t b, uint32_t& ec, uint32_t& eb, uint32_t& tot_c,
                                   uint32_t& tot_b) {
    __shared__ uint32_t sc[RB / 64], sb[RB / 64];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    uint32_t ic = c, ib = b;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t oc = __shfl_up(ic, d, 64), ob = __shfl_up(ib, d, 64);
        if (lane >= d) { ic += oc; ib += ob; }
    }
    if (lane == 63) { sc[wid] = ic; sb[wid] = ib; }
    __syncthreads();
    uint32_t pc = 0, pb = 0;
    tot_c = 0; tot_b = 0;
#pragma unroll
    for (int w = 0; w < RB / 64; w++) {
        if (w < wid) { pc += sc[w]; pb += sb[w]; }
        tot_c += sc[w]; tot_b += sb[w];
    }
    ec = pc + ic - c;
    eb = pb + ib - b;
}

__global__ __launch_bounds__(RB) void k_roll_count(RollArgs a, uint32_t* blk_cnt, uint32_t* blk_bytes) {
    const int64_t n = (int64_t)a.R + a.W;
    const int64_t pos = (int64_t)blockIdx.x * RB + threadIdx.x;
    uint32_t c = 0, b = 0;
    if (pos < n) {
        uint32_t slot, len;
        if (pos_amount(a, pos, slot, len)) { c = 1; b = len; }
    }
    uint32_t ec, eb, tc, tb;
    block_scan2(c, b, ec, eb, tc, tb);
    if (threadIdx.x == 0) { blk_cnt[blockIdx.x] = tc; blk_bytes[blockIdx.x] = tb; }
}

// One workgroup: exclusive scan of the per-block counts (in place, 64-bit
// byte offsets) and the two totals.
__global__ __launch_bounds__(RB) void k_roll_scan(uint32_t* blk_cnt, const uint32_t* blk_bytes,
                                                  uint64_t* blk_boff, int nblk, uint64_t* totals) {
    uint64_t carry_c = 0, carry_b = 0;
    for (int base = 0; base < nblk; base += RB) {
        const int i = base + threadIdx.x;
        const uint32_t c = i < nblk ? blk_cnt[i] : 0, b = i < nblk ? blk_bytes[i] : 0;
        uint32_t ec, eb, tc, tb;
        block_scan2(c, b, ec, eb, tc, tb);
        if (i < nblk) { blk_cnt[i] = (uint32_t)(carry_c + ec); blk_boff[i] = carry_b + eb; }
        carry_c += tc; carry_b += tb;
        __syncthreads();
    }
    if (threadIdx.x == 0) { totals[0] = carry_c; totals[1] = carry_b; }
}

// Writes the sampled entries straight into pinned host memory (a few hundred
// per 5k-txn batch: no device staging, no copy); entries past the host
// buffers' capacities are dropped and the caller re-emits after growing them.
__global__ __launch_bounds__(RB) void k_roll_emit(RollArgs a, const uint32_t* blk_cnt, const uint64_t* blk_boff,
                                                  int64_t* out_amount, uint32_t* out_len, uint64_t* out_off,
                                                  uint8_t* out_bytes, uint64_t cap_n, uint64_t cap_b) {
    __shared__ const uint8_t* e_src[RB];
    __shared__ uint64_t e_off[RB];
    __shared__ uint32_t e_len[RB];
    const int64_t n = (int64_t)a.R + a.W;
    const int64_t pos = (int64_t)blockIdx.x * RB + threadIdx.x;
    uint32_t c = 0, b = 0, slot = 0, len = 0;
    int64_t x = 0;
    if (pos < n) {
        x = pos_amount(a, pos, slot, len);
        if (x) { c = 1; b = len; }
    }
    uint32_t ec, eb, tc, tb;
    block_scan2(c, b, ec, eb, tc, tb);
    if (c) {
        const uint64_t i = blk_cnt[blockIdx.x] + ec;
        const uint64_t off = blk_boff[blockIdx.x] + eb;
        const bool fits = i < cap_n && off + len <= cap_b;
        if (fits) {
            out_amount[i] = x;
            out_len[i] = len;
            out_off[i] = off;
        }
        e_src[ec] = a.key_bytes + a.key_off[slot];
        e_off[ec] = off;
        e_len[ec] = fits ? len : 0;
    }
    __syncthreads();
    // the block's sampled keys, one after another, each copied by the whole
    // block (a long key is not one lane's serial byte loop across the link)
    for (uint32_t j = 0; j < tc; j++) {
        const uint8_t* src = e_src[j];
        uint8_t* dst = out_bytes + e_off[j];
        for (uint32_t k = threadIdx.x; k < e_len[j]; k += RB) dst[k] = src[k];
    }
}

template <class T>
int grow_pinned(T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return FDBCS_OK;
    size_t c = std::max<size_t>(n + n / 2, 1024);
    if (p) hipHostFree(p);
    p = nullptr;
    cap = 0;
    if (hipHostMalloc((void**)&p, c * sizeof(T), hipHostMallocDefault) != hipSuccess) return FDBCS_E_NOMEM;
    cap = c;
    return FDBCS_OK;
}

template <class T>
int grow_dev(T*& p, size_t& cap, size_t n) {
    if (n <= cap && p) return FDBCS_OK;
    size_t c = std::max<size_t>(n, cap * 2);
    c = std::max<size_t>(c, 256);
    if (p) hipFree(p);
    p = nullptr;
    cap = 0;
    if (hipMalloc(&p, c * sizeof(T)) != hipSuccess) return FDBCS_E_NOMEM;
    cap = c;
    return FDBCS_OK;
}

int kcmp(const std::string& a, const uint8_t* b, uint32_t bl) {
    const uint32_t n = std::min<uint32_t>((uint32_t)a.size(), bl);
    const int c = n ? memcmp(a.data(), b, n) : 0;
    if (c) return c < 0 ? -1 : 1;
    return a.size() < bl ? -1 : (a.size() > bl ? 1 : 0);
}

}  // namespace

// The sample: IndexedSet<Key, int64_t> (flow/IndexedSet.h) as an
// open-addressing hash table whose keys live in one byte arena (no allocation
// per sampled key on the Resolver's per-batch path), plus a sorted view with
// prefix sums rebuilt lazily before a query: queries are rare next to adds
// (the master asks every MIN_BALANCE_TIME), the reverse of the trade the
// reference's balanced tree makes.  The expiry queue holds one group per
// batch (all its entries share one expiration).
struct FlatSample {
    struct E {
        uint64_t h, off;
        uint32_t len, st;  // st: 0 empty, 1 live, 2 erased
        int64_t m;
    };
    std::vector<E> t;
    size_t live = 0, used = 0, garbage = 0;
    std::string arena;

    static uint64_t mix(uint64_t z) {
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    static uint64_t hash(const uint8_t* p, uint32_t n) {
        uint64_t h = mix(0x9E3779B97F4A7C15ull ^ n);
        for (; n >= 8; p += 8, n -= 8) {
            uint64_t w;
            memcpy(&w, p, 8);
            h = mix(h ^ w);
        }
        uint64_t w = 0;
        if (n) memcpy(&w, p, n);
        return mix(h ^ w);
    }
    void place(const E& e) {
        const size_t mask = t.size() - 1;
        size_t i = e.h & mask;
        while (t[i].st) i = (i + 1) & mask;
        t[i] = e;
    }
    // rebuild at capacity cap: drops erased slots and compacts the arena
    void rehash(size_t cap) {
        std::vector<E> old(cap, E{});
        old.swap(t);
        std::string na;
        na.reserve(arena.size() - garbage);
        for (const E& e : old)
            if (e.st == 1) {
                E n = e;
                n.off = na.size();
                na.append(arena, e.off, e.len);
                place(n);
            }
        arena.swap(na);
        garbage = 0;
        used = live;
    }
    // the metric of key k (0: not in the sample)
    int64_t get(const uint8_t* k, uint32_t len, uint64_t h) const {
        if (t.empty()) return 0;
        const size_t mask = t.size() - 1;
        for (size_t i = h & mask; t[i].st; i = (i + 1) & mask) {
            const E& e = t[i];
            if (e.st == 1 && e.h == h && e.len == len && (len == 0 || !memcmp(arena.data() + e.off, k, len)))
                return e.m;
        }
        return 0;
    }
    // IndexedSet::addMetric (flow/IndexedSet.h:587-598) followed by the
    // erase-at-zero of StorageMetrics.actor.h:136-137 / :177-178
    void add(const uint8_t* k, uint32_t len, uint64_t h, int64_t m) {
        if (t.empty()) t.assign(1024, E{});
        if ((used + 1) * 2 > t.size()) rehash((live + 1) * 4 > t.size() ? t.size() * 2 : t.size());
        else if (garbage > (1u << 20) && garbage * 2 > arena.size()) rehash(t.size());
        const size_t mask = t.size() - 1;
        size_t i = h & mask, tomb = SIZE_MAX;
        for (; t[i].st; i = (i + 1) & mask) {
            E& e = t[i];
            if (e.st == 1 && e.h == h && e.len == len && (len == 0 || !memcmp(arena.data() + e.off, k, len))) {
                e.m += m;
                if (e.m == 0) {
                    e.st = 2;
                    live--;
                    garbage += len;
                }
                return;
            }
            if (e.st == 2 && tomb == SIZE_MAX) tomb = i;
        }
        if (m == 0) return;
        if (tomb == SIZE_MAX) used++;
        t[tomb != SIZE_MAX ? tomb : i] = E{h, arena.size(), len, 1, m};
        arena.append((const char*)k, len);
        live++;
    }
};

struct fdbcs_sample {
    int64_t units = 0;
    uint64_t seed = 0;
    uint64_t seq = 0;  // batches rolled so far (draw counter)
    fdbcs* attached = nullptr;  // fdbcs_sample_attach: the engine whose ingest rolls for this sample
    // batches rolled by the attached engine, not yet in the sample: the
    // Resolver's commit path only copies their entries; the inserts happen at
    // the next poll / query (drain), in batch order, before anything reads or
    // expires the sample -- nothing observable changes
    struct Pending {
        double exp;
        std::vector<fdbcs_dev::LmEntry> ent;
        std::vector<uint8_t> bytes;
    };
    std::deque<Pending> pending;
    FlatSample sample;
    struct GItem {
        uint64_t h, off;
        uint32_t len;
        int64_t delta;
    };
    struct Group {
        double exp;
        std::string bytes;
        std::vector<GItem> items;
    };
    std::deque<Group> queue;
    size_t queued = 0;
    // query view
    mutable bool dirty = true;
    mutable std::vector<std::string> vstore;
    mutable std::vector<const std::string*> keys;
    mutable std::vector<int64_t> prefix;  // prefix[i] = sumTo(i); size n+1
    // device roll buffers
    uint32_t* d_cnt = nullptr;
    size_t cnt_cap = 0;
    uint32_t* d_bytes = nullptr;
    size_t bytes_cap = 0;
    uint64_t* d_boff = nullptr;
    size_t boff_cap = 0;
    // pinned host outputs (written by the kernels)
    uint64_t* h_tot = nullptr;
    size_t tot_cap = 0;
    int64_t* h_amt = nullptr;
    size_t amt_cap = 0;
    uint32_t* h_len = nullptr;
    size_t len_cap = 0;
    uint64_t* h_off = nullptr;
    size_t off_cap = 0;
    uint8_t* h_out = nullptr;
    size_t out_cap = 0;

    void add_metric(const uint8_t* k, uint32_t len, int64_t m) {
        dirty = true;
        sample.add(k, len, FlatSample::hash(k, len), m);
    }
    void view() const {
        if (!dirty) return;
        std::vector<std::pair<std::string, int64_t>> ents;
        ents.reserve(sample.live);
        for (const auto& e : sample.t)
            if (e.st == 1) ents.emplace_back(std::string(sample.arena, e.off, e.len), e.m);
        std::sort(ents.begin(), ents.end(), [](const auto& x, const auto& y) {
            return kcmp(x.first, (const uint8_t*)y.first.data(), (uint32_t)y.first.size()) < 0;
        });
        vstore.clear();
        vstore.reserve(ents.size());
        keys.clear();
        prefix.assign(1, 0);
        prefix.reserve(ents.size() + 1);
        for (auto& kv : ents) {
            vstore.push_back(std::move(kv.first));
            prefix.push_back(prefix.back() + kv.second);
        }
        for (const auto& k : vstore) keys.push_back(&k);
        dirty = false;
    }
    // index of the first key >= k (IndexedSet::lower_bound)
    int64_t lower_bound(const uint8_t* k, uint32_t kl) const {
        int64_t lo = 0, hi = (int64_t)keys.size();
        while (lo < hi) {
            const int64_t mid = (lo + hi) >> 1;
            if (kcmp(*keys[mid], k, kl) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // IndexedSet::index (flow/IndexedSet.h:1043-1063): first x with
    // metric < sumTo(x + 1), or end
    int64_t index(int64_t m) const {
        const auto it = std::upper_bound(prefix.begin() + 1, prefix.end(), m);
        return (int64_t)(it - (prefix.begin() + 1));
    }
    int64_t estimate(const uint8_t* b, uint32_t bl, const uint8_t* e, uint32_t el) const {
        view();
        return prefix[lower_bound(e, el)] - prefix[lower_bound(b, bl)];
    }
    ~fdbcs_sample() {
        hipFree(d_cnt); hipFree(d_bytes); hipFree(d_boff);
        hipHostFree(h_tot); hipHostFree(h_amt); hipHostFree(h_len); hipHostFree(h_off); hipHostFree(h_out);
    }
};

namespace {

// keyBetween (fdbclient/FDBTypes.h:304-325) with SPLIT_KEY_SIZE_LIMIT
// (fdbclient/Knobs.cpp:60: KEY_SIZE_LIMIT / 2 = 5000).
constexpr int SPLIT_KEY_SIZE_LIMIT = 5000;
std::string key_between(const std::string& b, const std::string& e) {
    int pos = 0;
    const int mn = (int)std::min(b.size(), e.size());
    for (; pos < mn && pos < SPLIT_KEY_SIZE_LIMIT; pos++)
        if (b[pos] != e[pos]) return e.substr(0, pos + 1);
    if (pos < SPLIT_KEY_SIZE_LIMIT && b.size() < e.size()) return e.substr(0, pos + 1);
    return e;
}

bool str_less(const std::string& a, const std::string& b) {
    return kcmp(a, (const uint8_t*)b.data(), (uint32_t)b.size()) < 0;
}

// StorageMetricSample::splitEstimate (StorageMetrics.actor.h:38-73) over the
// sorted view: iterators are indices, end() = n.
std::string split_estimate(const fdbcs_sample* s, const std::string& rb, const std::string& re, int64_t offset,
                           bool front) {
    s->view();
    const int64_t n = (int64_t)s->keys.size();
    auto K = [&](int64_t i) -> const std::string& { return *s->keys[i]; };
    auto est = [&](const std::string& b, const std::string& e) {
        return s->estimate((const uint8_t*)b.data(), (uint32_t)b.size(), (const uint8_t*)e.data(),
                           (uint32_t)e.size());
    };
    const int64_t anchor = front ? s->prefix[s->lower_bound((const uint8_t*)rb.data(), (uint32_t)rb.size())] + offset
                                 : s->prefix[s->lower_bound((const uint8_t*)re.data(), (uint32_t)re.size())] - offset;
    int64_t fwd = s->index(anchor);
    if (fwd == n || !str_less(K(fwd), re)) return re;
    if (!front && !str_less(rb, K(fwd))) return rb;
    int64_t bck = fwd;
    while ((fwd != n && str_less(K(fwd), re)) || (bck != 0 && str_less(rb, K(bck)))) {
        if (bck != 0 && str_less(rb, K(bck))) {
            const int64_t it = bck;
            bck--;
            const std::string& lo = bck != 0 ? (str_less(K(bck), rb) ? rb : K(bck)) : rb;
            std::string split = key_between(lo, K(it));
            if (!front || (est(rb, split) > 0 && (int)split.size() <= SPLIT_KEY_SIZE_LIMIT)) return split;
        }
        if (fwd != n && str_less(K(fwd), re)) {
            const int64_t it = fwd + 1;
            const std::string& hi = it != n ? (str_less(re, K(it)) ? re : K(it)) : re;
            std::string split = key_between(K(fwd), hi);
            if (front || (est(split, re) > 0 && (int)split.size() <= SPLIT_KEY_SIZE_LIMIT)) return split;
            fwd = it;
        }
    }
    return front ? re : rb;
}

}  // namespace

extern "C" {

int fdbcs_sample_create(fdbcs_sample** out, int64_t units_per_sample, uint64_t seed) {
    if (!out || units_per_sample <= 0) return FDBCS_E_ARG;
    fdbcs_sample* s = new (std::nothrow) fdbcs_sample();
    if (!s) return FDBCS_E_NOMEM;
    s->units = units_per_sample;
    s->seed = seed;
    *out = s;
    return FDBCS_OK;
}

void fdbcs_sample_destroy(fdbcs_sample* s) {
    if (s && s->attached) fdbcs_dev::engine_lm_attach(s->attached, nullptr, nullptr, 0, 0, 0);
    delete s;
}

int fdbcs_sample_attach(fdbcs_sample* s, fdbcs* cs, int64_t offset_per_key) {
    if (!s || offset_per_key < 0) return FDBCS_E_ARG;
    if (s->attached) fdbcs_dev::engine_lm_attach(s->attached, nullptr, nullptr, 0, 0, 0);
    s->attached = cs;
    if (cs) fdbcs_dev::engine_lm_attach(cs, s, &s->seq, s->seed, s->units, offset_per_key);
    return FDBCS_OK;
}

}  // extern "C"

namespace fdbcs_dev {
void sample_unlink(const void* owner, const fdbcs* cs) {
    fdbcs_sample* s = static_cast<fdbcs_sample*>(const_cast<void*>(owner));
    if (s->attached == cs) s->attached = nullptr;
}
}  // namespace fdbcs_dev

namespace {

// The batch's entries into the sample and its expiry group, in the Resolver's
// add order (addAndExpire, StorageMetrics.actor.h:108-113): entry i of the m
// taken is entry order[i] (amt, len, off: its amount, key length, key bytes
// at bytes + off).
template <class A, class L, class O>
void sample_insert(fdbcs_sample* s, double expiration, uint64_t m, A amt, L len, O off, const uint8_t* bytes,
                   const std::vector<uint32_t>* order) {
    fdbcs_sample::Group g{expiration, std::string(), {}};
    g.items.reserve(m);
    uint64_t nb = 0;
    for (uint64_t i = 0; i < m; i++) nb += len(order ? (*order)[i] : (uint32_t)i);
    g.bytes.reserve(nb);
    for (uint64_t i = 0; i < m; i++) {
        const uint32_t e = order ? (*order)[i] : (uint32_t)i;
        g.bytes.append((const char*)bytes + off(e), len(e));
    }
    s->dirty = true;
    uint64_t o = 0;
    for (uint64_t i = 0; i < m; i++) {
        const uint32_t e = order ? (*order)[i] : (uint32_t)i;
        const uint32_t ln = len(e);
        const uint8_t* k = (const uint8_t*)g.bytes.data() + o;
        const uint64_t h = FlatSample::hash(k, ln);
        s->sample.add(k, ln, h, amt(e));
        g.items.push_back({h, o, ln, -amt(e)});
        o += ln;
    }
    s->queued += m;
    s->queue.push_back(std::move(g));
}

// the pending batches of the attached engine's rolls into the sample, oldest first
void drain(fdbcs_sample* s) {
    while (!s->pending.empty()) {
        fdbcs_sample::Pending& p = s->pending.front();
        const uint64_t m = p.ent.size();
        std::vector<uint32_t> order(m);
        for (uint64_t i = 0; i < m; i++) order[i] = (uint32_t)i;
        const auto& E = p.ent;
        std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return E[a].pos < E[b].pos; });
        sample_insert(
            s, p.exp, m, [&](uint32_t e) { return E[e].amount; }, [&](uint32_t e) { return E[e].len; },
            [&](uint32_t e) { return E[e].off; }, p.bytes.data(), &order);
        s->pending.pop_front();
    }
}
void drain(const fdbcs_sample* s) { drain(const_cast<fdbcs_sample*>(s)); }  // (queries: nothing observable moves)

}  // namespace

extern "C" {

int fdbcs_sample_add_batch(fdbcs_sample* s, fdbcs* cs, const fdbcs_batch_view* dev_batch, int64_t offset_per_key,
                           double expiration, int64_t* out_sampled) {
    if (!s || !cs || offset_per_key < 0) return FDBCS_E_ARG;
    if (!dev_batch) {  // the engine's ingest rolled this batch already (fdbcs_sample_attach): no launch, no wait
        fdbcs_dev::LmTake tk;
        if (fdbcs_dev::engine_lm_take(cs, s, s->seq, offset_per_key, tk)) {
            const uint64_t m = (uint64_t)tk.count;
            bool fits = m <= tk.cap_n;
            uint64_t nb = 0;
            for (uint64_t i = 0; fits && i < m; i++) {
                fits = tk.ent[i].off + tk.ent[i].len <= tk.cap_b;
                nb = std::max<uint64_t>(nb, tk.ent[i].off + tk.ent[i].len);
            }
            if (fits) {  // (copied now: the next batch's ingest reuses the pinned outputs)
                s->pending.push_back({expiration, std::vector<fdbcs_dev::LmEntry>(tk.ent, tk.ent + m),
                                      std::vector<uint8_t>(tk.bytes, tk.bytes + nb)});
                s->seq++;
                // (a caller that never polls or queries: bounded, ~10 MB at config 2; the
                // Resolver's metrics requests and polls drain it off the commit path)
                if (s->pending.size() > 1024) drain(s);
                if (out_sampled) *out_sampled = (int64_t)m;
                return FDBCS_OK;
            }
            // (past the pinned outputs' capacities: the rest below rolls the still-resident batch again)
        }
    }
    drain(s);  // (the batches before this one enter the sample first)
    // the buffers and launches belong on the engine's device, whatever the
    // calling thread's current one (the shim's G-GPU mode hands rank 0's
    // engine to the Resolver's thread); restored on every return
    struct DeviceScope {
        int prev = -1;
        explicit DeviceScope(int d) {
            if (hipGetDevice(&prev) != hipSuccess || prev == d) prev = -1;
            else if (hipSetDevice(d) != hipSuccess) prev = -1;
        }
        ~DeviceScope() {
            if (prev >= 0) hipSetDevice(prev);
        }
    } scope(fdbcs_dev::engine_device(cs));
    fdbcs_batch_view dv;
    if (dev_batch) dv = *dev_batch;
    else {
        const int r = fdbcs_last_device_batch(cs, &dv);
        if (r) return r;
    }
    if (dv.txn_count < 0 || dv.read_count < 0 || dv.write_count < 0) return FDBCS_E_ARG;
    const uint64_t seq = s->seq;  // (advanced once the batch is in the sample)
    const int64_t n = (int64_t)dv.read_count + dv.write_count;
    if (out_sampled) *out_sampled = 0;
    if (n == 0 || dv.txn_count == 0) {
        s->seq++;
        return FDBCS_OK;
    }
    hipStream_t st = (hipStream_t)fdbcs_stream(cs);
    const int64_t nblk = (n + RB - 1) / RB;
    if (nblk > INT32_MAX) return FDBCS_E_CAPACITY;
    int r;
    if ((r = grow_dev(s->d_cnt, s->cnt_cap, nblk)) || (r = grow_dev(s->d_bytes, s->bytes_cap, nblk)) ||
        (r = grow_dev(s->d_boff, s->boff_cap, nblk)) || (r = grow_pinned(s->h_tot, s->tot_cap, 2)) ||
        (r = grow_pinned(s->h_amt, s->amt_cap, 1)) || (r = grow_pinned(s->h_len, s->len_cap, 1)) ||
        (r = grow_pinned(s->h_off, s->off_cap, 1)) || (r = grow_pinned(s->h_out, s->out_cap, 1)))
        return r;
    RollArgs a{dv.read_off, dv.write_off, dv.key_off, dv.key_len, dv.key_bytes, dv.txn_count, dv.read_count,
               dv.write_count, s->seed, seq, offset_per_key, s->units};
    hipLaunchKernelGGL(k_roll_count, dim3((unsigned)nblk), dim3(RB), 0, st, a, s->d_cnt, s->d_bytes);
    hipLaunchKernelGGL(k_roll_scan, dim3(1), dim3(RB), 0, st, s->d_cnt, s->d_bytes, s->d_boff, (int)nblk, s->h_tot);
    // one round trip in the common case: emit into the current host buffers,
    // and again after growing them if the totals say they were too small
    for (int pass = 0; pass < 2; pass++) {
        const size_t cap_n = std::min(std::min(s->amt_cap, s->len_cap), s->off_cap);
        hipLaunchKernelGGL(k_roll_emit, dim3((unsigned)nblk), dim3(RB), 0, st, a, s->d_cnt, s->d_boff, s->h_amt,
                           s->h_len, s->h_off, s->h_out, (uint64_t)cap_n, (uint64_t)s->out_cap);
        LM_HIPOK(hipGetLastError());
        LM_HIPOK(hipStreamSynchronize(st));
        const uint64_t m = s->h_tot[0], nb = s->h_tot[1];
        if (m <= cap_n && nb <= s->out_cap) break;
        if (pass == 1) return FDBCS_E_CAPACITY;
        if ((r = grow_pinned(s->h_amt, s->amt_cap, m)) || (r = grow_pinned(s->h_len, s->len_cap, m)) ||
            (r = grow_pinned(s->h_off, s->off_cap, m)) || (r = grow_pinned(s->h_out, s->out_cap, nb)))
            return r;
    }
    const uint64_t m = s->h_tot[0];
    if (out_sampled) *out_sampled = (int64_t)m;
    // addAndExpire (StorageMetrics.actor.h:108-113), in the Resolver's order
    // (the ordered compaction's); the batch's queue entries form one group
    // sharing its key bytes
    const int64_t* amt = s->h_amt;
    const uint32_t* len = s->h_len;
    const uint64_t* off = s->h_off;
    sample_insert(
        s, expiration, m, [&](uint32_t e) { return amt[e]; }, [&](uint32_t e) { return len[e]; },
        [&](uint32_t e) { return off[e]; }, s->h_out, nullptr);
    s->seq++;
    return FDBCS_OK;
}

int fdbcs_sample_add_metric(fdbcs_sample* s, const uint8_t* key, uint32_t len, int64_t metric) {
    if (!s || (len && !key)) return FDBCS_E_ARG;
    drain(s);
    // an entry's metric stays >= 0 (a negative one would break the prefix-sum
    // index; the Resolver's amounts are positive and expire back to 0)
    if (metric < 0 && s->sample.get(key, len, FlatSample::hash(key, len)) + metric < 0) return FDBCS_E_ARG;
    s->add_metric(key, len, metric);
    return FDBCS_OK;
}

int fdbcs_sample_poll(fdbcs_sample* s, double now) {
    if (!s) return FDBCS_E_ARG;
    drain(s);
    // TransientStorageMetricSample::poll() (StorageMetrics.actor.h:150-164)
    while (!s->queue.empty() && s->queue.front().exp <= now) {
        const auto& g = s->queue.front();
        s->dirty = true;
        for (const auto& it : g.items) {
            if (it.delta == 0) return FDBCS_E_STATE;  // ASSERT(delta != 0)
            s->sample.add((const uint8_t*)g.bytes.data() + it.off, it.len, it.h, it.delta);
        }
        s->queued -= g.items.size();
        s->queue.pop_front();
    }
    return FDBCS_OK;
}

int64_t fdbcs_sample_estimate(const fdbcs_sample* s, const uint8_t* b, uint32_t bl, const uint8_t* e, uint32_t el) {
    if (!s || (bl && !b) || (el && !e)) return FDBCS_E_ARG;
    drain(s);
    return s->estimate(b, bl, e, el);
}

int32_t fdbcs_sample_split(const fdbcs_sample* s, const uint8_t* b, uint32_t bl, const uint8_t* e, uint32_t el,
                           int64_t offset, int front, uint8_t* out, uint32_t cap) {
    if (!s || (bl && !b) || (el && !e) || (cap && !out)) return FDBCS_E_ARG;
    drain(s);
    const std::string k = split_estimate(s, std::string((const char*)b, bl), std::string((const char*)e, el), offset,
                                         front != 0);
    if (k.size() > cap) return FDBCS_E_CAPACITY;
    if (!k.empty()) memcpy(out, k.data(), k.size());
    return (int32_t)k.size();
}

int64_t fdbcs_sample_size(const fdbcs_sample* s) {
    if (!s) return FDBCS_E_ARG;
    drain(s);
    return (int64_t)s->sample.live;
}

int64_t fdbcs_sample_queue_size(const fdbcs_sample* s) {
    if (!s) return FDBCS_E_ARG;
    drain(s);
    return (int64_t)s->queued;
}

int32_t fdbcs_sample_entry(const fdbcs_sample* s, int64_t i, uint8_t* out, uint32_t cap, int64_t* metric) {
    if (!s || i < 0 || (cap && !out)) return FDBCS_E_ARG;
    drain(s);
    s->view();
    if (i >= (int64_t)s->keys.size()) return FDBCS_E_ARG;
    const std::string& k = *s->keys[i];
    if (k.size() > cap) return FDBCS_E_CAPACITY;
    if (!k.empty()) memcpy(out, k.data(), k.size());
    if (metric) *metric = s->prefix[i + 1] - s->prefix[i];
    return (int32_t)k.size();
}

}  // extern "C"
