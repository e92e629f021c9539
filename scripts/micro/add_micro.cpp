// add_micro.cpp -- host cost of the per-transaction staging (fdbcs_batch_add)
// for config-2 batches (5,000 txns x 7 ranges, 16/17-byte keys), cold inputs
// as in the bench's timed loop.  Variants: the record append as in
// engine.hip; the same with non-temporal stores; descriptors only; warm.
//   g++ -O2 -march=native -o /tmp/am scripts/micro/add_micro.cpp
#include <immintrin.h>
#ifdef WITH_HIP
#include <hip/hip_runtime.h>
#endif

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Range {
    const uint8_t* b;
    uint32_t bl;
    const uint8_t* e;
    uint32_t el;
};
struct Hdr {
    int64_t snap;
    int32_t ro, wo, nr, nw;
};
using clk = std::chrono::steady_clock;

static inline uint64_t ld64(const uint8_t* p) {
    uint64_t x;
    memcpy(&x, p, 8);
    return x;
}
static inline int kcmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t n = al < bl ? al : bl;
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint64_t x = ld64(a + i), y = ld64(b + i);
        if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y) ? -1 : 1;
    }
    for (; i < n; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}
static inline void copy_small(uint8_t* d, const uint8_t* s, uint32_t n) {
    if (n >= 16 && n <= 32) {
        uint8_t t0[16], t1[16];
        memcpy(t0, s, 16);
        memcpy(t1, s + n - 16, 16);
        memcpy(d, t0, 16);
        memcpy(d + n - 16, t1, 16);
    } else {
        memcpy(d, s, n);
    }
}

// the engine's single-thread fdbcs_batch_add, as a separate (noinline) call per transaction
struct Stage {
    uint8_t* pin;
    uint64_t* toff;
    size_t used;
    int64_t T, R, W;
};
__attribute__((noinline)) int add_txn(Stage* st, int64_t snap, const Range* reads, int nreads, const Range* writes,
                                      int nwrites) {
    const int n = nreads + nwrites;
    uint64_t kbytes = 0;
    for (int i = 0; i < n; i++) {
        const Range& rg = i < nreads ? reads[i] : writes[i - nreads];
        if (rg.bl > 30001 || rg.el > 30001) return -6;
        if (kcmp(rg.b, rg.bl, rg.e, rg.el) >= 0) return -3;
        kbytes += (uint64_t)rg.bl + rg.el;
    }
    const size_t rec = (sizeof(Hdr) + 8 * (size_t)n + kbytes + 7) & ~size_t(7);
    uint8_t* p = st->pin + st->used;
    const Hdr h{snap, (int32_t)st->R, (int32_t)st->W, nreads, nwrites};
    memcpy(p, &h, sizeof h);
    uint32_t* lens = reinterpret_cast<uint32_t*>(p + sizeof h);
    uint8_t* kp = p + sizeof h + 8 * (size_t)n;
    for (int i = 0; i < n; i++) {
        const Range& rg = i < nreads ? reads[i] : writes[i - nreads];
        lens[2 * i] = rg.bl;
        lens[2 * i + 1] = rg.el;
        copy_small(kp, rg.b, rg.bl);
        kp += rg.bl;
        copy_small(kp, rg.e, rg.el);
        kp += rg.el;
    }
    st->toff[st->T] = st->used;
    st->used += rec;
    st->T++;
    st->R += nreads;
    st->W += nwrites;
    return 0;
}

// one pass: reads then writes, validate + copy together
__attribute__((noinline)) int add_txn2(Stage* st, int64_t snap, const Range* reads, int nreads, const Range* writes,
                                       int nwrites) {
    const int n = nreads + nwrites;
    uint8_t* p = st->pin + st->used;
    uint32_t* lens = reinterpret_cast<uint32_t*>(p + sizeof(Hdr));
    uint8_t* kp = p + sizeof(Hdr) + 8 * (size_t)n;
    int bad = 0;
    auto put = [&](const Range& rg) {
        bad |= (rg.bl > 30001) | (rg.el > 30001) | (kcmp(rg.b, rg.bl, rg.e, rg.el) >= 0);
        lens[0] = rg.bl;
        lens[1] = rg.el;
        lens += 2;
        copy_small(kp, rg.b, rg.bl);
        kp += rg.bl;
        copy_small(kp, rg.e, rg.el);
        kp += rg.el;
    };
    for (int i = 0; i < nreads; i++) put(reads[i]);
    for (int i = 0; i < nwrites; i++) put(writes[i]);
    if (bad) return -3;
    const Hdr h{snap, (int32_t)st->R, (int32_t)st->W, nreads, nwrites};
    memcpy(p, &h, sizeof h);
    const size_t rec = ((size_t)(kp - p) + 7) & ~size_t(7);
    st->toff[st->T] = st->used;
    st->used += rec;
    st->T++;
    st->R += nreads;
    st->W += nwrites;
    return 0;
}

struct Batch {
    std::vector<uint8_t> bytes;
    std::vector<Range> reads, writes;
    std::vector<int64_t> snap;
};

int main(int argc, char** argv) {
    const int T = 5000, NB = argc > 1 ? atoi(argv[1]) : 40;
    std::vector<Batch> bs(NB);
    uint64_t x = 88172645463325252ull;
    auto rnd = [&]() { x ^= x << 13; x ^= x >> 7; x ^= x << 17; return x; };
    for (auto& B : bs) {
        B.bytes.resize((size_t)T * 7 * 2 * 17);
        B.reads.resize(T * 5);
        B.writes.resize(T * 2);
        B.snap.resize(T);
        for (int r = 0; r < T * 7; r++) {
            uint8_t* p = &B.bytes[(size_t)r * 34];
            uint64_t a = rnd(), c = rnd();
            memcpy(p, &a, 8); memcpy(p + 8, &c, 8);
            memcpy(p + 17, p, 16); p[33] = 0;
            Range rg{p, 16, p + 17, 17};
            if (r < T * 5) B.reads[r] = rg; else B.writes[r - T * 5] = rg;
        }
    }
    uint8_t* stream = (uint8_t*)aligned_alloc(64, 8 << 20);
#ifdef WITH_HIP
    uint8_t* dstage = nullptr;
    const bool dma = argc > 3 && atoi(argv[3]);
    if (argc > 2) {  // the stream in hipHostMalloc'd (pinned) memory, flags argv[2]
        if (hipHostMalloc((void**)&stream, 8 << 20, (unsigned)atoi(argv[2])) != hipSuccess) return 1;
        if (hipMalloc((void**)&dstage, 8 << 20) != hipSuccess) return 1;
        printf("stream: hipHostMalloc flags %s%s\n", argv[2], dma ? ", copied H2D after every batch" : "");
    }
#endif
    uint64_t* toff = (uint64_t*)aligned_alloc(64, 1 << 20);
    Range* desc = (Range*)aligned_alloc(64, 4 << 20);
    memset(stream, 0, 8 << 20);
    memset(desc, 0, 4 << 20);
    for (int variant = 0; variant < 8; variant++) {
        double tot = 0;
        long bad = 0;
        for (int i = 0; i < NB; i++) {
            const Batch& B = bs[i];
#ifdef WITH_HIP
            if (dma) hipMemcpy(dstage, stream, 2 << 20, hipMemcpyHostToDevice);  // as the engine's chunk copies
#endif
            if (variant == 3) {  // warm: touch the batch first (untimed)
                volatile uint64_t s = 0;
                for (size_t k = 0; k < B.bytes.size(); k += 64) s += B.bytes[k];
                for (size_t k = 0; k < B.reads.size(); k += 2) s += B.reads[k].bl;
                for (size_t k = 0; k < B.writes.size(); k += 2) s += B.writes[k].bl;
            }
            const auto t0 = clk::now();
            if (variant >= 6) {
                Stage st{stream, toff, 0, 0, 0, 0};
                for (int t = 0; t < T; t++)
                    bad += (variant == 6 ? add_txn : add_txn2)(&st, B.snap[t], B.reads.data() + 5 * t, 5,
                                                               B.writes.data() + 2 * t, 2);
                tot += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
                continue;
            }
            size_t used = 0;
            int R = 0, W = 0;
            for (int t = 0; t < T; t++) {
                const Range* rd = B.reads.data() + 5 * t;
                const Range* wr = B.writes.data() + 2 * t;
                const int n = 7;
                if (variant == 5) {  // read the descriptors only
                    for (int k = 0; k < n; k++) {
                        const Range& rg = k < 5 ? rd[k] : wr[k - 5];
                        bad += rg.bl + rg.el;
                    }
                    continue;
                }
                if (variant == 2) {  // descriptors only
                    for (int k = 0; k < n; k++) {
                        const Range& rg = k < 5 ? rd[k] : wr[k - 5];
                        bad += kcmp(rg.b, rg.bl, rg.e, rg.el) >= 0;
                        desc[R + W + k] = rg;
                    }
                    R += 5; W += 2;
                    continue;
                }
                uint64_t kb = 0;
                for (int k = 0; k < n; k++) {
                    const Range& rg = k < 5 ? rd[k] : wr[k - 5];
                    if (variant != 4) bad += kcmp(rg.b, rg.bl, rg.e, rg.el) >= 0;
                    kb += rg.bl + rg.el;
                }
                const size_t rec = (sizeof(Hdr) + 8 * n + kb + 7) & ~size_t(7);
                uint8_t* p = stream + used;
                const Hdr h{B.snap[t], R, W, 5, 2};
                if (variant == 1) {
                    // non-temporal: assemble the record in a stack buffer, stream it out in 8-byte stores
                    alignas(16) uint8_t buf[512];
                    memcpy(buf, &h, sizeof h);
                    uint32_t* lens = (uint32_t*)(buf + sizeof h);
                    uint8_t* kp = buf + sizeof h + 8 * n;
                    for (int k = 0; k < n; k++) {
                        const Range& rg = k < 5 ? rd[k] : wr[k - 5];
                        lens[2 * k] = rg.bl; lens[2 * k + 1] = rg.el;
                        copy_small(kp, rg.b, rg.bl); kp += rg.bl;
                        copy_small(kp, rg.e, rg.el); kp += rg.el;
                    }
                    for (size_t q = 0; q < rec; q += 8) _mm_stream_si64((long long*)(p + q), *(long long*)(buf + q));
                } else {
                    memcpy(p, &h, sizeof h);
                    uint32_t* lens = (uint32_t*)(p + sizeof h);
                    uint8_t* kp = p + sizeof h + 8 * n;
                    for (int k = 0; k < n; k++) {
                        const Range& rg = k < 5 ? rd[k] : wr[k - 5];
                        lens[2 * k] = rg.bl; lens[2 * k + 1] = rg.el;
                        copy_small(kp, rg.b, rg.bl); kp += rg.bl;
                        copy_small(kp, rg.e, rg.el); kp += rg.el;
                    }
                }
                toff[t] = used;
                used += rec;
                R += 5; W += 2;
            }
            if (variant == 1) _mm_sfence();
            tot += std::chrono::duration<double, std::micro>(clk::now() - t0).count();
        }
        const char* name[] = {"append (engine.hip)", "append, non-temporal stores", "descriptors only", "append, warm inputs", "append, no compare", "read descriptors only", "engine add (call per txn)", "one-pass add (call per txn)"};
        printf("%-30s %8.1f us per 5,000-txn batch (bad %ld)\n", name[variant], tot / NB, bad);
    }
    return 0;
}
