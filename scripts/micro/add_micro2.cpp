// add_micro2.cpp -- host cost of TxnStage::add (stage.hip) on config-2-shaped
// batches (5,000 txns: 5 reads, 80 % point [k, k\0) / 20 % short, + 2 point
// writes; uniform 16-byte keys), inputs prepared ahead (cold, as in the
// bench's timed loop).  v0 = the engine's add as of round 3 (two passes, key
// prefetch, point ranges as k\0); v1 = one pass with a slack check instead of
// the sizing pass; v2 = v1 with the compare and copy of keys <= 24 bytes from
// the same loaded words.
//   g++ -O2 -march=native -o /tmp/am2 scripts/micro/add_micro2.cpp && /tmp/am2
#include <algorithm>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

struct Range {
    const uint8_t* begin;
    uint32_t begin_len;
    const uint8_t* end;
    uint32_t end_len;
};
struct Hdr {
    int64_t snap;
    int32_t ro, wo, nr, nw;
};
struct Ent {
    uint32_t kofs;
    uint16_t blen, elen;
};
constexpr uint16_t SHARED = 0x8000;
constexpr uint32_t MAXK = 30001;

static inline uint64_t ld64(const uint8_t* p) {
    uint64_t x;
    memcpy(&x, p, 8);
    return x;
}
static inline int key_cmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t n = std::min(al, bl);
    uint32_t i = 0;
    for (; i + 8 <= n; i += 8) {
        const uint64_t x = ld64(a + i), y = ld64(b + i);
        if (x != y) return __builtin_bswap64(x) < __builtin_bswap64(y) ? -1 : 1;
    }
    for (; i < n; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return al < bl ? -2 : (al > bl ? 1 : 0);
}
static inline void copy_small(uint8_t* d, const uint8_t* s, uint32_t n) {
    if (n >= 16 && n <= 32) {
        uint8_t t0[16], t1[16];
        memcpy(t0, s, 16);
        memcpy(t1, s + n - 16, 16);
        memcpy(d, t0, 16);
        memcpy(d + n - 16, t1, 16);
    } else if (n >= 8 && n < 16) {
        const uint64_t x = ld64(s), y = ld64(s + n - 8);
        memcpy(d, &x, 8);
        memcpy(d + n - 8, &y, 8);
    } else if (n > 32) {
        memcpy(d, s, n);
    } else {
        for (uint32_t i = 0; i < n; i++) d[i] = s[i];
    }
}

struct Stage {
    uint8_t* pin;
    uint64_t* toff;
    uint64_t used = 0, cap = 0;
    int64_t T = 0, R = 0, W = 0, K = 0;
};

static inline bool put_ranges0(const Range* rg, int n, Ent* ent, const uint8_t* rec, uint8_t*& kp) {
    bool bad = false;
    for (int i = 0; i < n; i++) {
        const uint8_t *b = rg[i].begin, *e = rg[i].end;
        const uint32_t bl = rg[i].begin_len, el = rg[i].end_len;
        const int c = key_cmp(b, bl, e, el);
        bad |= c >= 0;
        copy_small(kp, b, bl);
        if (c == -2 && el == bl + 1 && e[bl] == 0) {
            ent[i] = Ent{(uint32_t)(kp - rec), (uint16_t)bl, (uint16_t)(el | SHARED)};
            kp[bl] = 0;
            kp += bl + 1;
        } else {
            ent[i] = Ent{(uint32_t)(kp - rec), (uint16_t)bl, (uint16_t)el};
            copy_small(kp + bl, e, el);
            kp += bl + el;
        }
    }
    return bad;
}

__attribute__((noinline)) int add_v0(Stage* st, int64_t snap, const Range* reads, int nr, const Range* writes, int nw) {
    const int n = nr + nw;
    uint64_t kbytes = 0;
    uint32_t longest = 0;
    for (int i = 0; i < nr; i++) {
        kbytes += (uint64_t)reads[i].begin_len + reads[i].end_len;
        longest = std::max({longest, reads[i].begin_len, reads[i].end_len});
        __builtin_prefetch(reads[i].begin);
        __builtin_prefetch(reads[i].end);
    }
    for (int i = 0; i < nw; i++) {
        kbytes += (uint64_t)writes[i].begin_len + writes[i].end_len;
        longest = std::max({longest, writes[i].begin_len, writes[i].end_len});
        __builtin_prefetch(writes[i].begin);
        __builtin_prefetch(writes[i].end);
    }
    if (longest > MAXK) return -6;
    const uint64_t rec = (sizeof(Hdr) + 8 * (uint64_t)n + kbytes + 7) & ~uint64_t(7);
    if (st->used + rec + 8 * (uint64_t)(st->T + 1) + 16 > st->cap) return -9;
    uint8_t* p = st->pin + st->used;
    Ent* ent = reinterpret_cast<Ent*>(p + sizeof(Hdr));
    uint8_t* kp = p + sizeof(Hdr) + sizeof(Ent) * (size_t)n;
    bool bad = put_ranges0(reads, nr, ent, p, kp);
    bad |= put_ranges0(writes, nw, ent + nr, p, kp);
    if (bad) return -3;
    const uint64_t rec_used = ((uint64_t)(kp - p) + 7) & ~uint64_t(7);
    const Hdr h{snap, (int32_t)st->R, (int32_t)st->W, nr, nw};
    memcpy(p, &h, sizeof h);
    st->toff[st->T] = st->used;
    st->used += rec_used;
    st->T++;
    st->K += kbytes;
    st->R += nr;
    st->W += nw;
    return 0;
}

// one range; false: begin >= end.  Keys of <= 24 bytes compare and copy from
// the same loaded words; longer ones take the general path
static inline bool put_one(const Range& r, Ent& ent, const uint8_t* rec, uint8_t*& kp, uint64_t& kb) {
    const uint8_t *b = r.begin, *e = r.end;
    const uint32_t bl = r.begin_len, el = r.end_len;
    kb += (uint64_t)bl + el;
    int c;
    if (bl == 16 && el >= 16) {  // the common shape: 16-byte begin
        uint64_t b0, b1, e0, e1;
        memcpy(&b0, b, 8);
        memcpy(&b1, b + 8, 8);
        memcpy(&e0, e, 8);
        memcpy(&e1, e + 8, 8);
        memcpy(kp, &b0, 8);
        memcpy(kp + 8, &b1, 8);
        if (b0 != e0) c = __builtin_bswap64(b0) < __builtin_bswap64(e0) ? -1 : 1;
        else if (b1 != e1) c = __builtin_bswap64(b1) < __builtin_bswap64(e1) ? -1 : 1;
        else c = el > 16 ? -2 : 0;
        if (c == -2 && el == 17 && e[16] == 0) {
            ent = Ent{(uint32_t)(kp - rec), 16, (uint16_t)(17 | SHARED)};
            kp[16] = 0;
            kp += 17;
            return true;
        }
    } else {
        c = key_cmp(b, bl, e, el);
        copy_small(kp, b, bl);
        if (c == -2 && el == bl + 1 && e[bl] == 0) {
            ent = Ent{(uint32_t)(kp - rec), (uint16_t)bl, (uint16_t)(el | SHARED)};
            kp[bl] = 0;
            kp += bl + 1;
            return c < 0;
        }
    }
    ent = Ent{(uint32_t)(kp - rec), (uint16_t)bl, (uint16_t)el};
    copy_small(kp + bl, e, el);
    kp += bl + el;
    return c < 0;
}

template <bool FAST>
__attribute__((noinline)) int add_v1(Stage* st, int64_t snap, const Range* reads, int nr, const Range* writes, int nw) {
    const int n = nr + nw;
    // slack check instead of a sizing pass: every key fits in MAXK bytes
    const uint64_t worst = sizeof(Hdr) + 8 * (uint64_t)n + 2 * (uint64_t)MAXK * n + 8;
    if (st->used + worst + 8 * (uint64_t)(st->T + 1) + 16 > st->cap) return -9;  // (the engine: the sizing pass)
    uint8_t* p = st->pin + st->used;
    Ent* ent = reinterpret_cast<Ent*>(p + sizeof(Hdr));
    uint8_t* kp = p + sizeof(Hdr) + sizeof(Ent) * (size_t)n;
    bool ok = true;
    uint64_t kb = 0;
    uint32_t longest = 0;
    for (int i = 0; i < nr + nw; i++) {
        const Range& r = i < nr ? reads[i] : writes[i - nr];
        longest = std::max({longest, r.begin_len, r.end_len});
        if (FAST) {
            ok &= put_one(r, ent[i], p, kp, kb);
        } else {
            uint8_t* kp0 = kp;
            bool bad = put_ranges0(&r, 1, ent + i, p, kp);
            (void)kp0;
            ok &= !bad;
            kb += (uint64_t)r.begin_len + r.end_len;
        }
    }
    if (longest > MAXK) return -6;
    if (!ok) return -3;
    const Hdr h{snap, (int32_t)st->R, (int32_t)st->W, nr, nw};
    memcpy(p, &h, sizeof h);
    st->toff[st->T] = st->used;
    st->used += ((uint64_t)(kp - p) + 7) & ~uint64_t(7);
    st->T++;
    st->K += kb;
    st->R += nr;
    st->W += nw;
    return 0;
}

struct Batch {
    std::vector<uint8_t> bytes;
    std::vector<Range> reads, writes;
    std::vector<int64_t> snap;
};

int main() {
    const int T = 5000, NB = 40;
    uint64_t x = 88172645463325252ull;
    auto rnd = [&] {
        x ^= x << 13;
        x ^= x >> 7;
        x ^= x << 17;
        return x;
    };
    std::vector<Batch> bs(NB);
    for (auto& B : bs) {
        B.bytes.resize((size_t)T * 7 * 34);
        B.reads.resize(T * 5);
        B.writes.resize(T * 2);
        B.snap.resize(T);
        for (int r = 0; r < T * 7; r++) {
            uint8_t* p = &B.bytes[(size_t)r * 34];
            const uint64_t a = rnd(), b = rnd();
            memcpy(p, &a, 8);
            memcpy(p + 8, &b, 8);
            Range rg{p, 16, p + 17, 17};
            memcpy(p + 17, p, 16);
            p[33] = 0;
            if (r < T * 5 && rnd() % 5 == 0) {  // short read: end = begin + U[1,16] as a big-endian integer
                uint64_t lo = __builtin_bswap64(b) + 1 + rnd() % 16, hi = __builtin_bswap64(a) + (lo < 16);
                lo = __builtin_bswap64(lo);
                hi = __builtin_bswap64(hi);
                memcpy(p + 17, &hi, 8);
                memcpy(p + 25, &lo, 8);
                rg.end_len = 16;
            }
            if (r < T * 5) B.reads[r] = rg;
            else B.writes[r - T * 5] = rg;
        }
        for (int t = 0; t < T; t++) B.snap[t] = t;
    }
    std::vector<uint8_t> pin(8 << 20);
    std::vector<uint64_t> toff(T + 1);
    const char* names[] = {"v0 engine (2 passes)", "v1 one pass", "v2 one pass, fused <=16-B compare+copy"};
    for (int rep = 0; rep < 3; rep++) {
        for (int v = 0; v < 3; v++) {
            double tot = 0;
            long bad = 0;
            for (auto& B : bs) {
                Stage st{pin.data(), toff.data()};
                st.cap = pin.size();
                const auto t0 = std::chrono::steady_clock::now();
                for (int t = 0; t < T; t++) {
                    const Range* rd = B.reads.data() + 5 * t;
                    const Range* wr = B.writes.data() + 2 * t;
                    bad += v == 0 ? add_v0(&st, B.snap[t], rd, 5, wr, 2)
                                  : (v == 1 ? add_v1<false>(&st, B.snap[t], rd, 5, wr, 2)
                                            : add_v1<true>(&st, B.snap[t], rd, 5, wr, 2));
                }
                tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
                if (rep == 0 && &B == &bs[0]) printf("  (%s: %llu stream bytes)\n", names[v], (unsigned long long)st.used);
            }
            printf("%-42s %8.1f us per 5,000-txn batch (errors %ld)\n", names[v], tot / NB, bad);
        }
    }
}
