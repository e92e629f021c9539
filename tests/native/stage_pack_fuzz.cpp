// stage_pack_fuzz.cpp -- foundationdb_amd/csrc/stage_pack.h (the add's range
// check and copy) against a plain restatement, on random ranges: point ranges
// [k, k\x00), short ranges, equal and reversed keys, proper prefixes, lengths
// 0..100 with most at the configs' 16 / 17 (shared point ends above 32).  Built and run by
// tests/test_stage_pack.py (g++, no GPU).  Exit 0: identical records.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../foundationdb_amd/csrc/stage_pack.h"

struct Ent {
    uint32_t kofs;
    uint16_t blen, elen;
};
constexpr uint16_t SHARED = 0x8000;

// the reference's key order (SkipList.cpp:113-120): bytes, then length
static int ref_cmp(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t n = al < bl ? al : bl;
    const int c = n ? memcmp(a, b, n) : 0;
    if (c) return c < 0 ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

static bool ref_put(const fdbcs_range* rg, int n, Ent* ent, const uint8_t* rec, uint8_t*& kp,
                    uint32_t share_above = FDBCS_PACK_SHARE_ABOVE) {
    bool bad = false;
    for (int i = 0; i < n; i++) {
        const fdbcs_range& r = rg[i];
        if (ref_cmp(r.begin, r.begin_len, r.end, r.end_len) >= 0) bad = true;
        // (keys up to FDBCS_PACK_SHARE_ABOVE bytes are copied whole: no shared end)
        const bool point = r.begin_len > share_above && r.end_len == r.begin_len + 1 &&
                           memcmp(r.begin, r.end, r.begin_len) == 0 && r.end[r.begin_len] == 0;
        ent[i].kofs = (uint32_t)(kp - rec);
        ent[i].blen = (uint16_t)r.begin_len;
        memcpy(kp, r.begin, r.begin_len);
        if (point) {
            ent[i].elen = (uint16_t)(r.end_len | SHARED);
            kp[r.begin_len] = 0;
            kp += r.begin_len + 1;
        } else {
            ent[i].elen = (uint16_t)r.end_len;
            memcpy(kp + r.begin_len, r.end, r.end_len);
            kp += r.begin_len + r.end_len;
        }
    }
    return bad;
}

static uint64_t s = 88172645463325252ull;
static uint64_t rnd() {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    return s;
}

int main(int argc, char** argv) {
    const int rounds = argc > 1 ? atoi(argv[1]) : 20000;
    std::vector<uint8_t> arena(1 << 16);  // (8 ranges of two <= 101-byte keys)
    for (int it = 0; it < rounds; it++) {
        const int n = 1 + (int)(rnd() % 8);
        std::vector<fdbcs_range> rg(n);
        size_t used = 0;
        for (int i = 0; i < n; i++) {
            const uint32_t lens[] = {16, 16, 16, 17, 0, 1, 7, 8, 9, 15, 23, 24, 25, 31, 32, 33, 40, 41, 64, 100};
            uint32_t bl = lens[rnd() % 20];
            uint8_t* b = &arena[used];
            for (uint32_t k = 0; k < bl; k++) b[k] = (uint8_t)(rnd() % 4 == 0 ? 0 : rnd());
            used += bl;
            uint8_t* e = &arena[used];
            uint32_t el;
            switch (rnd() % 7) {
                case 0: case 1:  // point range
                    memcpy(e, b, bl); e[bl] = 0; el = bl + 1; break;
                case 2: {  // short range: the begin plus a small amount at byte j
                    memcpy(e, b, bl); el = bl;
                    if (bl) { const uint32_t j = (uint32_t)(rnd() % bl); e[j] = (uint8_t)(e[j] + 1 + rnd() % 3); }
                    break;
                }
                case 3:  // equal
                    memcpy(e, b, bl); el = bl; break;
                case 4: {  // proper prefix either way, or a longer end with a nonzero byte
                    memcpy(e, b, bl);
                    el = (uint32_t)(rnd() % (bl + 3));
                    for (uint32_t k = bl; k < el; k++) e[k] = (uint8_t)rnd();
                    break;
                }
                case 5:  // point-like but the extra byte is not zero
                    memcpy(e, b, bl); e[bl] = (uint8_t)(1 + rnd() % 255); el = bl + 1; break;
                default:  // random
                    el = lens[rnd() % 20];
                    for (uint32_t k = 0; k < el; k++) e[k] = (uint8_t)rnd();
            }
            used += el + 1;
            rg[i] = fdbcs_range{b, bl, e, el};
            if (el == 0 && rnd() % 2) rg[i].end = nullptr;  // (an empty key may come without a pointer)
            if (bl == 0 && rnd() % 2) rg[i].begin = nullptr;
        }
        std::vector<uint8_t> r1(4096, 0xAB), r2(4096, 0xAB);
        std::vector<Ent> e1(n), e2(n);
        uint8_t *k1 = r1.data(), *k2 = r2.data();
        const bool b1 = fdbcs_pack::put_ranges<Ent, SHARED>(rg.data(), n, e1.data(), r1.data(), k1);
        const bool b2 = ref_put(rg.data(), n, e2.data(), r2.data(), k2);
        bool ok = b1 == b2 && (k1 - r1.data()) == (k2 - r2.data()) && r1 == r2;
        for (int i = 0; ok && i < n; i++)
            ok = e1[i].kofs == e2[i].kofs && e1[i].blen == e2[i].blen && e1[i].elen == e2[i].elen;
        for (int i = 0; ok && i < n; i++) {  // and the compare alone, both ways
            const fdbcs_range& x = rg[i];
            const int c1 = fdbcs_pack::key_cmp(x.begin, x.begin_len, x.end, x.end_len);
            const int c2 = ref_cmp(x.begin, x.begin_len, x.end, x.end_len);
            const int d1 = fdbcs_pack::key_cmp(x.end, x.end_len, x.begin, x.begin_len);
            const int d2 = ref_cmp(x.end, x.end_len, x.begin, x.begin_len);
            ok = (c1 == -2 ? -1 : c1) == c2 && (d1 == -2 ? -1 : d1) == d2;
            if (ok && c1 == -2) ok = x.begin_len < x.end_len && (x.begin_len == 0 || !memcmp(x.begin, x.end, x.begin_len));
        }
        // the borrowed batches' pack (every point range shares its end) and
        // its size pass (stage.hip pack_borrowed): same records as the
        // restatement at threshold 0, and the size pass's bytes and status
        {
            std::vector<uint8_t> r3(4096, 0xAB), r4(4096, 0xAB);
            std::vector<Ent> e3(n), e4(n);
            uint8_t *k3 = r3.data(), *k4 = r4.data();
            const int nr = (int)(rnd() % (n + 1));
            const bool b3 = fdbcs_pack::put_ranges<Ent, SHARED, 0>(rg.data(), nr, e3.data(), r3.data(), k3) |
                            fdbcs_pack::put_ranges<Ent, SHARED, 0>(rg.data() + nr, n - nr, e3.data() + nr, r3.data(), k3);
            const bool b4 = ref_put(rg.data(), n, e4.data(), r4.data(), k4, 0);
            int st = 0;
            const uint64_t sz = fdbcs_pack::ranges_bytes<0>(rg.data(), nr, rg.data() + nr, n - nr, st);
            ok = ok && b3 == b4 && (k3 - r3.data()) == (k4 - r4.data()) && r3 == r4 &&
                 st == (b4 ? FDBCS_E_RANGE : FDBCS_OK) && (b4 || sz == (uint64_t)(k4 - r4.data()));
            for (int i = 0; ok && i < n; i++)
                ok = e3[i].kofs == e4[i].kofs && e3[i].blen == e4[i].blen && e3[i].elen == e4[i].elen;
        }
        if (!ok) {
            printf("mismatch at round %d (bad %d/%d, bytes %ld/%ld)\n", it, b1, b2, (long)(k1 - r1.data()),
                   (long)(k2 - r2.data()));
            return 1;
        }
    }
    printf("ok %d rounds\n", rounds);
    return 0;
}
