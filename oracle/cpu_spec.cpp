// cpu_spec.cpp -- C++ CPU restatement of the Resolver conflict-set semantics.
//
// TEST INFRASTRUCTURE ONLY.  Built into oracle/liboracle_spec.so and loaded
// by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, only
// as the checker / reported CPU baseline.  The product library
// (foundationdb_amd/libfdbcs.so) never links or calls it.
//
// PARITY UNPINNED (see oracle/spec.py header and DESIGN.md §Oracle): the
// reference fdbserver/SkipList.cpp is unbuildable here without stand-ins for
// its flow/boost headers, which the task forbids, and it ships no golden
// vectors.  This file restates SURVEY.md Appendix A, citing the reference
// lines each step follows, and is differential-tested against the naive
// oracle/spec.py on random streams (tests/test_oracle.py).
//
// Layout: the history (the reference's SkipList, SkipList.cpp:281-867) is a
// vector of sorted chunks of (key, version) so that searches are
// O(log H) and edits are O(chunk); level randomness in the reference never
// affects results, so any ordered container is valid.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "../include/fdbcs.h"

namespace {

typedef std::string Key;

// compare(): SkipList.cpp:113-120 -- unsigned bytewise, shorter first.
static inline int cmpk(const uint8_t* a, size_t al, const uint8_t* b, size_t bl) {
    size_t n = al < bl ? al : bl;
    int c = n ? memcmp(a, b, n) : 0;
    if (c) return c < 0 ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}
static inline int cmpk(const Key& a, const Key& b) {
    return cmpk((const uint8_t*)a.data(), a.size(), (const uint8_t*)b.data(), b.size());
}

struct Chunk {
    std::vector<Key> k;
    std::vector<int64_t> v;
    int64_t mx = INT64_MIN;
    void remax() {
        mx = INT64_MIN;
        for (int64_t x : v) mx = std::max(mx, x);
    }
};

struct Pos {
    size_t c, i;
};

struct History {
    static const size_t kSplit = 512, kTarget = 256;
    int64_t v0 = 0;
    std::vector<Chunk> ch;  // no empty chunks

    size_t nch() const { return ch.size(); }
    bool valid(Pos p) const { return p.c < ch.size(); }
    Pos end() const { return Pos{ch.size(), 0}; }
    const Key& key(Pos p) const { return ch[p.c].k[p.i]; }
    int64_t ver(Pos p) const { return ch[p.c].v[p.i]; }
    Pos next(Pos p) const {
        if (++p.i >= ch[p.c].k.size()) { p.c++; p.i = 0; }
        return p;
    }
    int64_t size() const {
        int64_t n = 0;
        for (auto& c : ch) n += c.k.size();
        return n;
    }
    // first position with key >= k
    Pos lower_bound(const Key& k) const {
        // last chunk whose first key <= k
        size_t lo = 0, hi = ch.size();
        while (lo < hi) {
            size_t mid = (lo + hi) / 2;
            if (cmpk(ch[mid].k[0], k) <= 0) lo = mid + 1; else hi = mid;
        }
        if (lo == 0) return Pos{0, 0};
        size_t c = lo - 1;
        auto& kk = ch[c].k;
        size_t i = std::lower_bound(kk.begin(), kk.end(), k,
                                    [](const Key& a, const Key& b) { return cmpk(a, b) < 0; }) - kk.begin();
        if (i == kk.size()) return Pos{c + 1, 0};
        return Pos{c, i};
    }
    // version of the last boundary < k (position p = lower_bound(k)), else v0
    int64_t value_before(Pos p) const {
        if (p.i > 0) return ch[p.c].v[p.i - 1];
        if (p.c > 0) return ch[p.c - 1].v.back();
        return v0;
    }
    void fix_chunk(size_t c) {  // split an oversize chunk, drop an empty one
        Chunk& x = ch[c];
        if (x.k.empty()) { ch.erase(ch.begin() + c); return; }
        if (x.k.size() <= kSplit) { x.remax(); return; }
        size_t n = x.k.size(), parts = (n + kTarget - 1) / kTarget;
        std::vector<Chunk> out(parts);
        for (size_t p = 0; p < parts; p++) {
            size_t a = n * p / parts, b = n * (p + 1) / parts;
            out[p].k.assign(std::make_move_iterator(x.k.begin() + a), std::make_move_iterator(x.k.begin() + b));
            out[p].v.assign(x.v.begin() + a, x.v.begin() + b);
            out[p].remax();
        }
        ch.erase(ch.begin() + c);
        ch.insert(ch.begin() + c, std::make_move_iterator(out.begin()), std::make_move_iterator(out.end()));
    }

    // Spec step 1: conflict iff max over [b,e) (plus valueBefore(b) when b is
    // not a boundary) > snap.  SkipList.cpp:755-837 (CheckMax).
    bool read_conflict(const Key& b, const Key& e, int64_t snap) const {
        Pos p = lower_bound(b);
        if (!(valid(p) && key(p) == b)) {
            if (value_before(p) > snap) return true;
        }
        // scan boundaries with b <= key < e
        while (valid(p)) {
            const Chunk& c = ch[p.c];
            if (p.i == 0 && c.mx <= snap && cmpk(c.k.back(), e) < 0) {  // whole chunk inside, no conflict
                p.c++;
                continue;
            }
            for (size_t i = p.i; i < c.k.size(); i++) {
                if (cmpk(c.k[i], e) >= 0) return false;
                if (c.v[i] > snap) return true;
            }
            p.c++;
            p.i = 0;
        }
        return false;
    }

    // Spec step 4 for one range, applied last-to-first as in
    // SkipList::addConflictRanges (SkipList.cpp:511-522): keep the pre-write
    // value at e (insert e with valueBefore(e) if e is not a boundary), erase
    // [b, e), insert b with `now`.
    void apply_write(const Key& b, const Key& e, int64_t now) {
        Pos pe = lower_bound(e);
        bool found = valid(pe) && key(pe) == e;
        int64_t vb = found ? 0 : value_before(pe);
        Pos pb = lower_bound(b);
        if (ch.empty()) {
            ch.emplace_back();
            pb = Pos{0, 0};
        } else if (!valid(pb)) {
            pb = Pos{ch.size() - 1, ch.back().k.size()};  // b above every key: append
        } else if (valid(pe) && pe.c == pb.c) {           // erase [pb, pe) inside one chunk
            Chunk& c = ch[pb.c];
            c.k.erase(c.k.begin() + pb.i, c.k.begin() + pe.i);
            c.v.erase(c.v.begin() + pb.i, c.v.begin() + pe.i);
        } else {                                          // erase [pb, pe) across chunks
            size_t ce = valid(pe) ? pe.c : ch.size();
            Chunk& c = ch[pb.c];
            c.k.resize(pb.i);
            c.v.resize(pb.i);
            if (valid(pe)) {  // pe.i < size, so chunk pe.c stays non-empty
                Chunk& d = ch[pe.c];
                d.k.erase(d.k.begin(), d.k.begin() + pe.i);
                d.v.erase(d.v.begin(), d.v.begin() + pe.i);
                d.remax();
            }
            if (ce > pb.c + 1) ch.erase(ch.begin() + pb.c + 1, ch.begin() + ce);
        }
        Chunk& c = ch[pb.c];
        c.k.insert(c.k.begin() + pb.i, b);
        c.v.insert(c.v.begin() + pb.i, now);
        if (!found) {
            c.k.insert(c.k.begin() + pb.i + 1, e);
            c.v.insert(c.v.begin() + pb.i + 1, vb);
        }
        fix_chunk(pb.c);
    }

    // Spec step 6: SkipList::removeBefore (SkipList.cpp:665-702) over the
    // window driven by ConflictBatch::detectConflicts (:1198-1206).
    void remove_before(int64_t oldest, Key& removal_key, int64_t budget) {
        Pos p = lower_bound(removal_key);
        bool prev_above = true;  // first scanned node always kept
        size_t first_c = p.c;
        std::vector<std::pair<size_t, std::vector<char>>> marks;  // per touched chunk keep flags
        while (valid(p) && budget > 0) {
            budget--;
            if (marks.empty() || marks.back().first != p.c)
                marks.emplace_back(p.c, std::vector<char>(ch[p.c].k.size(), 1));
            bool above = ver(p) >= oldest;
            if (!(above || prev_above)) marks.back().second[p.i] = 0;
            prev_above = above;
            p = next(p);
        }
        removal_key = valid(p) ? key(p) : Key();
        (void)first_c;
        // apply removals from the back so chunk indices stay valid
        for (auto it = marks.rbegin(); it != marks.rend(); ++it) {
            Chunk& c = ch[it->first];
            size_t w = 0;
            for (size_t i = 0; i < c.k.size(); i++) {
                if (!it->second[i]) continue;
                if (w != i) { c.k[w] = std::move(c.k[i]); c.v[w] = c.v[i]; }
                w++;
            }
            c.k.resize(w);
            c.v.resize(w);
            fix_chunk(it->first);
        }
    }
};

struct Oracle {
    History h;
    int64_t oldest = 0;  // ConflictSet::oldestVersion (SkipList.cpp:950)
    Key removal_key;     // ConflictSet::removalKey (SkipList.cpp:949)
};

struct Point {      // KeyInfo (SkipList.cpp:134-144)
    const uint8_t* k;
    uint32_t len;
    uint8_t type;   // tie digit: readEnd 0 < writeEnd 1 < writeBegin 2 < readBegin 3 (SkipList.cpp:169-172)
    int32_t idx;    // range index (reads: r, writes: R + w)
};

static inline bool point_less(const Point& a, const Point& b) {
    int c = cmpk(a.k, a.len, b.k, b.len);
    if (c) return c < 0;
    return a.type < b.type;
}

}  // namespace

extern "C" {

void* orc_create(int64_t v0) {
    Oracle* o = new Oracle();
    o->h.v0 = v0;
    return o;
}
void orc_destroy(void* p) { delete (Oracle*)p; }
void orc_clear(void* p, int64_t v) {  // clearConflictSet: SkipList.cpp:957-959
    Oracle* o = (Oracle*)p;
    o->h.ch.clear();
    o->h.v0 = v;
}
int64_t orc_size(void* p) { return ((Oracle*)p)->h.size(); }
int64_t orc_v0(void* p) { return ((Oracle*)p)->h.v0; }
int64_t orc_oldest(void* p) { return ((Oracle*)p)->oldest; }
int32_t orc_removal_key(void* p, uint8_t* buf, int32_t cap) {
    Oracle* o = (Oracle*)p;
    int32_t n = (int32_t)o->removal_key.size();
    if (buf) memcpy(buf, o->removal_key.data(), std::min(n, cap));
    return n;
}

// detectConflicts over a whole packed batch (addTransaction x T then
// detectConflicts: SkipList.cpp:979-1008, 1163-1208).
int orc_detect(void* p, const fdbcs_batch_view* b, int64_t now, int64_t new_oldest, uint8_t* verdict) {
    Oracle* o = (Oracle*)p;
    const int T = b->txn_count, R = b->read_count, W = b->write_count;
    auto key_of = [&](int64_t slot) {
        return Key((const char*)b->key_bytes + b->key_off[slot], b->key_len[slot]);
    };
    for (int64_t s = 0; s < 2 * (int64_t)(R + W); s += 2) {
        if (cmpk(b->key_bytes + b->key_off[s], b->key_len[s], b->key_bytes + b->key_off[s + 1], b->key_len[s + 1]) >= 0)
            return FDBCS_E_RANGE;
    }
    // addTransaction: tooOld = snapshot < oldest && has reads (SkipList.cpp:985)
    std::vector<char> too_old(T), conflict(T, 0);
    for (int t = 0; t < T; t++)
        too_old[t] = b->snapshot[t] < o->oldest && b->read_off[t + 1] > b->read_off[t];
    // 1. history read check (SkipList.cpp:1173, 1210-1233)
    for (int t = 0; t < T; t++) {
        if (too_old[t]) continue;
        for (int r = b->read_off[t]; r < b->read_off[t + 1] && !conflict[t]; r++)
            if (o->h.read_conflict(key_of(2 * (int64_t)r), key_of(2 * (int64_t)r + 1), b->snapshot[t])) conflict[t] = 1;
    }
    // 2. intra-batch: endpoints sorted with the tie digit (sortPoints,
    //    SkipList.cpp:227-279), rank = point index, bitset "any"/"set"
    //    (MiniConflictSet, :1028-1130; driver :1133-1153).
    std::vector<Point> pts;
    pts.reserve(2 * (size_t)(R + W));
    for (int t = 0; t < T; t++) {
        if (too_old[t]) continue;
        for (int r = b->read_off[t]; r < b->read_off[t + 1]; r++) {
            int64_t s = 2 * (int64_t)r;
            pts.push_back({b->key_bytes + b->key_off[s], b->key_len[s], 3, r});
            pts.push_back({b->key_bytes + b->key_off[s + 1], b->key_len[s + 1], 0, r});
        }
        for (int w = b->write_off[t]; w < b->write_off[t + 1]; w++) {
            int64_t s = 2 * (int64_t)R + 2 * (int64_t)w;
            pts.push_back({b->key_bytes + b->key_off[s], b->key_len[s], 2, R + w});
            pts.push_back({b->key_bytes + b->key_off[s + 1], b->key_len[s + 1], 1, R + w});
        }
    }
    std::sort(pts.begin(), pts.end(), point_less);
    std::vector<int32_t> rb(R + W), re(R + W);
    for (size_t i = 0; i < pts.size(); i++) {
        if (pts[i].type >= 2) rb[pts[i].idx] = (int32_t)i; else re[pts[i].idx] = (int32_t)i;
    }
    const size_t P = pts.size();
    std::vector<uint64_t> bits((P + 63) / 64 + 1, 0), blk((P + 4095) / 4096 + 1, 0);  // blk: any bit in 4096-bit block
    auto any = [&](int32_t a, int32_t e) -> bool {  // any bit in [a, e)
        while (a < e) {
            if ((a & 4095) == 0 && a + 4096 <= e) {
                if (blk[a >> 12]) {
                    for (int32_t w = a >> 6; w < (a + 4096) >> 6; w++) if (bits[w]) return true;
                }
                a += 4096;
                continue;
            }
            int32_t w = a >> 6, lo = a & 63;
            int32_t hi = std::min<int32_t>(64, lo + (e - a));
            uint64_t m = (hi == 64 ? ~0ull : ((1ull << hi) - 1)) & ~((1ull << lo) - 1);
            if (bits[w] & m) return true;
            a += hi - lo;
        }
        return false;
    };
    auto set = [&](int32_t a, int32_t e) {
        for (int32_t i = a; i < e;) {
            int32_t w = i >> 6, lo = i & 63;
            int32_t hi = std::min<int32_t>(64, lo + (e - i));
            uint64_t m = (hi == 64 ? ~0ull : ((1ull << hi) - 1)) & ~((1ull << lo) - 1);
            bits[w] |= m;
            blk[i >> 12] = 1;
            i += hi - lo;
        }
    };
    for (int t = 0; t < T; t++) {
        if (conflict[t]) continue;
        bool c = too_old[t];
        for (int r = b->read_off[t]; r < b->read_off[t + 1] && !c && !too_old[t]; r++)
            if (any(rb[r], re[r])) c = true;
        conflict[t] = c;
        if (!c)
            for (int w = b->write_off[t]; w < b->write_off[t + 1]; w++) set(rb[R + w], re[R + w]);
    }
    // 3. combineWriteConflictRanges (SkipList.cpp:1320-1337)
    std::vector<std::pair<Key, Key>> comb;
    {
        int active = 0;
        for (auto& pt : pts) {
            if (pt.idx < R) continue;
            int w = pt.idx - R;
            // owner of write w
            int t = int(std::upper_bound(b->write_off, b->write_off + T + 1, w) - b->write_off) - 1;
            if (conflict[t]) continue;
            if (pt.type == 2) {
                if (++active == 1) comb.emplace_back(Key((const char*)pt.k, pt.len), Key());
            } else {
                if (--active == 0) comb.back().second = Key((const char*)pt.k, pt.len);
            }
        }
    }
    // 4. mergeWriteConflictRanges: ranges applied last to first
    //    (SkipList.cpp:1235-1258, 511-522)
    for (size_t j = comb.size(); j-- > 0;) o->h.apply_write(comb[j].first, comb[j].second, now);
    // 5. verdicts (SkipList.cpp:1188-1196; Resolver.actor.cpp:159-166)
    for (int t = 0; t < T; t++)
        verdict[t] = !conflict[t] ? FDBCS_COMMITTED : (too_old[t] ? FDBCS_TOO_OLD : FDBCS_CONFLICT);
    // 6. compaction window (SkipList.cpp:1198-1206)
    if (new_oldest > o->oldest) {
        o->oldest = new_oldest;
        o->h.remove_before(o->oldest, o->removal_key, 3 * (int64_t)comb.size() + 10);
    }
    return FDBCS_OK;
}

int64_t orc_dump(void* p, int64_t cap, int64_t* versions, uint32_t* key_len, uint64_t* key_off,
                 uint8_t* key_bytes, uint64_t key_bytes_cap) {
    Oracle* o = (Oracle*)p;
    int64_t n = 0;
    uint64_t off = 0;
    for (auto& c : o->h.ch) {
        for (size_t i = 0; i < c.k.size(); i++) {
            if (n >= cap || off + c.k[i].size() > key_bytes_cap) return FDBCS_E_CAPACITY;
            versions[n] = c.v[i];
            key_len[n] = (uint32_t)c.k[i].size();
            key_off[n] = off;
            memcpy(key_bytes + off, c.k[i].data(), c.k[i].size());
            off += c.k[i].size();
            n++;
        }
    }
    return n;
}

int orc_load(void* p, int64_t n, const int64_t* versions, const uint32_t* key_len, const uint64_t* key_off,
             const uint8_t* key_bytes, int64_t v0, int64_t oldest, const uint8_t* rk, uint32_t rk_len) {
    Oracle* o = (Oracle*)p;
    o->h.ch.clear();
    o->h.v0 = v0;
    o->oldest = oldest;
    o->removal_key = Key((const char*)rk, rk_len);
    for (int64_t i = 0; i < n; i += History::kTarget) {
        Chunk c;
        for (int64_t j = i; j < std::min<int64_t>(n, i + History::kTarget); j++) {
            c.k.emplace_back((const char*)key_bytes + key_off[j], key_len[j]);
            c.v.push_back(versions[j]);
        }
        c.remax();
        o->h.ch.push_back(std::move(c));
    }
    return FDBCS_OK;
}

// fdbcs_nth_after's restatement (config 4's generator): the key
// of the boundary steps[i] positions after the first boundary >= key i.
int orc_nth_after(void* p, int32_t n, const uint8_t* key_bytes, const uint64_t* key_off, const uint32_t* key_len,
                  const int64_t* steps, uint8_t* out, uint32_t out_stride, int32_t* out_len) {
    const History& h = ((Oracle*)p)->h;
    for (int32_t q = 0; q < n; q++) {
        Pos pos = h.lower_bound(Key((const char*)key_bytes + key_off[q], key_len[q]));
        int64_t left = steps[q];
        while (h.valid(pos) && left > 0) {  // whole chunks, then within one
            const int64_t room = (int64_t)h.ch[pos.c].k.size() - (int64_t)pos.i;
            if (left >= room) {
                left -= room;
                pos = Pos{pos.c + 1, 0};
            } else {
                pos.i += (size_t)left;
                left = 0;
            }
        }
        if (!h.valid(pos)) {
            out_len[q] = -1;
            continue;
        }
        const Key& k = h.key(pos);
        out_len[q] = (int32_t)k.size();
        if (k.size() <= out_stride) memcpy(out + (size_t)q * out_stride, k.data(), k.size());
    }
    return 0;
}

}  // extern "C"
