// resolvers.hip -- key-range resolvers: the proxy side of FoundationDB's
// multi-resolver scale-out, so that G conflict sets (one per GPU) present to
// the commit path exactly as G reference Resolvers do.
//
//   fdbcs_split_batch     ResolutionRequestBuilder::addTransaction
//                         (fdbserver/MasterProxyServer.actor.cpp:267-307) with
//                         a static key -> resolver map: resolver g owns
//                         [bound[g-1], bound[g]) (bound[-1] = "", bound[G-1] =
//                         +inf).  A transaction goes to resolver g iff one of
//                         its read or write ranges intersects g's keys; it
//                         carries every such range UNCLIPPED, in order, with
//                         its read_snapshot.  Transactions keep their order.
//   fdbcs_scatter_verdicts the proxy's combine (:558-569): verdict[t] = min
//                         over the resolvers that received t of their verdicts
//                         (TransactionCommitted when none did).  Each resolver
//                         scatters its sub-batch verdicts into a T-byte array
//                         prefilled with TransactionCommitted; the element-wise
//                         MIN over resolvers (an RCCL MIN all-reduce across
//                         GPUs) is the proxy's combined verdict.
// Metadata ("txnState") transactions are a proxy concern outside the
// conflict set and are not modelled.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>

#include "../../include/fdbcs.h"

namespace {

int kcmp_host(const uint8_t* a, uint32_t al, const uint8_t* b, uint32_t bl) {
    const uint32_t n = std::min(al, bl);
    const int c = n ? memcmp(a, b, n) : 0;
    if (c) return c < 0 ? -1 : 1;
    return al < bl ? -1 : (al > bl ? 1 : 0);
}

struct Bounds {
    int G;
    const uint8_t* bytes;
    const uint64_t* off;  // [G-1]
    const uint32_t* len;  // [G-1]
    // resolver owning key k: number of bounds <= k
    int owner(const uint8_t* k, uint32_t kl) const {
        int lo = 0, hi = G - 1;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (kcmp_host(bytes + off[mid], len[mid], k, kl) <= 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;
    }
    // does [b, e) intersect resolver g's keys [bound[g-1], bound[g])?
    bool hits(int g, const uint8_t* b, uint32_t bl, const uint8_t* e, uint32_t el) const {
        if (g > 0 && kcmp_host(e, el, bytes + off[g - 1], len[g - 1]) <= 0) return false;  // e <= lo
        if (g < G - 1 && kcmp_host(b, bl, bytes + off[g], len[g]) >= 0) return false;      // b >= hi
        return true;
    }
    // does a range ending at e end exactly at resolver g's first key?
    bool ends_at_lo(int g, const uint8_t* e, uint32_t el) const {
        return g > 0 && kcmp_host(e, el, bytes + off[g - 1], len[g - 1]) == 0;
    }
    // the writes an exact protocol-B shard needs: those intersecting its keys,
    // and those ending exactly at its first key (the shard holding a range's
    // end creates the end node, SURVEY.md §8e "splitter ends")
    bool write_hits(int g, const uint8_t* b, uint32_t bl, const uint8_t* e, uint32_t el, bool keep_all) const {
        return hits(g, b, bl, e, el) || (keep_all && ends_at_lo(g, e, el));
    }
};

__global__ __launch_bounds__(256) void k_scatter_verdicts(const uint8_t* __restrict__ sub,
                                                          const int32_t* __restrict__ index, int n,
                                                          uint8_t* __restrict__ global) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) global[index[i]] = sub[i];
}

}  // namespace

extern "C" {

static int split_batch(const fdbcs_batch_view* in, int32_t nres, const uint8_t* bound_bytes,
                       const uint64_t* bound_off, const uint32_t* bound_len, int32_t resolver,
                       fdbcs_batch_view* out, int64_t* snapshot, int32_t* read_off, int32_t* write_off,
                       uint64_t* key_off, uint32_t* key_len, int32_t* txn_index, bool keep_all) {
    if (!in || !out || nres < 1 || resolver < 0 || resolver >= nres) return FDBCS_E_ARG;
    if (nres > 1 && (!bound_bytes || !bound_off || !bound_len)) return FDBCS_E_ARG;
    for (int g = 1; g + 1 < nres; g++)
        if (kcmp_host(bound_bytes + bound_off[g - 1], bound_len[g - 1], bound_bytes + bound_off[g], bound_len[g]) >= 0)
            return FDBCS_E_ARG;  // bounds must ascend strictly
    const Bounds B{nres, bound_bytes, bound_off, bound_len};
    const int64_t T = in->txn_count, R = in->read_count;
    int32_t t_out = 0, r_out = 0, w_out = 0;
    // pass 1: which transactions, how many ranges of each kind
    read_off[0] = 0;
    write_off[0] = 0;
    for (int64_t t = 0; t < T; t++) {
        int nr = 0, nw = 0;
        for (int32_t r = in->read_off[t]; r < in->read_off[t + 1]; r++) {
            const uint64_t s = 2 * (uint64_t)r;
            if (B.hits(resolver, in->key_bytes + in->key_off[s], in->key_len[s], in->key_bytes + in->key_off[s + 1],
                       in->key_len[s + 1]))
                nr++;
        }
        for (int32_t w = in->write_off[t]; w < in->write_off[t + 1]; w++) {
            const uint64_t s = 2 * (uint64_t)R + 2 * (uint64_t)w;
            if (B.write_hits(resolver, in->key_bytes + in->key_off[s], in->key_len[s],
                             in->key_bytes + in->key_off[s + 1], in->key_len[s + 1], keep_all))
                nw++;
        }
        if (nr + nw == 0 && !keep_all) continue;
        snapshot[t_out] = in->snapshot[t];
        txn_index[t_out] = (int32_t)t;
        read_off[t_out + 1] = read_off[t_out] + nr;
        write_off[t_out + 1] = write_off[t_out] + nw;
        t_out++;
        r_out += nr;
        w_out += nw;
    }
    // pass 2: key slots (reads first, then writes), pointing into the input's key bytes
    int32_t rr = 0, ww = 0;
    for (int64_t t = 0; t < T; t++) {
        for (int32_t r = in->read_off[t]; r < in->read_off[t + 1]; r++) {
            const uint64_t s = 2 * (uint64_t)r;
            if (!B.hits(resolver, in->key_bytes + in->key_off[s], in->key_len[s], in->key_bytes + in->key_off[s + 1],
                        in->key_len[s + 1]))
                continue;
            key_off[2 * rr] = in->key_off[s];
            key_len[2 * rr] = in->key_len[s];
            key_off[2 * rr + 1] = in->key_off[s + 1];
            key_len[2 * rr + 1] = in->key_len[s + 1];
            rr++;
        }
        for (int32_t w = in->write_off[t]; w < in->write_off[t + 1]; w++) {
            const uint64_t s = 2 * (uint64_t)R + 2 * (uint64_t)w;
            if (!B.write_hits(resolver, in->key_bytes + in->key_off[s], in->key_len[s],
                              in->key_bytes + in->key_off[s + 1], in->key_len[s + 1], keep_all))
                continue;
            const uint64_t d = 2 * (uint64_t)r_out + 2 * (uint64_t)ww;
            key_off[d] = in->key_off[s];
            key_len[d] = in->key_len[s];
            key_off[d + 1] = in->key_off[s + 1];
            key_len[d + 1] = in->key_len[s + 1];
            ww++;
        }
    }
    *out = fdbcs_batch_view{};
    out->txn_count = t_out;
    out->read_count = r_out;
    out->write_count = w_out;
    out->snapshot = snapshot;
    out->read_off = read_off;
    out->write_off = write_off;
    out->key_off = key_off;
    out->key_len = key_len;
    out->key_bytes = in->key_bytes;
    out->key_bytes_len = in->key_bytes_len;
    return FDBCS_OK;
}

int fdbcs_split_batch(const fdbcs_batch_view* in, int32_t nres, const uint8_t* bound_bytes,
                      const uint64_t* bound_off, const uint32_t* bound_len, int32_t resolver,
                      fdbcs_batch_view* out, int64_t* snapshot, int32_t* read_off, int32_t* write_off,
                      uint64_t* key_off, uint32_t* key_len, int32_t* txn_index) {
    return split_batch(in, nres, bound_bytes, bound_off, bound_len, resolver, out, snapshot, read_off, write_off,
                       key_off, key_len, txn_index, false);
}

int fdbcs_split_batch_keep_all(const fdbcs_batch_view* in, int32_t nres, const uint8_t* bound_bytes,
                               const uint64_t* bound_off, const uint32_t* bound_len, int32_t resolver,
                               fdbcs_batch_view* out, int64_t* snapshot, int32_t* read_off, int32_t* write_off,
                               uint64_t* key_off, uint32_t* key_len, int32_t* txn_index) {
    return split_batch(in, nres, bound_bytes, bound_off, bound_len, resolver, out, snapshot, read_off, write_off,
                       key_off, key_len, txn_index, true);
}

int32_t fdbcs_key_owner(int32_t nres, const uint8_t* bound_bytes, const uint64_t* bound_off,
                        const uint32_t* bound_len, const uint8_t* key, uint32_t key_len) {
    if (nres < 1) return FDBCS_E_ARG;
    return Bounds{nres, bound_bytes, bound_off, bound_len}.owner(key, key_len);
}

int fdbcs_scatter_verdicts(fdbcs* cs, const uint8_t* dev_sub, const int32_t* dev_index, int32_t n,
                           uint8_t* dev_global) {
    if (n < 0 || (n && (!dev_sub || !dev_index || !dev_global))) return FDBCS_E_ARG;
    if (n == 0) return FDBCS_OK;
    hipStream_t s = cs ? (hipStream_t)fdbcs_stream(cs) : nullptr;
    hipLaunchKernelGGL(k_scatter_verdicts, dim3((n + 255) / 256), dim3(256), 0, s, dev_sub, dev_index, n, dev_global);
    return hipGetLastError() == hipSuccess ? FDBCS_OK : FDBCS_E_HIP;
}

}  // extern "C"
