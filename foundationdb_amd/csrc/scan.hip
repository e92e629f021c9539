// scan.hip -- device-wide exclusive scans whose length may live on the device.
//
// Three launches (reduce per segment -> scan of segment sums -> rescan with
// offsets) over a fixed grid, so that the element count can be produced by an
// earlier kernel on the same stream without a host round trip.
#include "kernels.h"
#include "devutil.h"

namespace fdbcs_dev {

static constexpr int SCAN_BLOCKS = 256;
static constexpr int SCAN_THREADS = 256;

template <typename TIn, typename TOut>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_reduce(const TIn* __restrict__ in, const int32_t* n_ptr,
                                                              int32_t n_host, TOut* __restrict__ bsum) {
    __shared__ TOut tmp[SCAN_THREADS / 64 + 1];
    const int n = n_ptr ? *n_ptr : n_host;
    const int seg = (n + gridDim.x - 1) / gridDim.x;
    const int beg = blockIdx.x * seg;
    const int end = min(n, beg + seg);
    TOut s = 0;
    for (int i = beg + threadIdx.x; i < end; i += blockDim.x) s += (TOut)in[i];
    s = block_reduce_sum(s, tmp);
    if (threadIdx.x == 0) bsum[blockIdx.x] = s;
}

template <typename TOut>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_top(TOut* __restrict__ bsum, int nb) {
    __shared__ TOut tmp[SCAN_THREADS / 64 + 1];
    TOut v = threadIdx.x < nb ? bsum[threadIdx.x] : 0;
    TOut total;
    TOut ex = block_excl_scan(v, tmp, total);
    if (threadIdx.x < nb) bsum[threadIdx.x] = ex;
    if (threadIdx.x == 0) bsum[nb] = total;
}

template <typename TIn, typename TOut>
__global__ __launch_bounds__(SCAN_THREADS) void k_scan_down(const TIn* __restrict__ in, TOut* __restrict__ out,
                                                            const int32_t* n_ptr, int32_t n_host,
                                                            const TOut* __restrict__ bsum, TOut* total_out) {
    __shared__ TOut tmp[SCAN_THREADS / 64 + 1];
    const int n = n_ptr ? *n_ptr : n_host;
    const int seg = (n + gridDim.x - 1) / gridDim.x;
    const int beg = blockIdx.x * seg;
    const int end = min(n, beg + seg);
    TOut carry = bsum[blockIdx.x];
    for (int base = beg; base < end; base += blockDim.x) {
        int i = base + threadIdx.x;
        TOut v = i < end ? (TOut)in[i] : 0;
        TOut tot;
        TOut ex = block_excl_scan(v, tmp, tot);
        if (i < end) out[i] = carry + ex;
        carry += tot;
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        out[n] = bsum[gridDim.x];
        if (total_out) *total_out = bsum[gridDim.x];
    }
}

template <typename TIn, typename TOut>
static void scan_impl(const TIn* in, TOut* out, const int32_t* n_ptr, int32_t n_host, TOut* total_out, int64_t* tmp,
                      hipStream_t s) {
    int nb = SCAN_BLOCKS;
    if (!n_ptr) nb = std::max(1, std::min(SCAN_BLOCKS, (n_host + 1023) / 1024));
    TOut* bsum = reinterpret_cast<TOut*>(tmp);
    hipLaunchKernelGGL((k_scan_reduce<TIn, TOut>), dim3(nb), dim3(SCAN_THREADS), 0, s, in, n_ptr, n_host, bsum);
    hipLaunchKernelGGL((k_scan_top<TOut>), dim3(1), dim3(SCAN_THREADS), 0, s, bsum, nb);
    hipLaunchKernelGGL((k_scan_down<TIn, TOut>), dim3(nb), dim3(SCAN_THREADS), 0, s, in, out, n_ptr, n_host, bsum,
                       total_out);
}

void scan_i32(const int32_t* in, int32_t* out, const int32_t* n_ptr, int32_t n_host, int32_t* total_out,
              int64_t* tmp, hipStream_t s) {
    scan_impl<int32_t, int32_t>(in, out, n_ptr, n_host, total_out, tmp, s);
}

void scan_i64_from_i32(const int32_t* in, int64_t* out, const int32_t* n_ptr, int32_t n_host, int64_t* total_out,
                       int64_t* tmp, hipStream_t s) {
    scan_impl<int32_t, int64_t>(in, out, n_ptr, n_host, total_out, tmp, s);
}

}  // namespace fdbcs_dev
