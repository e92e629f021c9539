// devutil.h -- wave64 / workgroup scan and reduction helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <limits>

namespace fdbcs_dev {

// Wave64 scans and reductions on DPP lane moves (row_shr within 16-lane rows,
// then row_bcast:15 / row_bcast:31 across rows), which run on the VALU at
// register latency -- __shfl_* would lower to ds_bpermute round trips.
// Lanes whose DPP source is outside the row (or whose row is masked) read
// `identity`.
template <int CTRL, int RM = 0xf>
__device__ inline uint32_t dpp32(uint32_t identity, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, RM, 0xf, false);
}

template <int CTRL, int RM = 0xf, typename T>
__device__ inline T dpp_move(T identity, T v) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, dpp32<CTRL, RM>(__builtin_bit_cast(uint32_t, identity), __builtin_bit_cast(uint32_t, v)));
    } else {
        static_assert(sizeof(T) == 8, "32- or 64-bit lanes");
        const uint64_t i = __builtin_bit_cast(uint64_t, identity), x = __builtin_bit_cast(uint64_t, v);
        const uint64_t lo = dpp32<CTRL, RM>((uint32_t)i, (uint32_t)x);
        const uint64_t hi = dpp32<CTRL, RM>((uint32_t)(i >> 32), (uint32_t)(x >> 32));
        return __builtin_bit_cast(T, lo | (hi << 32));
    }
}

template <typename T, typename Op>
__device__ inline T wave_incl_scan_op(T x, T identity, Op op) {
    x = op(x, dpp_move<0x111>(identity, x));       // row_shr:1
    x = op(x, dpp_move<0x112>(identity, x));       // row_shr:2
    x = op(x, dpp_move<0x114>(identity, x));       // row_shr:4
    x = op(x, dpp_move<0x118>(identity, x));       // row_shr:8
    x = op(x, dpp_move<0x142, 0xa>(identity, x));  // row_bcast:15 -> rows 1, 3
    x = op(x, dpp_move<0x143, 0xc>(identity, x));  // row_bcast:31 -> rows 2, 3
    return x;
}

template <typename T>
__device__ inline T wave_read_lane(T v, int lane) {
    if constexpr (sizeof(T) == 4) {
        return __builtin_bit_cast(T, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), lane));
    } else {
        const uint64_t x = __builtin_bit_cast(uint64_t, v);
        const uint64_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)x, lane);
        const uint64_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(x >> 32), lane);
        return __builtin_bit_cast(T, lo | (hi << 32));
    }
}

template <typename T>
__device__ inline T wave_incl_scan(T x) {
    return wave_incl_scan_op(x, T(0), [](T a, T b) { return a + b; });
}

// Full-wave reductions (every lane active) broadcast the result to all lanes.
template <typename T>
__device__ inline T wave_reduce_sum(T x) {
    return wave_read_lane(wave_incl_scan(x), 63);
}

template <typename T>
__device__ inline T wave_reduce_min(T x) {
    const T highest = std::numeric_limits<T>::max();
    return wave_read_lane(wave_incl_scan_op(x, highest, [](T a, T b) { return a < b ? a : b; }), 63);
}

template <typename T>
__device__ inline T wave_reduce_max(T x) {
    const T lowest = std::numeric_limits<T>::lowest();
    return wave_read_lane(wave_incl_scan_op(x, lowest, [](T a, T b) { return a > b ? a : b; }), 63);
}

// Exclusive scan across the workgroup.  `tmp` must hold blockDim.x/64 + 1
// elements of LDS.  Every thread must call it.  Returns the exclusive prefix;
// `total` receives the workgroup sum.
template <typename T>
__device__ inline T block_excl_scan(T v, T* tmp, T& total) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T x = wave_incl_scan(v);
    if (lane == 63) tmp[wid] = x;
    __syncthreads();
    if (wid == 0) {  // scan of the wave totals by one wavefront
        const T y = lane < nw ? tmp[lane] : T(0);
        const T z = wave_incl_scan(y);
        if (lane < nw) tmp[lane] = z - y;
        if (lane == nw - 1) tmp[nw] = z;
    }
    __syncthreads();
    T r = x - v + tmp[wid];
    total = tmp[nw];
    __syncthreads();
    return r;
}

template <typename T>
__device__ inline T block_reduce_sum(T v, T* tmp) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T x = wave_reduce_sum(v);
    if (lane == 0) tmp[wid] = x;
    __syncthreads();
    T s = 0;
    for (int w = 0; w < nw; w++) s += tmp[w];
    __syncthreads();
    return s;
}

template <typename T>
__device__ inline T block_reduce_max(T v, T* tmp) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
    T x = wave_reduce_max(v);
    if (lane == 0) tmp[wid] = x;
    __syncthreads();
    T s = tmp[0];
    for (int w = 1; w < nw; w++) s = tmp[w] > s ? tmp[w] : s;
    __syncthreads();
    return s;
}

}  // namespace fdbcs_dev
