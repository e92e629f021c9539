// devutil.h -- wave64 / workgroup scan and reduction helpers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace fdbcs_dev {

template <typename T>
__device__ inline T wave_incl_scan(T x) {
    const int lane = threadIdx.x & 63;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        T y = __shfl_up(x, d, 64);
        if (lane >= d) x += y;
    }
    return x;
}

template <typename T>
__device__ inline T wave_reduce_sum(T x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) x += __shfl_xor(x, d, 64);
    return x;
}

template <typename T>
__device__ inline T wave_reduce_max(T x) {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        T y = __shfl_xor(x, d, 64);
        x = y > x ? y : x;
    }
    return x;
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
