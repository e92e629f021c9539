// Microbenchmark: LDS bitonic sort of 1024 records per workgroup (sample-sort building block).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>
#include "../../foundationdb_amd/csrc/common.h"
using namespace fdbcs_dev;

__device__ inline bool lt3(uint64_t ah, uint64_t al, uint64_t am, uint64_t bh, uint64_t bl, uint64_t bm) {
    return (ah < bh) | ((ah == bh) & ((al < bl) | ((al == bl) & (am < bm))));
}

// V3: plain key compare, SoA, 1 pair per thread-iteration
template <int P>
__global__ __launch_bounds__(256) void k_v3(const uint64_t* in, uint64_t* out) {
    __shared__ uint64_t H[P], L[P], M[P];
    const uint64_t* src = in + (size_t)blockIdx.x * 3 * P;
    for (int i = threadIdx.x; i < P; i += 256) { H[i] = src[3*i]; L[i] = src[3*i+1]; M[i] = src[3*i+2]; }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
        for (int j = k >> 1; j > 0; j >>= 1) {
            for (int i = threadIdx.x; i < P / 2; i += 256) {
                const int a = ((i & ~(j - 1)) << 1) | (i & (j - 1)), b = a | j;
                uint64_t ah = H[a], al = L[a], am = M[a], bh = H[b], bl = L[b], bm = M[b];
                const bool up = (a & k) == 0;
                const bool sw = up ? lt3(bh, bl, bm, ah, al, am) : lt3(ah, al, am, bh, bl, bm);
                if (sw) { H[a] = bh; L[a] = bl; M[a] = bm; H[b] = ah; L[b] = al; M[b] = am; }
            }
            __syncthreads();
        }
    uint64_t* dst = out + (size_t)blockIdx.x * 3 * P;
    for (int i = threadIdx.x; i < P; i += 256) { dst[3*i] = H[i]; dst[3*i+1] = L[i]; dst[3*i+2] = M[i]; }
}

// V4: register-resident: each thread keeps 4 records; steps with j < 4 are done in registers,
// larger j through LDS exchange.  (P = 1024, 256 threads)
__global__ __launch_bounds__(256) void k_v4(const uint64_t* in, uint64_t* out) {
    constexpr int P = 1024;
    __shared__ uint64_t H[P], L[P], M[P];
    const uint64_t* src = in + (size_t)blockIdx.x * 3 * P;
    uint64_t h[4], l[4], m[4];
    const int t = threadIdx.x;
    for (int q = 0; q < 4; q++) { int i = 4 * t + q; h[q] = src[3*i]; l[q] = src[3*i+1]; m[q] = src[3*i+2]; }
    for (int k = 2; k <= P; k <<= 1) {
        for (int j = k >> 1; j > 0; j >>= 1) {
            if (j >= 4) {
                // exchange through LDS: write all, sync, read partner, compare
                for (int q = 0; q < 4; q++) { int i = 4 * t + q; H[i] = h[q]; L[i] = l[q]; M[i] = m[q]; }
                __syncthreads();
                for (int q = 0; q < 4; q++) {
                    int i = 4 * t + q, p = i ^ j;
                    uint64_t ph = H[p], pl = L[p], pm = M[p];
                    bool up = (i & k) == 0;
                    bool lower = i < p;
                    bool plt = lt3(ph, pl, pm, h[q], l[q], m[q]);
                    // lower position keeps min if up
                    bool take = (lower == up) ? plt : !plt;
                    if (take) { h[q] = ph; l[q] = pl; m[q] = pm; }
                }
                __syncthreads();
            } else {
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    int i = 4 * t + q, p = i ^ j;
                    if (p > i) {
                        int pq = q ^ j;
                        bool up = (i & k) == 0;
                        bool sw = up ? lt3(h[pq], l[pq], m[pq], h[q], l[q], m[q]) : lt3(h[q], l[q], m[q], h[pq], l[pq], m[pq]);
                        if (sw) { uint64_t x; x = h[q]; h[q] = h[pq]; h[pq] = x; x = l[q]; l[q] = l[pq]; l[pq] = x; x = m[q]; m[q] = m[pq]; m[pq] = x; }
                    }
                }
            }
        }
    }
    uint64_t* dst = out + (size_t)blockIdx.x * 3 * P;
    for (int q = 0; q < 4; q++) { int i = 4 * t + q; dst[3*i] = h[q]; dst[3*i+1] = l[q]; dst[3*i+2] = m[q]; }
}

int main() {
    const int P = 1024, NB = 176;
    std::vector<uint64_t> h(3 * P * NB);
    uint64_t x = 88172645463325252ull;
    for (auto& v : h) { x ^= x << 13; x ^= x >> 7; x ^= x << 17; v = x; }
    uint64_t *din, *dout;
    hipMalloc(&din, h.size() * 8); hipMalloc(&dout, h.size() * 8);
    hipMemcpy(din, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    auto timeit = [&](const char* name, auto launch) {
        for (int w = 0; w < 3; w++) launch();
        hipDeviceSynchronize();
        hipEventRecord(e0);
        for (int it = 0; it < 20; it++) launch();
        hipEventRecord(e1); hipEventSynchronize(e1);
        float ms; hipEventElapsedTime(&ms, e0, e1);
        std::vector<uint64_t> o(h.size()); hipMemcpy(o.data(), dout, o.size() * 8, hipMemcpyDeviceToHost);
        bool ok = true;
        for (int b = 0; b < NB && ok; b++) for (int i = 1; i < P; i++) {
            const uint64_t* p = &o[(size_t)b * 3 * P + 3 * (i - 1)]; const uint64_t* q = p + 3;
            if (std::make_tuple(q[0], q[1], q[2]) < std::make_tuple(p[0], p[1], p[2])) { ok = false; break; }
        }
        printf("%-28s %8.2f us/launch  sorted=%d\n", name, ms * 1000 / 20, ok);
    };
    timeit("v3 SoA 1 pair/iter", [&] { hipLaunchKernelGGL(k_v3<1024>, dim3(NB), dim3(256), 0, 0, din, dout); });
    timeit("v4 regs(4/thr)+LDS", [&] { hipLaunchKernelGGL(k_v4, dim3(NB), dim3(256), 0, 0, din, dout); });
    timeit("v3 P=256", [&] { hipLaunchKernelGGL(k_v3<256>, dim3(NB), dim3(256), 0, 0, din, dout); });
    return 0;
}
