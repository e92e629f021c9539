// host_path_micro.hip -- costs that bound the Resolver's per-transaction path
// (addTransaction x T + detectConflicts, Resolver.actor.cpp:140-153) on one
// MI355X box: HIP call overheads, H2D streaming, zero-copy reads, host append.
//   hipcc -O2 --offload-arch=gfx950 -o /tmp/hpm scripts/micro/host_path_micro.hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                  \
    do {                                                                       \
        hipError_t e = (x);                                                    \
        if (e != hipSuccess) {                                                 \
            printf("HIP error %s at %d\n", hipGetErrorString(e), __LINE__);    \
            return 1;                                                          \
        }                                                                      \
    } while (0)

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1000000) p[0] = 1;
}

// zero-copy: copy n bytes from host-mapped memory to device memory
__global__ void k_zc(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const size_t MB2 = 2 << 20;
    uint8_t *pin, *dev, *mapped, *mapped_dev;
    CK(hipHostMalloc((void**)&pin, 8 * MB2, hipHostMallocDefault));
    CK(hipHostMalloc((void**)&mapped, 8 * MB2, hipHostMallocMapped));
    CK(hipHostGetDevicePointer((void**)&mapped_dev, mapped, 0));
    CK(hipMalloc((void**)&dev, 8 * MB2));
    memset(pin, 1, 8 * MB2);
    memset(mapped, 1, 8 * MB2);
    // warm
    for (int i = 0; i < 20; i++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
    CK(hipMemcpyAsync(dev, pin, MB2, hipMemcpyHostToDevice, s));
    CK(hipStreamSynchronize(s));

    // 1. launch overhead (CPU time per launch), and launch+sync round trip
    {
        const int N = 2000;
        auto a = clk::now();
        for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
        auto b = clk::now();
        CK(hipStreamSynchronize(s));
        auto c = clk::now();
        printf("launch: %.2f us CPU per launch, %.2f us per kernel drained\n", us(a, b) / N, us(a, c) / N);
        double tot = 0;
        for (int i = 0; i < 200; i++) {
            auto x = clk::now();
            hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, nullptr);
            hipStreamSynchronize(s);
            tot += us(x, clk::now());
        }
        printf("launch+sync round trip: %.2f us\n", tot / 200);
    }
    // 2. H2D memcpy issue cost and bandwidth per size
    for (size_t sz : {(size_t)4096, (size_t)65536, (size_t)262144, (size_t)1 << 20, MB2, 4 * MB2}) {
        const int N = 200;
        double issue = 0;
        auto a = clk::now();
        for (int i = 0; i < N; i++) {
            auto x = clk::now();
            hipMemcpyAsync(dev, pin, sz, hipMemcpyHostToDevice, s);
            issue += us(x, clk::now());
        }
        CK(hipStreamSynchronize(s));
        auto c = clk::now();
        printf("H2D %8zu B: issue %.2f us CPU, %.2f us each drained (%.1f GB/s)\n", sz, issue / N, us(a, c) / N,
               sz / (us(a, c) / N) / 1e3);
    }
    // 3. one H2D + sync latency (small)
    {
        double tot = 0;
        for (int i = 0; i < 200; i++) {
            auto x = clk::now();
            hipMemcpyAsync(pin, dev, 5000, hipMemcpyDeviceToHost, s);
            hipStreamSynchronize(s);
            tot += us(x, clk::now());
        }
        printf("D2H 5000 B + sync: %.2f us\n", tot / 200);
    }
    // 4. zero-copy kernel read of host-mapped memory
    for (size_t sz : {(size_t)262144, MB2, 4 * MB2}) {
        for (int blocks : {256, 1024, 4096}) {
            const int N = 50;
            hipLaunchKernelGGL(k_zc, dim3(blocks), dim3(256), 0, s, (const uint4*)mapped_dev, (uint4*)dev, sz / 16);
            CK(hipStreamSynchronize(s));
            auto a = clk::now();
            for (int i = 0; i < N; i++)
                hipLaunchKernelGGL(k_zc, dim3(blocks), dim3(256), 0, s, (const uint4*)mapped_dev, (uint4*)dev,
                                   sz / 16);
            CK(hipStreamSynchronize(s));
            double t = us(a, clk::now()) / N;
            printf("zero-copy read %8zu B, %4d blocks: %.2f us (%.1f GB/s)\n", sz, blocks, t, sz / t / 1e3);
        }
    }
    // 5. host memcpy into pinned memory
    {
        std::vector<uint8_t> src(MB2, 3);
        auto a = clk::now();
        for (int i = 0; i < 50; i++) memcpy(pin + (i & 3) * MB2, src.data(), MB2);
        printf("host memcpy 2 MiB -> pinned: %.2f us\n", us(a, clk::now()) / 50);
    }
    // 6. host append of a config-2 batch (35,000 ranges of 16/17-byte keys):
    //    copy begin+end bytes, write (offset, lens), compare begin < end
    {
        const int NR = 35000;
        std::vector<uint8_t> keys((size_t)NR * 33);
        for (size_t i = 0; i < keys.size(); i++) keys[i] = (uint8_t)(i * 2654435761u >> 13);
        for (int r = 0; r < NR; r++) keys[(size_t)r * 33 + 16 + 16] = 0, memcpy(&keys[(size_t)r * 33 + 16], &keys[(size_t)r * 33], 16);
        struct Meta { uint64_t off; uint32_t bl, el; };
        Meta* meta = (Meta*)(pin + 4 * MB2);
        uint8_t* bytes = pin;
        double best = 1e9;
        int bad = 0;
        for (int it = 0; it < 20; it++) {
            auto a = clk::now();
            uint64_t off = 0;
            for (int r = 0; r < NR; r++) {
                const uint8_t* b = &keys[(size_t)r * 33];
                const uint8_t* e = b + 16;
                const uint32_t bl = 16, el = 17;
                const uint32_t n = bl < el ? bl : el;
                int c = memcmp(b, e, n);
                if (c > 0 || (c == 0 && bl >= el)) bad++;
                memcpy(bytes + off, b, bl);
                memcpy(bytes + off + bl, e, el);
                meta[r] = Meta{off, bl, el};
                off += bl + el;
            }
            best = std::min(best, us(a, clk::now()));
        }
        printf("host append 35,000 ranges (1.16 MB keys): %.2f us (bad %d)\n", best, bad);
    }
    CK(hipFree(dev));
    CK(hipHostFree(pin));
    CK(hipHostFree(mapped));
    return 0;
}
