// host_write_devmem.hip -- can the host write device memory directly (large
// BAR), and how fast?  Fine-grained device memory (hipExtMallocWithFlags
// hipDeviceMallocFinegrained), written by the CPU as the staging stream would
// be (16- and 24-byte pieces in order), then read by a kernel.
//   hipcc --offload-arch=gfx950 -O2 -o /tmp/hwd scripts/micro/host_write_devmem.hip && /tmp/hwd
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_sum(const uint64_t* p, size_t n, unsigned long long* out) {
    unsigned long long s = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += p[i];
    atomicAdd(out, s);
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
    const size_t bytes = 2 << 20;
    for (int mode = 0; mode < 3; mode++) {
        void* d = nullptr;
        hipError_t e;
        const char* name;
        if (mode == 0) {
            name = "hipExtMallocWithFlags(Finegrained)";
            e = hipExtMallocWithFlags(&d, bytes, hipDeviceMallocFinegrained);
        } else if (mode == 1) {
            name = "hipExtMallocWithFlags(Uncached)";
            e = hipExtMallocWithFlags(&d, bytes, hipDeviceMallocUncached);
        } else {
            name = "hipHostMalloc(Mapped|Coherent) (host memory, for comparison)";
            e = hipHostMalloc(&d, bytes, hipHostMallocMapped | hipHostMallocCoherent);
        }
        printf("%s: %s ptr %p\n", name, hipGetErrorString(e), d);
        if (e != hipSuccess) continue;
        hipPointerAttribute_t at{};
        hipPointerGetAttributes(&at, d);
        printf("  attr type %d hostPointer %p devicePointer %p\n", (int)at.type, at.hostPointer, at.devicePointer);
        uint8_t* h = (uint8_t*)(at.hostPointer ? at.hostPointer : d);
        // host writes: 24-byte headers and 16-byte keys in order, like the stage
        std::vector<uint8_t> src(64, 7);
        for (int rep = 0; rep < 3; rep++) {
            const double t0 = now_us();
            size_t o = 0;
            uint64_t k = 0;
            while (o + 64 <= bytes) {
                memcpy(h + o, src.data(), 24);
                o += 24;
                for (int j = 0; j < 7 && o + 16 <= bytes; j++) {
                    k++;
                    memcpy(h + o, &k, 8);
                    memcpy(h + o + 8, &k, 8);
                    o += 16;
                }
            }
            __atomic_thread_fence(__ATOMIC_SEQ_CST);
            const double t1 = now_us();
            printf("  host wrote %zu bytes in pieces: %.1f us (%.2f GB/s)\n", o, t1 - t0, o / (t1 - t0) / 1e3);
        }
        unsigned long long* out;
        hipMalloc(&out, 8);
        hipMemset(out, 0, 8);
        k_sum<<<256, 256>>>((const uint64_t*)d, bytes / 8, out);
        unsigned long long r = 0;
        hipMemcpy(&r, out, 8, hipMemcpyDeviceToHost);
        printf("  kernel sum %llu (%s)\n", r, hipGetErrorString(hipDeviceSynchronize()));
        hipFree(out);
        if (mode < 2) hipFree(d);
        else hipHostFree(d);
    }
    return 0;
}
