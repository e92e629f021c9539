// Back-to-back launch cost on one stream (hipEvent timing, no profiler):
// empty kernels of a few shapes, and a dependent chain of tiny kernels that
// each read what the previous one wrote.
//   hipcc --offload-arch=gfx950 -O3 scripts/micro/launch_cost.hip -o /tmp/launch_cost && /tmp/launch_cost
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1023 && blockIdx.x == 1 << 30) p[0] = 1;
}
__global__ void k_chain(int* p) {
    if (threadIdx.x == 0 && blockIdx.x == 0) p[0] = p[0] + 1;
}
__global__ void k_lds(int* p) {
    __shared__ int s[16384];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    if (p && s[(threadIdx.x + 1) & 1023] == -1) p[0] = 1;
}

int main() {
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int* d;
    hipMalloc(&d, 4096);
    hipMemset(d, 0, 4096);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    struct Shape { const char* name; int kind, blocks, threads; } shapes[] = {
        {"empty 1x64", 0, 1, 64},       {"empty 2x1024", 0, 2, 1024}, {"empty 64x256", 0, 64, 256},
        {"empty 1024x256", 0, 1024, 256}, {"chain 1x64", 1, 1, 64},   {"lds64K 2x1024", 2, 2, 1024},
    };
    for (auto& sh : shapes) {
        for (int rep = 0; rep < 3; rep++) {
            const int n = 2000;
            hipEventRecord(a, s);
            for (int i = 0; i < n; i++) {
                if (sh.kind == 0) hipLaunchKernelGGL(k_empty, dim3(sh.blocks), dim3(sh.threads), 0, s, d);
                else if (sh.kind == 1) hipLaunchKernelGGL(k_chain, dim3(sh.blocks), dim3(sh.threads), 0, s, d);
                else hipLaunchKernelGGL(k_lds, dim3(sh.blocks), dim3(sh.threads), 0, s, d);
            }
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("%-16s rep %d: %.2f us per launch\n", sh.name, rep, 1000.0 * ms / n);
        }
    }
    // the same empty kernels from a captured graph (no host launch cost per kernel)
    for (int blocks : {1, 64, 1024}) {
        const int n = 200;
        hipGraph_t g;
        hipGraphExec_t ge;
        hipStreamBeginCapture(s, hipStreamCaptureModeGlobal);
        for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_empty, dim3(blocks), dim3(256), 0, s, d);
        hipStreamEndCapture(s, &g);
        hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
        hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
        for (int rep = 0; rep < 3; rep++) {
            hipEventRecord(a, s);
            for (int k = 0; k < 10; k++) hipGraphLaunch(ge, s);
            hipEventRecord(b, s);
            hipEventSynchronize(b);
            float ms;
            hipEventElapsedTime(&ms, a, b);
            printf("graph empty %4dx256 rep %d: %.2f us per kernel\n", blocks, rep, 1000.0 * ms / (10 * n));
        }
    }
    // host enqueue rate alone: launches into a stream held back by a long kernel
    return 0;
}
