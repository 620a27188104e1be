// Probe: 1 MB host->device over PCIe -- DMA (hipMemcpyAsync) vs a kernel that
// reads the pinned host buffer directly (zero copy), timed with HIP events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
__global__ void pull(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n16)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}
int main()
{
    const size_t sizes[] = {256 << 10, 1 << 20, 4 << 20};
    void* h; CK(hipHostMalloc(&h, 8 << 20, hipHostMallocDefault));
    void* hc; CK(hipHostMalloc(&hc, 8 << 20, hipHostMallocCoherent));
    void* d; CK(hipMalloc(&d, 8 << 20));
    memset(h, 1, 8 << 20); memset(hc, 1, 8 << 20);
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
    printf("{\"rows\": [\n");
    bool first = true;
    for (size_t n : sizes) {
        for (int mode = 0; mode < 6; ++mode) {
            const int grids[] = {0, 64, 256, 1024, 256, 0};
            float best = 1e9f;
            for (int r = 0; r < 30; ++r) {
                CK(hipEventRecord(e0, s));
                if (mode == 0) CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
                else if (mode == 5) CK(hipMemcpyAsync(d, hc, n, hipMemcpyHostToDevice, s));
                else hipLaunchKernelGGL(pull, dim3(grids[mode]), dim3(256), 0, s, (const uint4*)(mode == 4 ? hc : h), (uint4*)d, n / 16);
                CK(hipEventRecord(e1, s));
                CK(hipEventSynchronize(e1));
                float ms; CK(hipEventElapsedTime(&ms, e0, e1));
                if (ms < best) best = ms;
            }
            const char* names[] = {"dma_default", "kernel_g64", "kernel_g256", "kernel_g1024", "kernel_g256_coherent", "dma_coherent"};
            printf("%s {\"bytes\": %zu, \"how\": \"%s\", \"us\": %.2f, \"GBps\": %.1f}", first ? "" : ",\n", n, names[mode], best * 1e3, n / (best * 1e-3) / 1e9);
            first = false;
        }
    }
    printf("\n]}\n");
    return 0;
}
