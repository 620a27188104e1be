// Copy-pattern sweep (tuning tool): what streaming shape reaches the highest
// read+write bandwidth on this MI355X?  Variants: chunk per wave-iteration,
// grid size, non-temporal loads/stores.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int U, int NTL, int NTS>
__global__ __launch_bounds__(256) void copyk(const u4* __restrict__ src, u4* __restrict__ dst, int64_t units)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t u = wave; u < units; u += nw) {
        u4 v[U];
        const u4* s = src + u * U * 64 + lane;
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = NTL ? __builtin_nontemporal_load(s + k * 64) : s[k * 64];
        u4* d = dst + u * U * 64 + lane;
#pragma unroll
        for (int k = 0; k < U; ++k) {
            if (NTS) __builtin_nontemporal_store(v[k], d + k * 64); else d[k * 64] = v[k];
        }
    }
}

template <int U, int NTL, int NTS>
void run(u4* src, u4* dst, size_t bytes, int grid)
{
    const int64_t units = bytes / (U * 1024);
    hipLaunchKernelGGL((copyk<U, NTL, NTS>), dim3(grid), dim3(256), 0, 0, src, dst, units);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((copyk<U, NTL, NTS>), dim3(grid), dim3(256), 0, 0, src, dst, units);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("copy U=%2d ntl=%d nts=%d grid %6d : %7.1f GB/s (r+w)\n", U, NTL, NTS, grid,
           2.0 * 5 * units * U * 1024 / (ms * 1e-3) / 1e9);
}

int main()
{
    const size_t bytes = 8ull << 30;
    u4 *src, *dst;
    (void)hipMalloc(&src, bytes);
    (void)hipMalloc(&dst, bytes);
    (void)hipMemset(src, 1, bytes);
    (void)hipMemset(dst, 0, bytes);
    for (int grid : {1024, 4096, 16384, 65536}) {
        run<1, 0, 0>(src, dst, bytes, grid);
        run<4, 0, 0>(src, dst, bytes, grid);
        run<8, 0, 0>(src, dst, bytes, grid);
        run<4, 1, 0>(src, dst, bytes, grid);
        run<4, 0, 1>(src, dst, bytes, grid);
        run<4, 1, 1>(src, dst, bytes, grid);
    }
    return 0;
}
