// Streaming bandwidth ceiling for a given read:write byte mix (tuning tool).
// Each wave: loads R 1-KiB chunks (16 B/lane, coalesced) then stores W chunks,
// persistent grid; reports (read + written bytes) / time.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

template <int R, int W, bool NT>
__global__ __launch_bounds__(256) void mix(const uint4* __restrict__ src, uint4* __restrict__ dst, int64_t units)
{
    const int lane = threadIdx.x & 63;
    const int64_t wave = (blockIdx.x * 256 + threadIdx.x) >> 6;
    const int64_t nw = (int64_t)gridDim.x * 4;
    for (int64_t u = wave; u < units; u += nw) {
        uint4 acc = make_uint4(0, 0, 0, 0);
        const uint4* s = src + u * R * 64;
#pragma unroll
        for (int k = 0; k < R; ++k) {
            uint4 v = s[k * 64 + lane];
            acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
        }
        uint4* d = dst + u * W * 64;
#pragma unroll
        for (int k = 0; k < W; ++k) {
            uint4 o = make_uint4(acc.x + k, acc.y, acc.z, acc.w);
            if constexpr (NT) {
                typedef unsigned int u4 __attribute__((ext_vector_type(4)));
                u4 x = {o.x, o.y, o.z, o.w};
                __builtin_nontemporal_store(x, reinterpret_cast<u4*>(d + k * 64 + lane));
            } else {
                d[k * 64 + lane] = o;
            }
        }
    }
}

template <int R, int W, bool NT>
void run(const char* name, uint4* src, uint4* dst, size_t budget_bytes, int grid)
{
    const int64_t units = budget_bytes / ((R + W) * 1024);
    hipLaunchKernelGGL((mix<R, W, NT>), dim3(grid), dim3(256), 0, 0, src, dst, units);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((mix<R, W, NT>), dim3(grid), dim3(256), 0, 0, src, dst, units);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double bytes = 5.0 * units * (R + W) * 1024;
    printf("%-28s grid %5d  %8.1f GB/s\n", name, grid, bytes / (ms * 1e-3) / 1e9);
}

int main()
{
    const size_t budget = 16ull << 30;   // 16 GiB of traffic per launch
    uint4 *src, *dst;
    (void)hipMalloc(&src, budget);
    (void)hipMalloc(&dst, budget);
    (void)hipMemset(src, 1, budget);
    (void)hipMemset(dst, 0, budget);
    for (int grid : {1024, 2048, 4096}) {
        run<6, 0, false>("read only (6:0)", src, dst, budget, grid);
        run<0, 8, false>("write only (0:8)", src, dst, budget, grid);
        run<0, 8, true>("write only nt (0:8)", src, dst, budget, grid);
        run<4, 4, false>("copy 1:1 (4:4)", src, dst, budget, grid);
        run<6, 8, false>("4:2:0 mix (6:8)", src, dst, budget, grid);
        run<6, 8, true>("4:2:0 mix nt (6:8)", src, dst, budget, grid);
        run<6, 4, false>("4:4:4 mix (6:4)", src, dst, budget, grid);
    }
    return 0;
}
