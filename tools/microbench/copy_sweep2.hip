// Streaming-shape sweep, part 2 (tuning tool): one-shot grids (every thread
// copies U 16-B chunks once), workgroup sizes, and pure-read / pure-write
// kernels, to find what reaches the guide's ~6.3 TB/s float4-copy figure
// (MI355X_MICROARCH.md "HBM3E peak BW") and what the read/write split costs.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));

template <int U, int NT, int BS>
__global__ __launch_bounds__(BS) void copy1(const u4* __restrict__ src, u4* __restrict__ dst)
{
    const int64_t base = (static_cast<int64_t>(blockIdx.x) * BS * U) + threadIdx.x;
    u4 v[U];
#pragma unroll
    for (int k = 0; k < U; ++k) v[k] = NT ? __builtin_nontemporal_load(src + base + k * BS) : src[base + k * BS];
#pragma unroll
    for (int k = 0; k < U; ++k) {
        if (NT) __builtin_nontemporal_store(v[k], dst + base + k * BS);
        else dst[base + k * BS] = v[k];
    }
}

template <int U, int NT, int BS>
__global__ __launch_bounds__(BS) void read1(const u4* __restrict__ src, unsigned* __restrict__ sink)
{
    const int64_t base = (static_cast<int64_t>(blockIdx.x) * BS * U) + threadIdx.x;
    unsigned acc = 0;
#pragma unroll
    for (int k = 0; k < U; ++k) {
        const u4 v = NT ? __builtin_nontemporal_load(src + base + k * BS) : src[base + k * BS];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;   // keeps the loads
}

template <int U, int NT, int BS>
__global__ __launch_bounds__(BS) void write1(u4* __restrict__ dst)
{
    const int64_t base = (static_cast<int64_t>(blockIdx.x) * BS * U) + threadIdx.x;
    const u4 v = {static_cast<unsigned>(base), 1u, 2u, 3u};
#pragma unroll
    for (int k = 0; k < U; ++k) {
        if (NT) __builtin_nontemporal_store(v, dst + base + k * BS);
        else dst[base + k * BS] = v;
    }
}

template <typename F>
static float time_ms(F launch, int reps)
{
    launch();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < reps; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / reps;
}

template <int U, int NT, int BS>
static void run(u4* src, u4* dst, unsigned* sink, size_t bytes)
{
    const int64_t chunks = bytes / 16;
    const unsigned grid = static_cast<unsigned>(chunks / (BS * U));
    const float c = time_ms([&] { hipLaunchKernelGGL((copy1<U, NT, BS>), dim3(grid), dim3(BS), 0, 0, src, dst); }, 5);
    const float r = time_ms([&] { hipLaunchKernelGGL((read1<U, NT, BS>), dim3(grid), dim3(BS), 0, 0, src, sink); }, 5);
    const float w = time_ms([&] { hipLaunchKernelGGL((write1<U, NT, BS>), dim3(grid), dim3(BS), 0, 0, dst); }, 5);
    printf("one-shot U=%d nt=%d bs=%4d grid %8u : copy %7.1f GB/s (r+w)  read %7.1f GB/s  write %7.1f GB/s\n", U, NT,
           BS, grid, 2.0 * bytes / (c * 1e-3) / 1e9, bytes / (r * 1e-3) / 1e9, bytes / (w * 1e-3) / 1e9);
}

int main()
{
    const size_t bytes = 4ull << 30;
    u4 *src, *dst;
    unsigned* sink;
    (void)hipMalloc(&src, bytes);
    (void)hipMalloc(&dst, bytes);
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(src, 1, bytes);
    (void)hipMemset(dst, 0, bytes);
    run<1, 0, 256>(src, dst, sink, bytes);
    run<1, 1, 256>(src, dst, sink, bytes);
    run<2, 0, 256>(src, dst, sink, bytes);
    run<2, 1, 256>(src, dst, sink, bytes);
    run<4, 0, 256>(src, dst, sink, bytes);
    run<4, 1, 256>(src, dst, sink, bytes);
    run<1, 0, 1024>(src, dst, sink, bytes);
    run<1, 1, 1024>(src, dst, sink, bytes);
    run<4, 1, 1024>(src, dst, sink, bytes);
    run<8, 1, 256>(src, dst, sink, bytes);
    return 0;
}
