// Memory-only model of the pixel kernel's access pattern (tuning tool): per
// wave-task, 6 KiB of contiguous coefficient reads and 8 KiB of BGRX writes
// into a 3840x2160 frame batch, with different write shapes:
//   seg512: 128x16 px strips, each store instruction two 512-B row segments
//           (lanes 0-31 row y, 32-63 row y+2) -- the fused kernel today;
//   seg1k : 256x8 px strips, each store instruction one 1-KiB row segment;
// (A 512-px variant was dropped: 3840 is not a multiple of 512, its task
// count overran the frame and the kernel faulted -- run() now checks every
// shape's extent on the host before launching.)
// One task per wave, 4 waves per workgroup, tasks in frame raster order.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, PITCH = W * 4;

template <int kShape>   // 0 seg512, 1 seg1k
__global__ __launch_bounds__(256) void strips(const u4* __restrict__ coefs, uint8_t* __restrict__ out, int64_t tasks)
{
    const int lane = threadIdx.x & 63;
    const int64_t task = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (task >= tasks) return;
    // reads: 6 KiB contiguous, 6 x 1 KiB wave-loads
    const u4* src = coefs + task * 384 + lane;
    u4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < 6; ++k) acc ^= __builtin_nontemporal_load(src + 64 * k);
    constexpr int kStripW = kShape == 0 ? 128 : 256;
    constexpr int kRows = 2048 / kStripW;
    constexpr int kStrips = W / kStripW;
    const int64_t per_frame = static_cast<int64_t>(kStrips) * (H / kRows);
    const int64_t f = task / per_frame;
    const int64_t t = task - f * per_frame;
    const int sy = static_cast<int>(t / kStrips), sx = static_cast<int>(t % kStrips);
    uint8_t* base = out + f * static_cast<int64_t>(PITCH) * H + static_cast<int64_t>(sy * kRows) * PITCH + sx * kStripW * 4;
    if constexpr (kShape == 0) {
        const int x = (lane & 31) * 16, y0 = 2 * (lane >> 5);
#pragma unroll
        for (int it = 0; it < 4; ++it)
#pragma unroll
            for (int h = 0; h < 2; ++h)
                __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(base + (4 * it + h + y0) * PITCH + x));
    } else if constexpr (kShape == 1) {
#pragma unroll
        for (int y = 0; y < 8; ++y) __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(base + y * PITCH + lane * 16));
    }
}

template <int kShape>
static void run(const u4* coefs, uint8_t* out, int frames, const char* name, size_t in_bytes, size_t out_bytes)
{
    constexpr int kStripW = kShape == 0 ? 128 : 256, kRows = 2048 / kStripW;
    static_assert(W % kStripW == 0 && H % kRows == 0, "strips must tile the frame exactly");
    const int64_t tasks = static_cast<int64_t>(frames) * (W / kStripW) * (H / kRows);
    if (static_cast<size_t>(tasks) * 6144 > in_bytes || static_cast<size_t>(frames) * PITCH * H > out_bytes) {
        printf("%s: extent check failed, not launched\n", name);
        return;
    }
    const unsigned grid = static_cast<unsigned>((tasks + 3) / 4);
    hipLaunchKernelGGL((strips<kShape>), dim3(grid), dim3(256), 0, 0, coefs, out, tasks);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((strips<kShape>), dim3(grid), dim3(256), 0, 0, coefs, out, tasks);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double bytes = static_cast<double>(tasks) * (6144 + 8192);
    printf("%-7s %d frames: %7.1f GB/s (r+w), %.3f ms/launch\n", name, frames, bytes * 5 / (ms * 1e-3) / 1e9, ms / 5);
}

int main()
{
    const int frames = 128;
    const size_t out_bytes = static_cast<size_t>(frames) * PITCH * H;
    const size_t in_bytes = static_cast<size_t>(frames) * (W * H / 2048) * 6144;
    u4* coefs;
    uint8_t* out;
    (void)hipMalloc(&coefs, in_bytes);
    (void)hipMalloc(&out, out_bytes);
    (void)hipMemset(coefs, 1, in_bytes);
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(coefs, out, frames, "seg512", in_bytes, out_bytes);
        run<1>(coefs, out, frames, "seg1k", in_bytes, out_bytes);
    }
    return 0;
}
