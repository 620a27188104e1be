// Memory-only model of the pixel kernel's access pattern, second sweep (tuning
// tool): does the per-wave task size, or the strip shape of the writes, set
// the 4:2:0 kernel's ~5.5 TB/s ceiling?  Every variant moves the same bytes
// (3 B/px of reads, 4 B/px of writes over a 128-frame 3840x2160 batch):
//   L6S8 strip : 6 x 16-B loads + 8 x 16-B stores per lane (48-block task,
//                128x16 px strip, two 512-B row segments per store) -- today;
//   L6S8 linear: same per-lane volume, writes one contiguous 8 KiB per task;
//   L3S4 strip : 24-block task, 64x16 px strip (four 256-B row segments per
//                store instruction);
//   L3S4 linear: same volume, contiguous 4 KiB per task;
//   L1S1 mix   : one-shot: each thread loads one 16-B chunk and stores
//                4/3 chunks on average (3 of 4 threads one chunk, ... ) --
//                modelled as 3 loads + 4 stores per 4 threads, linear.
// One task per wave, 4 waves per workgroup, tasks in raster order.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, PITCH = W * 4;
constexpr int64_t kFramePx = static_cast<int64_t>(W) * H;

// kL loads, kS stores of 16 B per lane; kStripW = 0 -> linear output
template <int kL, int kS, int kStripW>
__global__ __launch_bounds__(256) void strips(const u4* __restrict__ coefs, uint8_t* __restrict__ out, int64_t tasks)
{
    const int lane = threadIdx.x & 63;
    const int64_t task = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (task >= tasks) return;
    const u4* src = coefs + task * (64 * kL) + lane;
    u4 acc = {0, 0, 0, 0};
#pragma unroll
    for (int k = 0; k < kL; ++k) acc ^= __builtin_nontemporal_load(src + 64 * k);
    if constexpr (kStripW == 0) {
        u4* dst = reinterpret_cast<u4*>(out) + task * (64 * kS) + lane;
#pragma unroll
        for (int k = 0; k < kS; ++k) __builtin_nontemporal_store(acc, dst + 64 * k);
    } else {
        constexpr int kRows = 16;                      // 4:2:0 MCU row height
        constexpr int kLanesPerRow = kStripW * 4 / 16; // 16-B chunks per strip row
        constexpr int kRowsPerStore = 64 / kLanesPerRow;
        static_assert(kS * kRowsPerStore == kRows, "strip must be covered by the stores");
        constexpr int kStrips = W / kStripW;
        const int64_t per_frame = static_cast<int64_t>(kStrips) * (H / kRows);
        const int64_t f = task / per_frame;
        const int64_t t = task - f * per_frame;
        const int sy = static_cast<int>(t / kStrips), sx = static_cast<int>(t % kStrips);
        uint8_t* base = out + f * static_cast<int64_t>(PITCH) * H + static_cast<int64_t>(sy * kRows) * PITCH +
                        sx * kStripW * 4;
        const int x = (lane % kLanesPerRow) * 16, y0 = lane / kLanesPerRow;
#pragma unroll
        for (int it = 0; it < kS; ++it)
            __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(base + (it * kRowsPerStore + y0) * PITCH + x));
    }
}

// one-shot mix: group of 256 threads = 192 load chunks + 256 store chunks
__global__ __launch_bounds__(256) void oneshot_mix(const u4* __restrict__ coefs, uint8_t* __restrict__ out,
                                                   int64_t groups)
{
    const int64_t g = blockIdx.x;
    if (g >= groups) return;
    u4 acc = {0, 0, 0, 0};
    if (threadIdx.x < 192) acc = __builtin_nontemporal_load(coefs + g * 192 + threadIdx.x);
    acc.x += __shfl_xor(acc.x, 1);
    __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(out) + g * 256 + threadIdx.x);
}

static float time_ms(void (*launch)(const u4*, uint8_t*, int64_t, unsigned), const u4* c, uint8_t* o, int64_t n,
                     unsigned grid)
{
    launch(c, o, n, grid);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) launch(c, o, n, grid);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms / 5;
}

template <int kL, int kS, int kStripW>
static void launch_strips(const u4* c, uint8_t* o, int64_t n, unsigned grid)
{
    hipLaunchKernelGGL((strips<kL, kS, kStripW>), dim3(grid), dim3(256), 0, 0, c, o, n);
}
static void launch_mix(const u4* c, uint8_t* o, int64_t n, unsigned grid)
{
    hipLaunchKernelGGL(oneshot_mix, dim3(grid), dim3(256), 0, 0, c, o, n);
}

template <int kL, int kS, int kStripW>
static void run(const u4* coefs, uint8_t* out, int frames, const char* name, size_t in_bytes, size_t out_bytes)
{
    const int64_t px_per_task = kS * 64 * 16 / 4;
    const int64_t tasks = frames * kFramePx / px_per_task;
    if (static_cast<size_t>(tasks) * kL * 1024 > in_bytes || static_cast<size_t>(tasks) * kS * 1024 > out_bytes ||
        (kStripW && (W % kStripW != 0))) {
        printf("%s: extent check failed, not launched\n", name);
        return;
    }
    const unsigned grid = static_cast<unsigned>((tasks + 3) / 4);
    const float ms = time_ms(launch_strips<kL, kS, kStripW>, coefs, out, tasks, grid);
    const double bytes = static_cast<double>(tasks) * (kL + kS) * 1024;
    printf("%-12s %d frames: %7.1f GB/s (r+w), %.3f ms/launch\n", name, frames, bytes / (ms * 1e-3) / 1e9, ms);
}

int main()
{
    const int frames = 128;
    const size_t out_bytes = static_cast<size_t>(frames) * PITCH * H;
    const size_t in_bytes = static_cast<size_t>(frames) * kFramePx * 3 / 2 * 2;
    u4* coefs;
    uint8_t* out;
    (void)hipMalloc(&coefs, in_bytes);
    (void)hipMalloc(&out, out_bytes);
    (void)hipMemset(coefs, 1, in_bytes);
    for (int rep = 0; rep < 2; ++rep) {
        run<6, 8, 128>(coefs, out, frames, "L6S8 strip", in_bytes, out_bytes);
        run<6, 8, 0>(coefs, out, frames, "L6S8 linear", in_bytes, out_bytes);
        run<3, 4, 64>(coefs, out, frames, "L3S4 strip", in_bytes, out_bytes);
        run<3, 4, 0>(coefs, out, frames, "L3S4 linear", in_bytes, out_bytes);
        run<12, 16, 256>(coefs, out, frames, "L12S16 strip", in_bytes, out_bytes);
        const int64_t groups = static_cast<int64_t>(out_bytes / 4096);
        const float ms = time_ms(launch_mix, coefs, out, groups, static_cast<unsigned>(groups));
        printf("%-12s %d frames: %7.1f GB/s (r+w), %.3f ms/launch\n", "one-shot mix", frames,
               static_cast<double>(groups) * 7168 / (ms * 1e-3) / 1e9, ms);
    }
    return 0;
}
