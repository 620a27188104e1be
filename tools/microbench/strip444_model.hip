// Memory-only model of the 4:4:4 pixel kernel's access pattern (tuning tool):
// per wave-task 6 KiB of contiguous coefficient reads (6 x 16 B per lane) and
// a 128x8 px BGRX strip of writes (4 store instructions per lane, each two
// 512-B row segments), over a 128-frame 3840x2160 batch.  T consecutive tasks
// per wave with the next task's loads issued before the current task's stores
// (the kernel's register prefetch); T = 1 is one task per wave.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, PITCH = W * 4;
constexpr int kStrips = W / 128, kTasksPerFrame = kStrips * (H / 8);

template <int T, int kTail, int kLds>
__global__ __launch_bounds__(256) void strips(const u4* __restrict__ coefs, uint8_t* __restrict__ out, int64_t tasks)
{
    // kLds bytes of LDS per workgroup: limits residency like the kernel's 10 KiB per wave
    __shared__ u4 lds[kLds / 16 > 0 ? kLds / 16 : 1];
    const int lane = threadIdx.x & 63;
    if constexpr (kLds > 0) lds[threadIdx.x] = u4{0, 0, 0, 0};
    const int64_t w = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    const int64_t t0 = w * T;
    if (t0 >= tasks) return;
    const int64_t t1 = t0 + T < tasks ? t0 + T : tasks;
    u4 pre[6];
#pragma unroll
    for (int k = 0; k < 6; ++k) pre[k] = __builtin_nontemporal_load(coefs + t0 * 384 + lane + 64 * k);
    for (int64_t t = t0; t < t1; ++t) {
        u4 acc = pre[0] ^ pre[1] ^ pre[2] ^ pre[3] ^ pre[4] ^ pre[5];
        if constexpr (kLds > 0) acc ^= lds[(threadIdx.x + t) & 255];
        if (t + 1 < t1) {
#pragma unroll
            for (int k = 0; k < 6; ++k) pre[k] = __builtin_nontemporal_load(coefs + (t + 1) * 384 + lane + 64 * k);
        }
#pragma unroll 1
        for (int k = 0; k < kTail; ++k) acc.x = acc.x * 3 + acc.y;   // optional VALU between load and store
        const int64_t f = t / kTasksPerFrame, tt = t - f * kTasksPerFrame;
        const int sy = static_cast<int>(tt / kStrips), sx = static_cast<int>(tt % kStrips);
        uint8_t* base = out + f * static_cast<int64_t>(PITCH) * H + static_cast<int64_t>(sy * 8) * PITCH + sx * 512;
        const int x = (lane & 31) * 16, y0 = lane >> 5;
#pragma unroll
        for (int it = 0; it < 4; ++it)
            __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(base + (2 * it + y0) * PITCH + x));
    }
}

template <int T, int kTail, int kLds = 0>
static void run(const u4* coefs, uint8_t* out, int frames)
{
    const int64_t tasks = static_cast<int64_t>(frames) * kTasksPerFrame;
    const int64_t waves = (tasks + T - 1) / T;
    const unsigned grid = static_cast<unsigned>((waves + 3) / 4);
    auto launch = [&] { hipLaunchKernelGGL((strips<T, kTail, kLds>), dim3(grid), dim3(256), 0, 0, coefs, out, tasks); };
    launch();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    printf("4:4:4 pattern T=%2d valu=%3d lds=%5d: %7.1f GB/s (r+w), %.3f ms/launch\n", T, kTail, kLds,
           static_cast<double>(tasks) * 10240 / (ms * 1e-3) / 1e9, ms);
}

int main()
{
    const int frames = 128;
    u4* coefs;
    uint8_t* out;
    const size_t in_bytes = static_cast<size_t>(frames) * kTasksPerFrame * 6144;
    (void)hipMalloc(&coefs, in_bytes + 4096);
    (void)hipMalloc(&out, static_cast<size_t>(frames) * PITCH * H);
    (void)hipMemset(coefs, 1, in_bytes);
    for (int rep = 0; rep < 2; ++rep) {
        run<1, 0>(coefs, out, frames);
        run<2, 0>(coefs, out, frames);
        run<4, 0>(coefs, out, frames);
        run<8, 0>(coefs, out, frames);
        run<16, 0>(coefs, out, frames);
        run<1, 64>(coefs, out, frames);
        run<8, 64>(coefs, out, frames);
        run<8, 0, 40960>(coefs, out, frames);   // 4 groups/CU = 4 waves/SIMD, the kernel's residency
        run<8, 0, 32768>(coefs, out, frames);   // 5 groups/CU
        run<8, 0, 26624>(coefs, out, frames);   // 6 groups/CU
        run<1, 0, 40960>(coefs, out, frames);
        run<2, 0, 32768>(coefs, out, frames);
    }
    return 0;
}
