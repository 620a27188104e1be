// Memory+latency model of a "one-shot" workgroup-cooperative decode (tuning
// tool).  tools/microbench/strip_pattern2.hip measured a one-shot 3:4 mix
// (each 256-thread group loads 3 KiB and stores 4 KiB, one memory
// instruction per thread) at ~6.6 TB/s against ~5.6 TB/s for the wave-task
// patterns of today's kernel.  This model adds what a decode kernel of that
// shape must also do, one knob at a time:
//   strip  : the group's 4 KiB is a 64x16 px strip (16 rows x 256 B) of a
//            3840x2160 BGRX frame instead of a contiguous 4 KiB;
//   lds    : loads go through LDS with a workgroup barrier, and a second
//            barrier before the stores (the row/column/colour phases);
//   valu K : K dependent VALU ops per wave between the barriers (the IDCT and
//            colour work is ~100-150 VALU per wave for a 24-block task);
//   frame  : the group's frame record is read with a scalar load that the
//            coefficient address depends on (frame = group / groups_per_frame).
// Groups of 8 waves (48-block tasks: 6 KiB in, 8 KiB out) are measured too.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, PITCH = W * 4;
constexpr int64_t kFramePx = static_cast<int64_t>(W) * H;

struct FrameRec {   // 64 B like the kernel's FrameDev
    int64_t coef_base;   // in 16-B chunks
    int64_t out_base;    // bytes
    int pad[12];
};

// kWaves: 4 (24-block task, 64x16 strip) or 8 (48-block task, 128x16 strip)
template <int kWaves, bool kStrip, bool kLds, int kValu, bool kFrame>
__global__ __launch_bounds__(kWaves * 64) void model(const u4* __restrict__ coefs, uint8_t* __restrict__ out,
                                                      const FrameRec* __restrict__ frames, int64_t groups)
{
    constexpr int kThreads = kWaves * 64;
    constexpr int kLoads = kThreads * 3 / 4;          // 16-B load chunks per group
    constexpr int kStripW = kWaves * 16;              // px: 4 waves -> 64, 8 -> 128
    constexpr int kGroupsPerFrame = (W / kStripW) * (H / 16);
    __shared__ u4 lds[kLoads];
    const int64_t g = blockIdx.x;
    if (g >= groups) return;
    const int tid = threadIdx.x;
    int64_t cbase = g * kLoads, obase = g * kThreads * 16;
    int64_t t = g;
    if constexpr (kFrame || kStrip) {
        const int64_t f = g / kGroupsPerFrame;
        t = g - f * kGroupsPerFrame;
        if constexpr (kFrame) {
            const FrameRec fr = frames[f];   // uniform: scalar loads
            cbase = fr.coef_base + t * kLoads;
            obase = fr.out_base;
        } else {
            obase = f * static_cast<int64_t>(PITCH) * H;
        }
    }
    u4 acc = {0, 0, 0, 0};
    if (tid < kLoads) acc = __builtin_nontemporal_load(coefs + cbase + tid);
    if constexpr (kLds) {
        if (tid < kLoads) lds[tid] = acc;
        __syncthreads();
        acc = lds[(tid * 7) % kLoads];
    }
#pragma unroll 1
    for (int k = 0; k < kValu; ++k) {
        acc.x = acc.x * 3 + acc.y;
        acc.y ^= acc.x;
    }
    if constexpr (kLds) {
        __syncthreads();
        if (tid < kLoads) lds[tid] = acc;
        __syncthreads();
        acc = lds[tid % kLoads];
    }
    if constexpr (kStrip) {
        constexpr int kStrips = W / kStripW;
        const int sy = static_cast<int>(t / kStrips), sx = static_cast<int>(t % kStrips);
        constexpr int kLanesPerRow = kStripW * 4 / 16;   // 16 (4 waves) or 32 (8 waves)
        const int x = (tid % kLanesPerRow) * 16, y = tid / kLanesPerRow;
        uint8_t* p = out + obase + static_cast<int64_t>(sy * 16 + y) * PITCH + sx * kStripW * 4 + x;
        __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(p));
    } else {
        __builtin_nontemporal_store(acc, reinterpret_cast<u4*>(out + obase) + tid);
    }
}

template <int kWaves, bool kStrip, bool kLds, int kValu, bool kFrame>
static void run(const u4* coefs, uint8_t* out, const FrameRec* frames, int nframes, const char* name)
{
    constexpr int kThreads = kWaves * 64;
    const int64_t groups = nframes * kFramePx * 4 / (kThreads * 16);
    auto launch = [&] {
        hipLaunchKernelGGL((model<kWaves, kStrip, kLds, kValu, kFrame>), dim3(static_cast<unsigned>(groups)),
                           dim3(kThreads), 0, 0, coefs, out, frames, groups);
    };
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
    const double bytes = static_cast<double>(nframes) * kFramePx * 7;
    printf("%-34s %7.1f GB/s (r+w), %.3f ms/launch\n", name, bytes / (ms * 1e-3) / 1e9, ms);
}

int main()
{
    const int frames = 128;
    const size_t out_bytes = static_cast<size_t>(frames) * kFramePx * 4;
    const size_t in_bytes = static_cast<size_t>(frames) * kFramePx * 3;
    u4* coefs;
    uint8_t* out;
    FrameRec* fr;
    (void)hipMalloc(&coefs, in_bytes);
    (void)hipMalloc(&out, out_bytes);
    (void)hipMalloc(&fr, sizeof(FrameRec) * frames);
    (void)hipMemset(coefs, 1, in_bytes);
    FrameRec h[128] = {};
    for (int f = 0; f < frames; ++f) {
        h[f].coef_base = static_cast<int64_t>(f) * kFramePx * 3 / 16;
        h[f].out_base = static_cast<int64_t>(f) * kFramePx * 4;
    }
    (void)hipMemcpy(fr, h, sizeof(h), hipMemcpyHostToDevice);
    for (int rep = 0; rep < 2; ++rep) {
        run<4, false, false, 0, false>(coefs, out, fr, frames, "w4 linear");
        run<4, true, false, 0, false>(coefs, out, fr, frames, "w4 strip");
        run<4, true, true, 0, false>(coefs, out, fr, frames, "w4 strip lds");
        run<4, true, true, 64, false>(coefs, out, fr, frames, "w4 strip lds valu64");
        run<4, true, true, 128, false>(coefs, out, fr, frames, "w4 strip lds valu128");
        run<4, true, true, 256, false>(coefs, out, fr, frames, "w4 strip lds valu256");
        run<4, true, true, 128, true>(coefs, out, fr, frames, "w4 strip lds valu128 frame");
        run<8, false, false, 0, false>(coefs, out, fr, frames, "w8 linear");
        run<8, true, false, 0, false>(coefs, out, fr, frames, "w8 strip");
        run<8, true, true, 128, true>(coefs, out, fr, frames, "w8 strip lds valu128 frame");
    }
    return 0;
}
