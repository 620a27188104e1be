// Model of a workgroup-cooperative pixel kernel (tuning tool).  An 8-wave
// group handles one 48-block 4:2:0 task at a time (6 KiB of coefficients in:
// one 16-B load on 384 of its 512 lanes; a 128x16 px BGRX strip out: one
// 16-B store per lane), with the task's work modelled as two VALU phases of
// K dependent ops per wave separated by LDS exchanges and workgroup barriers
// (row pass -> transpose -> column + colour).  Variants:
//   oneshot : one task per group, grid = all tasks (dispatch-ordered);
//   pipe T  : T consecutive tasks per group, the next task's coefficients
//             loaded into registers before the current task's phases
//             (software pipelining, as today's per-wave kernel does).
// Compare with today's per-wave kernel (~5.65 TB/s at 4:2:0, ~1100 VALU per
// 48-block task = ~140 per wave of an 8-wave group, i.e. K ~ 23 here: 3 ops
// per loop iteration, two phases).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, PITCH = W * 4;
constexpr int64_t kFramePx = static_cast<int64_t>(W) * H;
constexpr int kThreads = 512, kLoads = 384, kStripW = 128;
constexpr int kStrips = W / kStripW, kTasksPerFrame = kStrips * (H / 16);

template <int K>
__device__ __forceinline__ u4 valu(u4 a)
{
#pragma unroll 1
    for (int k = 0; k < K; ++k) {
        a.x = a.x * 3 + a.y;
        a.y ^= a.x;
    }
    return a;
}

__device__ __forceinline__ void store_strip(uint8_t* __restrict__ out, int64_t task, int tid, u4 v)
{
    const int64_t f = task / kTasksPerFrame, t = task - f * kTasksPerFrame;
    const int sy = static_cast<int>(t / kStrips), sx = static_cast<int>(t % kStrips);
    const int x = (tid & 31) * 16, y = tid >> 5;
    uint8_t* p = out + f * kFramePx * 4 + static_cast<int64_t>(sy * 16 + y) * PITCH + sx * kStripW * 4 + x;
    __builtin_nontemporal_store(v, reinterpret_cast<u4*>(p));
}

template <int K, int T>
__global__ __launch_bounds__(kThreads) void coop(const u4* __restrict__ coefs, uint8_t* __restrict__ out,
                                                 int64_t tasks)
{
    __shared__ u4 lin[2][kLoads];
    __shared__ u4 mid[kThreads];
    const int tid = threadIdx.x;
    const int64_t t0 = static_cast<int64_t>(blockIdx.x) * T;
    const int64_t t1 = t0 + T < tasks ? t0 + T : tasks;
    u4 pre = {0, 0, 0, 0};
    if (tid < kLoads) pre = __builtin_nontemporal_load(coefs + t0 * kLoads + tid);
    int buf = 0;
    for (int64_t t = t0; t < t1; ++t) {
        if (tid < kLoads) lin[buf][tid] = pre;
        if (t + 1 < t1 && tid < kLoads) pre = __builtin_nontemporal_load(coefs + (t + 1) * kLoads + tid);
        __syncthreads();
        u4 a = lin[buf][(tid * 7) % kLoads];
        a = valu<K>(a);
        mid[tid ^ 37] = a;
        __syncthreads();
        a = valu<K>(mid[tid]);
        store_strip(out, t, tid, a);
        buf ^= 1;
    }
}

template <int K, int T>
static void run(const u4* coefs, uint8_t* out, int frames, const char* name)
{
    const int64_t tasks = static_cast<int64_t>(frames) * kTasksPerFrame;
    const unsigned grid = static_cast<unsigned>((tasks + T - 1) / T);
    auto launch = [&] { hipLaunchKernelGGL((coop<K, T>), dim3(grid), dim3(kThreads), 0, 0, coefs, out, tasks); };
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
    printf("%-12s K=%3d T=%3d: %7.1f GB/s (r+w), %.3f ms/launch\n", name, K, T,
           static_cast<double>(tasks) * 14336 / (ms * 1e-3) / 1e9, ms);
}

int main()
{
    const int frames = 128;
    u4* coefs;
    uint8_t* out;
    (void)hipMalloc(&coefs, static_cast<size_t>(frames) * kFramePx * 3);
    (void)hipMalloc(&out, static_cast<size_t>(frames) * kFramePx * 4);
    (void)hipMemset(coefs, 1, static_cast<size_t>(frames) * kFramePx * 3);
    for (int rep = 0; rep < 2; ++rep) {
        run<0, 1>(coefs, out, frames, "oneshot");
        run<12, 1>(coefs, out, frames, "oneshot");
        run<24, 1>(coefs, out, frames, "oneshot");
        run<0, 4>(coefs, out, frames, "pipe");
        run<12, 4>(coefs, out, frames, "pipe");
        run<24, 4>(coefs, out, frames, "pipe");
        run<24, 16>(coefs, out, frames, "pipe");
        run<24, 64>(coefs, out, frames, "pipe");
        run<36, 16>(coefs, out, frames, "pipe");
    }
    return 0;
}
