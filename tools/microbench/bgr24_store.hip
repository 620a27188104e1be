// BGR24 store shape (tuning tool): the same bytes written per wave-instruction
// as (a) 64 lanes x 12-B dwordx3 (two 384-B row segments, the kernel today) or
// (b) 48 lanes x 16-B dwordx4 (the same two segments after an LDS restage).
// One wave-task = 8 instructions over 16 rows of a 3840-px frame (pitch
// 11520 B), tasks in raster strip order.  Extents are checked on the host.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u3 __attribute__((ext_vector_type(3), aligned(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
constexpr int W = 3840, H = 2160, PITCH = W * 3, STRIP = 128, ROWS = 16;
constexpr int STRIPS = W / STRIP, BANDS = H / ROWS;
static_assert(W % STRIP == 0 && H % ROWS == 0, "exact tiling");

template <int kShape>
__global__ __launch_bounds__(256) void stores(uint8_t* __restrict__ out, int64_t tasks)
{
    const int lane = threadIdx.x & 63;
    const int64_t task = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6);
    if (task >= tasks) return;
    const int64_t f = task / (STRIPS * BANDS);
    const int t = static_cast<int>(task - f * (STRIPS * BANDS));
    uint8_t* base = out + f * static_cast<int64_t>(PITCH) * H + static_cast<int64_t>(t / STRIPS) * ROWS * PITCH +
                    (t % STRIPS) * STRIP * 3;
    const int half = lane >> 5, l = lane & 31;
#pragma unroll
    for (int it = 0; it < 8; ++it) {
        const int y = 2 * (it >> 1) * 2 + (it & 1) + 2 * half;   // 0..15, two rows per instruction
        if constexpr (kShape == 0) {
            const u3 v = {static_cast<unsigned>(task), 1u, 2u};
            __builtin_nontemporal_store(v, reinterpret_cast<u3*>(base + y * PITCH + l * 12));
        } else {
            if (l < 24) {
                const u4 v = {static_cast<unsigned>(task), 1u, 2u, 3u};
                __builtin_nontemporal_store(v, reinterpret_cast<u4*>(base + y * PITCH + l * 16));
            }
        }
    }
}

template <int kShape>
static void run(uint8_t* out, int frames, size_t bytes, const char* name)
{
    const int64_t tasks = static_cast<int64_t>(frames) * STRIPS * BANDS;
    if (static_cast<size_t>(frames) * PITCH * H > bytes) {
        printf("%s: extent check failed, not launched\n", name);
        return;
    }
    const unsigned grid = static_cast<unsigned>((tasks + 3) / 4);
    hipLaunchKernelGGL((stores<kShape>), dim3(grid), dim3(256), 0, 0, out, tasks);
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int i = 0; i < 5; ++i) hipLaunchKernelGGL((stores<kShape>), dim3(grid), dim3(256), 0, 0, out, tasks);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("%-10s %d frames: %7.1f GB/s written\n", name, frames,
           5.0 * frames * static_cast<double>(W) * H * 3 / (ms * 1e-3) / 1e9);
}

int main()
{
    const int frames = 128;
    const size_t bytes = static_cast<size_t>(frames) * PITCH * H;
    uint8_t* out;
    if (hipMalloc(&out, bytes) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        run<0>(out, frames, bytes, "dwordx3");
        run<1>(out, frames, bytes, "dwordx4x48");
    }
    return 0;
}
