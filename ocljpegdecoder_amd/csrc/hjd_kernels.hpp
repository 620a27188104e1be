// hjd_kernels.hpp -- the fused pixel-back-end kernels for gfx950 (CDNA4).
//
// Work decomposition:
//   task  = one "strip" of 48 consecutive coefficient blocks of one frame:
//           8 MCUs (4:2:0, 128x16 px) or 16 MCUs (4:4:4, 128x8 px) of one MCU row.
//   wave  = one task at a time; 4 independent waves per 256-thread workgroup,
//           each with a private 9 KiB LDS slice (no workgroup barriers);
//           persistent grid-stride loop over all tasks of all frames.
//   lane  = (g = lane>>3, r = lane&7): the 1-D IDCT of row r (row pass) and
//           column r (column pass) of block 6g+i for round i = 0..5 -- one
//           lane per 8-point transform, no redundant butterflies.
// Per task: coefficients (6 KiB int16, contiguous) are prefetched into VGPRs
// one task ahead, staged to LDS with ds_write_b128, gathered in natural order
// by zigzag offsets (dequant fused), row pass -> LDS transpose -> column pass
// -> int16 samples back into the block's own LDS slot -> colour stage reads
// rows (ds_read_b64), computes chroma terms once per chroma sample, and writes
// 16-byte BGRX stores (two 512-byte row segments per wave instruction).
#pragma once
#include "hjd_device.hpp"

namespace hjd {

constexpr int kTaskBlocks = 48;      // blocks per task (6 rounds x 8 lane groups)
constexpr int kSlotBytes = 144;      // LDS bytes per block slot (128 + 16 pad: bank spread)
constexpr int kRowBufBlock = 288;    // LDS bytes per block in the transpose buffer (256 + 32)
constexpr int kWaveLds = kTaskBlocks * kSlotBytes + 8 * kRowBufBlock;  // 9216
constexpr int kWavesPerGroup = 4;
constexpr int kGroupThreads = 64 * kWavesPerGroup;

// Device-side frame record built by hjd_plan_create.
struct FrameDev {
    int64_t coef_base;   // first block of the frame (in blocks)
    int64_t out_base;    // byte offset of pixel (0,0)
    int64_t task_begin;  // first global task id of this frame
    int32_t width, height, pitch;
    int32_t sampling;    // 0 = 4:4:4, 1 = 4:2:0
    int32_t mcu_w;       // MCUs per MCU row
    int32_t strips;      // tasks per MCU row
    int32_t qt[3];       // natural-order table index per component
    int32_t vec_ok;      // 1: 16-byte aligned rows -> dwordx4 stores
};
static_assert(sizeof(FrameDev) == 64, "FrameDev layout");

// Natural index n -> zigzag position (inverse of the JPEG zigzag, src/zigzag.h).
__device__ __forceinline__ int zz_of_natural(int n)
{
    // packed 6-bit table, 64 entries
    constexpr unsigned char kInv[64] = {
        0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
        3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
        10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
        21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
    return kInv[n];
}

__device__ __forceinline__ void wave_lds_sync()
{
    // LDS ops of one wave execute in order; this stops the compiler from
    // moving LDS accesses across the point and waits for outstanding ones.
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Binary search of the frame owning global task `task` (wave-uniform).
__device__ __forceinline__ int find_frame(const FrameDev* __restrict__ fr, int nframes, int64_t task)
{
    int lo = 0, hi = nframes - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (fr[mid].task_begin <= task) lo = mid; else hi = mid - 1;
    }
    return lo;
}

// Store 4 horizontally adjacent BGRX pixels (cropping at the frame edge).
__device__ __forceinline__ void store4(uint8_t* __restrict__ row, int x, int width, bool vec_ok,
                                       uint32_t p0, uint32_t p1, uint32_t p2, uint32_t p3)
{
    uint32_t* dst = reinterpret_cast<uint32_t*>(row) + x;
    if (vec_ok && x + 4 <= width) {
        *reinterpret_cast<uint4*>(dst) = make_uint4(p0, p1, p2, p3);
    } else {
        if (x + 0 < width) dst[0] = p0;
        if (x + 1 < width) dst[1] = p1;
        if (x + 2 < width) dst[2] = p2;
        if (x + 3 < width) dst[3] = p3;
    }
}

// Colour stage of one task (samples are int16, row-major, in the block slots).
template <int kSampling>
__device__ __forceinline__ void colour_stage(const char* __restrict__ slots, int lane, uint8_t* __restrict__ out,
                                             const FrameDev& f, int y_base, int x_base)
{
    const int cg = lane & 31;     // 4-pixel column group within the 128-px strip
    const int x0 = cg * 4;
    const int xa = x_base + x0;
    if constexpr (kSampling == 1) {
        const int m = cg >> 2;        // MCU within strip
        const int xm = x0 & 15;       // x within MCU: 0,4,8,12
#pragma unroll
        for (int it = 0; it < 4; ++it) {
            const int p = it * 2 + (lane >> 5);   // row pair 0..7 within the MCU row
            const int y0 = 2 * p;
            const char* yblk = slots + (m * 6 + (y0 >> 3) * 2 + (xm >> 3)) * kSlotBytes + (xm & 7) * 2;
            const int2 ya = *reinterpret_cast<const int2*>(yblk + (y0 & 7) * 16);
            const int2 yb = *reinterpret_cast<const int2*>(yblk + ((y0 + 1) & 7) * 16);
            const int coff = p * 16 + (xm >> 1) * 2;
            const int cu = *reinterpret_cast<const int*>(slots + (m * 6 + 4) * kSlotBytes + coff);
            const int cv = *reinterpret_cast<const int*>(slots + (m * 6 + 5) * kSlotBytes + coff);
            const ChromaTerms c0 = chroma_terms(static_cast<short>(cu), static_cast<short>(cv));
            const ChromaTerms c1 = chroma_terms(cu >> 16, cv >> 16);
            const int ya0 = y_base + y0;
            if (ya0 < f.height) {
                store4(out + static_cast<int64_t>(ya0) * f.pitch, xa, f.width, f.vec_ok,
                       pixel_bgrx(static_cast<short>(ya.x), c0), pixel_bgrx(ya.x >> 16, c0),
                       pixel_bgrx(static_cast<short>(ya.y), c1), pixel_bgrx(ya.y >> 16, c1));
            }
            if (ya0 + 1 < f.height) {
                store4(out + static_cast<int64_t>(ya0 + 1) * f.pitch, xa, f.width, f.vec_ok,
                       pixel_bgrx(static_cast<short>(yb.x), c0), pixel_bgrx(yb.x >> 16, c0),
                       pixel_bgrx(static_cast<short>(yb.y), c1), pixel_bgrx(yb.y >> 16, c1));
            }
        }
    } else {
        const int m = cg >> 1;        // MCU within strip (16 x 8 px)
        const int xm = x0 & 7;        // 0 or 4
#pragma unroll
        for (int it = 0; it < 2; ++it) {
            const int p = it * 2 + (lane >> 5);   // row pair 0..3
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int y = 2 * p + h;
                const char* base = slots + m * 3 * kSlotBytes + y * 16 + xm * 2;
                const int2 sy = *reinterpret_cast<const int2*>(base);
                const int2 su = *reinterpret_cast<const int2*>(base + kSlotBytes);
                const int2 sv = *reinterpret_cast<const int2*>(base + 2 * kSlotBytes);
                const int ya = y_base + y;
                if (ya < f.height) {
                    const uint32_t q0 = pixel_bgrx(static_cast<short>(sy.x),
                                                   chroma_terms(static_cast<short>(su.x), static_cast<short>(sv.x)));
                    const uint32_t q1 = pixel_bgrx(sy.x >> 16, chroma_terms(su.x >> 16, sv.x >> 16));
                    const uint32_t q2 = pixel_bgrx(static_cast<short>(sy.y),
                                                   chroma_terms(static_cast<short>(su.y), static_cast<short>(sv.y)));
                    const uint32_t q3 = pixel_bgrx(sy.y >> 16, chroma_terms(su.y >> 16, sv.y >> 16));
                    store4(out + static_cast<int64_t>(ya) * f.pitch, xa, f.width, f.vec_ok, q0, q1, q2, q3);
                }
            }
        }
    }
}

// Component (0 = Y, 1 = Cb, 2 = Cr) of round i's block for lane group g.
template <int kSampling>
__device__ __forceinline__ constexpr int round_component(int i)
{
    return kSampling == 1 ? (i < 4 ? 0 : i - 3) : (i % 3);
}

// IDCT of the task's 48 blocks (6 rounds).  kFmt 0: int16 zigzag staged in the
// LDS slots; kFmt 1: int32 natural rows read straight from global memory.
// Samples end up as int16 row-major in the block slots.
template <int kSampling, int kFmt>
__device__ __forceinline__ void idct_stage(char* __restrict__ slots, int* __restrict__ rowbuf, int lane,
                                           const int (&zoff)[8], const int (&q)[3][8],
                                           const int* __restrict__ src32, int nblk)
{
    const int g = lane >> 3, r = lane & 7;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int b = 6 * g + i;
        const int comp = round_component<kSampling>(i);
        int v[8];
        if constexpr (kFmt == 0) {
            const char* blk = slots + b * kSlotBytes;
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                const int coef = *reinterpret_cast<const short*>(blk + zoff[c]);
                v[c] = mul24(coef, q[comp][c]);   // dequant (src/decoder.cpp:340)
            }
        } else {
            int4 lo = make_int4(0, 0, 0, 0), hi = lo;
            if (b < nblk) {   // lanes past the strip's last block compute on zeros
                const int4* p = reinterpret_cast<const int4*>(src32 + b * 64 + r * 8);
                lo = p[0];
                hi = p[1];
            }
            v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
            v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        }
        idct8<false>(v);
        {
            int4* dst = reinterpret_cast<int4*>(reinterpret_cast<char*>(rowbuf) + g * kRowBufBlock + r * 32);
            dst[0] = make_int4(v[0], v[1], v[2], v[3]);
            dst[1] = make_int4(v[4], v[5], v[6], v[7]);
        }
        wave_lds_sync();
        {
            const char* col = reinterpret_cast<const char*>(rowbuf) + g * kRowBufBlock + r * 4;
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const int*>(col + k * 32);
        }
        idct8<true>(v);
        {
            char* blk = slots + b * kSlotBytes + r * 2;   // column r
#pragma unroll
            for (int k = 0; k < 8; ++k) *reinterpret_cast<short*>(blk + k * 16) = static_cast<short>(v[k]);
        }
        wave_lds_sync();
    }
}

template <int kSampling, int kFmt>
__global__ __launch_bounds__(kGroupThreads) void decode_kernel(const void* __restrict__ coefs,
                                                              const int* __restrict__ qt_pool,
                                                              const FrameDev* __restrict__ frames, int nframes,
                                                              int64_t total_tasks, uint8_t* __restrict__ out)
{
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerGroup * kWaveLds];
    const int wave = threadIdx.x >> 6;
    const int lane = threadIdx.x & 63;
    char* slots = lds + wave * kWaveLds;
    int* rowbuf = reinterpret_cast<int*>(slots + kTaskBlocks * kSlotBytes);
    const int r = lane & 7;

    int zoff[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) zoff[c] = 2 * zz_of_natural(r * 8 + c);

    const int64_t nwaves = static_cast<int64_t>(gridDim.x) * kWavesPerGroup;
    int64_t task = static_cast<int64_t>(blockIdx.x) * kWavesPerGroup + wave;

    constexpr int kMcuPerTask = kSampling == 1 ? 8 : 16;
    constexpr int kBpm = kSampling == 1 ? 6 : 3;
    constexpr int kMcuPx = kSampling == 1 ? 16 : 8;

    int cur_frame = -1;
    int q[3][8];
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < 8; ++k) q[c][k] = 0;

    // prefetch registers (kFmt 0 only): 6 x 16 B per lane = 6 KiB per wave
    int4 pre[6];
    auto locate = [&](int64_t t, int& fi, int64_t& blk0, int& nblk, int& my, int& mx0) {
        fi = find_frame(frames, nframes, t);
        const FrameDev& f = frames[fi];
        const int64_t local = t - f.task_begin;
        my = static_cast<int>(local / f.strips);
        const int s = static_cast<int>(local - static_cast<int64_t>(my) * f.strips);
        mx0 = s * kMcuPerTask;
        const int nmcu = min(kMcuPerTask, f.mcu_w - mx0);
        nblk = nmcu * kBpm;
        blk0 = f.coef_base + (static_cast<int64_t>(my) * f.mcu_w + mx0) * kBpm;
    };
    auto prefetch = [&](int64_t t) {
        int fi, nblk, my, mx0;
        int64_t blk0;
        locate(t, fi, blk0, nblk, my, mx0);
        const int4* src = reinterpret_cast<const int4*>(static_cast<const short*>(coefs) + blk0 * 64);
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const int j = lane + 64 * k;   // 16-byte chunk index within the task
            pre[k] = (j < nblk * 8) ? src[j] : make_int4(0, 0, 0, 0);
        }
    };

    if constexpr (kFmt == 0) {
        if (task < total_tasks) prefetch(task);
    }

    for (; task < total_tasks; task += nwaves) {
        int fi, nblk, my, mx0;
        int64_t blk0;
        locate(task, fi, blk0, nblk, my, mx0);
        const FrameDev& f = frames[fi];
        if (kFmt == 0 && fi != cur_frame) {   // wave-uniform: (re)load this lane's qtable rows
            cur_frame = fi;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const int4* qp = reinterpret_cast<const int4*>(qt_pool + f.qt[c] * 64 + r * 8);
                const int4 a = qp[0], b = qp[1];
                q[c][0] = a.x; q[c][1] = a.y; q[c][2] = a.z; q[c][3] = a.w;
                q[c][4] = b.x; q[c][5] = b.y; q[c][6] = b.z; q[c][7] = b.w;
            }
        }

        const int* src32 = nullptr;
        if constexpr (kFmt == 0) {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int j = lane + 64 * k;
                *reinterpret_cast<int4*>(slots + (j >> 3) * kSlotBytes + (j & 7) * 16) = pre[k];
            }
            wave_lds_sync();
            const int64_t next = task + nwaves;
            if (next < total_tasks) prefetch(next);
        } else {
            src32 = static_cast<const int*>(coefs) + blk0 * 64;
        }

        idct_stage<kSampling, kFmt>(slots, rowbuf, lane, zoff, q, src32, nblk);

        colour_stage<kSampling>(slots, lane, out + f.out_base, f, my * kMcuPx, mx0 * kMcuPx);
        wave_lds_sync();
    }
}

// IDCT only, out of place (the reference's batch_idct): one wave = 8 blocks.
__global__ __launch_bounds__(kGroupThreads) void idct_blocks_kernel(const int* __restrict__ in,
                                                                   int* __restrict__ out, int64_t nblocks)
{
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerGroup * 8 * kRowBufBlock];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 3, r = lane & 7;
    int* rowbuf = reinterpret_cast<int*>(lds + wave * 8 * kRowBufBlock);
    const int64_t ngroups = (nblocks + 7) / 8;
    for (int64_t grp = static_cast<int64_t>(blockIdx.x) * kWavesPerGroup + wave; grp < ngroups;
         grp += static_cast<int64_t>(gridDim.x) * kWavesPerGroup) {
        const int64_t b = grp * 8 + g;
        const bool valid = b < nblocks;
        int v[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (valid) {
            const int4* p = reinterpret_cast<const int4*>(in + b * 64 + r * 8);
            const int4 lo = p[0], hi = p[1];
            v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
            v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
        }
        idct8<false>(v);
        int4* dst = reinterpret_cast<int4*>(reinterpret_cast<char*>(rowbuf) + g * kRowBufBlock + r * 32);
        dst[0] = make_int4(v[0], v[1], v[2], v[3]);
        dst[1] = make_int4(v[4], v[5], v[6], v[7]);
        wave_lds_sync();
        const char* col = reinterpret_cast<const char*>(rowbuf) + g * kRowBufBlock + r * 4;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const int*>(col + k * 32);
        wave_lds_sync();
        idct8<true>(v);
        if (valid) {
#pragma unroll
            for (int k = 0; k < 8; ++k) out[b * 64 + k * 8 + r] = v[k];
        }
    }
}

// Colour stage alone (test hooks).
template <int kMode>
__global__ void csc_kernel(const int* __restrict__ y, const int* __restrict__ u, const int* __restrict__ v,
                           uint32_t* __restrict__ out, int64_t n)
{
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        out[i] = kMode == 0 ? pixel_bgrx(y[i], chroma_terms(u[i], v[i])) : pixel_bgrx_f64(y[i], u[i], v[i]);
    }
}

template <int kMode>
__global__ void csc_exhaustive_kernel(uint32_t* __restrict__ out)
{
    const int64_t n = int64_t(1) << 27;
    for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n;
         i += static_cast<int64_t>(gridDim.x) * blockDim.x) {
        const int Y = static_cast<int>(i >> 18) - 256;
        const int U = static_cast<int>((i >> 9) & 511) - 256;
        const int V = static_cast<int>(i & 511) - 256;
        out[i] = kMode == 0 ? pixel_bgrx(Y, chroma_terms(U, V)) : pixel_bgrx_f64(Y, U, V);
    }
}

}  // namespace hjd
