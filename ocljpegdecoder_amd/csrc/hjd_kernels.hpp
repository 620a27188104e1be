// hjd_kernels.hpp -- the fused pixel-back-end kernels for gfx950 (CDNA4).
//
// Work decomposition:
//   task  = one "strip" of 48 consecutive coefficient blocks of one frame:
//           8 MCUs (4:2:0, 128x16 px), 16 MCUs (4:4:4, 128x8 px), 12 MCUs
//           (4:2:2, 192x8 px) or 48 MCUs (gray, 384x8 px) of one MCU row.
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
constexpr int kRowStride = 48;       // transpose buffer: bytes per row (b128 row writes conflict-free)
constexpr int kRowBufBlock = 416;    // transpose buffer: bytes per block (104 dwords = 8 mod 32 banks)
constexpr int kWavesPerGroup = 4;
constexpr int kGroupThreads = 64 * kWavesPerGroup;

// Per-wave LDS layout of the fused kernel: 48 block slots plus a transpose
// buffer (10240 B, 4 waves per SIMD).  A 5-wave layout (transpose through the
// round's own slot, tables in LDS) measured -1.0 % at 4:4:4 and was removed
// (DESIGN.md s3.4).
struct KLayout {
    static constexpr int wave_lds = kTaskBlocks * kSlotBytes + 8 * kRowBufBlock;
    static constexpr int min_waves = 4;
    static_assert(kWavesPerGroup * wave_lds * min_waves <= 160 * 1024, "the groups per CU must fit the 160 KiB LDS");
};

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
    constexpr unsigned char kInv[64] = {
        0,  1,  5,  6,  14, 15, 27, 28, 2,  4,  7,  13, 16, 26, 29, 42,
        3,  8,  12, 17, 25, 30, 41, 43, 9,  11, 18, 24, 31, 40, 44, 53,
        10, 19, 23, 32, 39, 45, 52, 54, 20, 22, 33, 38, 46, 51, 55, 60,
        21, 34, 37, 47, 50, 56, 59, 61, 35, 36, 48, 49, 57, 58, 62, 63};
    return kInv[n];
}

// Cross-lane hand-off through the wave's private LDS slice.  The DS
// instructions of one wave execute in issue order, so a ds_read issued after a
// ds_write sees its data without any s_waitcnt; this only stops the compiler
// from reordering LDS accesses across the point (it still inserts the counted
// lgkmcnt waits where read results are consumed).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wave-uniform view of the frame that owns a task range (lives in SGPRs).
struct FrameCursor {
    int idx;
    int64_t begin, end;      // [begin, end) global task ids of this frame
    int64_t coef_base, out_base;
    int width, height, pitch, mcu_w, strips, vec_ok;
    int qt0, qt1, qt2;
};

__device__ __forceinline__ void cursor_load(FrameCursor& c, const FrameDev* __restrict__ fr, int nframes,
                                            int64_t total, int i)
{
    const FrameDev& f = fr[i];
    c.idx = i;
    c.begin = f.task_begin;
    c.end = (i + 1 < nframes) ? fr[i + 1].task_begin : total;
    c.coef_base = f.coef_base;
    c.out_base = f.out_base;
    c.width = f.width;
    c.height = f.height;
    c.pitch = f.pitch;
    c.mcu_w = f.mcu_w;
    c.strips = f.strips;
    c.vec_ok = f.vec_ok;
    c.qt0 = f.qt[0];
    c.qt1 = f.qt[1];
    c.qt2 = f.qt[2];
}

// The frame owning `task` (once per wave, scalar).  Batches of equal frames
// (the common case) have task_begin[i] = i * K: the guess task / K is checked
// against the record it loads anyway, so a wave start costs two dependent
// scalar loads instead of a ~log2(nframes)-deep binary search, which is the
// fallback for mixed plans.
__device__ __forceinline__ void cursor_seek(FrameCursor& c, const FrameDev* __restrict__ fr, int nframes,
                                            int64_t total, int64_t task)
{
    if (nframes > 1) {
        const int64_t k = fr[1].task_begin;   // tasks of frame 0
        if (k > 0 && task < (int64_t(1) << 32)) {
            const int64_t g = static_cast<uint32_t>(task) / static_cast<uint32_t>(k);   // 32-bit udiv
            if (g < nframes) {
                cursor_load(c, fr, nframes, total, static_cast<int>(g));
                if (c.begin <= task && task < c.end) return;
            }
        }
    }
    int lo = 0, hi = nframes - 1;
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (fr[mid].task_begin <= task) lo = mid; else hi = mid - 1;
    }
    cursor_load(c, fr, nframes, total, lo);
}

// Compile-time geometry of the kernel's sampling index (hjd_internal::
// sampling_geom): 0 4:4:4, 1 4:2:0, 2 4:2:2 (extension), 3 gray (extension),
// 4 4:1:1 = Y H4V1 (extension), 5 4:4:0 = Y H1V2 (extension).
template <int kSampling>
struct KGeom {
    static constexpr int kBpm = kSampling == 0 ? 3 : kSampling == 1 || kSampling == 4 ? 6
                              : kSampling == 2 || kSampling == 5 ? 4 : 1;
    static constexpr int kMcuW = kSampling == 4 ? 32 : kSampling == 1 || kSampling == 2 ? 16 : 8;   // MCU pixels
    static constexpr int kMcuH = kSampling == 1 || kSampling == 5 ? 16 : 8;
    static constexpr int kMcus = kTaskBlocks / kBpm;                          // MCUs per task
    static constexpr int kStripW = kMcus * kMcuW;                            // strip pixels
    static_assert(kMcus * kBpm == kTaskBlocks, "a task is 48 whole MCUs' blocks");
};

// Where a task's strip sits in its frame.
struct TaskGeom {
    int64_t blk0;   // first coefficient block (global)
    int nblk;       // blocks in the strip (48, fewer on the right edge)
    int y_base;     // first pixel row
    int x_base;     // first pixel column
};

template <int kSampling>
__device__ __forceinline__ TaskGeom task_geom(const FrameCursor& c, int64_t task)
{
    using G = KGeom<kSampling>;
    const int local = static_cast<int>(task - c.begin);
    const int my = local / c.strips;
    const int mx0 = (local - my * c.strips) * G::kMcus;
    TaskGeom g;
    g.nblk = min(G::kMcus, c.mcu_w - mx0) * G::kBpm;
    g.blk0 = c.coef_base + (static_cast<int64_t>(my) * c.mcu_w + mx0) * G::kBpm;
    g.y_base = my * G::kMcuH;
    g.x_base = mx0 * G::kMcuW;
    return g;
}

// Kernel variants (hjd_plan_set_variant): bit 0 = plain instead of
// non-temporal 16-byte output stores.
constexpr int kVarPlainStores = 1;
// bit 1: workgroup-interleaved task order (wave w of a group takes tasks
// 4q + w of the group's contiguous quad range) instead of one contiguous range
// per wave: the group's 4 waves then write adjacent 512-byte row segments.
constexpr int kVarWgInterleave = 2;
// Ablation bits: the stage-skipping measurement variants behind
// hjd_debug_plan_launch_stages (bench.py stage_times); their outputs are
// deliberately wrong.
constexpr int kAblNoStore = 4, kAblNoColour = 8, kAblNoIdct = 16;
// kAblNoCsc: the colour stage keeps its LDS reads and stores but skips the
// chroma terms and pixel math (stores raw sample words).
constexpr int kAblNoCsc = 64;
// Output format bit (include/hjd.h HJD_OUT_BGR24): 3-byte B,G,R pixels
// instead of 4-byte BGRX words.
constexpr int kOutBgr24 = 32;
// Gather pairs as ds_read_u16 | ds_read_u16_d16_hi (load_round_pk_d16): only
// valid where d16 loads zero the other half (sramecc+), chosen at launch.
constexpr int kVarD16 = 128;
// kAblGatherBroadcast: every lane gathers row 0 of its block (lanes of a
// block read the same words: no LDS bank conflicts), the same instructions as
// the product -- what the zigzag gather's conflicts cost.
constexpr int kAblGatherBroadcast = 256;
template <int kVariant>
constexpr int kOutBytes = (kVariant & kOutBgr24) != 0 ? 3 : 4;

// 4 horizontally adjacent pixels (BGRX words p0..p3) at row + loff.  `row` is wave-uniform
// (SGPRs) and loff a 32-bit per-lane byte offset, so the store uses the
// scalar-base addressing form (no 64-bit address arithmetic per row).  kFull:
// the whole strip row lies inside the frame and rows are 16-byte aligned ->
// one global_store_dwordx4 (nt by default: the output is streamed and never
// re-read by the kernel); otherwise per-pixel guarded dword stores (x = the
// first pixel's column).  BGR24: the four pixels are repacked into 12 bytes
// (three v_perm) and stored as one dwordx3 (rows 4-byte aligned), or as
// guarded bytes on edge strips.
template <bool kFull, int kVariant = 0>
__device__ __forceinline__ void store4(uint8_t* __restrict__ row, uint32_t loff, int x, int width, uint32_t p0,
                                       uint32_t p1, uint32_t p2, uint32_t p3)
{
    // Pin the row base in SGPRs as a global (addrspace 1) pointer and the lane
    // offset as a 32-bit VGPR in this block: otherwise LLVM hoists
    // base + zext(loff) into a 64-bit VGPR value (whose zero high half the
    // per-block instruction selector cannot see) and adds each row's offset
    // to it with VALU ops instead of using the scalar-base store form.
    typedef __attribute__((address_space(1))) uint8_t gbyte;
    typedef __attribute__((address_space(1))) uint32_t gword;
    gbyte* grow = (gbyte*)row;
    asm("" : "+s"(grow));
    asm("" : "+v"(loff));
    gword* dst = (gword*)(grow + loff);
    if constexpr ((kVariant & kAblNoStore) != 0) {
        asm volatile("" ::"v"(p0), "v"(p1), "v"(p2), "v"(p3));
        return;
    }
    if constexpr ((kVariant & kOutBgr24) != 0) {
        if constexpr (kFull) {
            typedef unsigned int u32x3 __attribute__((ext_vector_type(3), aligned(4)));
            typedef __attribute__((address_space(1))) u32x3 gvec3;
            const u32x3 v = {perm(p1, p0, 0x04020100u),    // b0 g0 r0 b1
                             perm(p2, p1, 0x05040201u),    // g1 r1 b2 g2
                             perm(p3, p2, 0x06050402u)};   // r2 b3 g3 r3
            __builtin_nontemporal_store(v, (gvec3*)dst);
        } else {
            gbyte* d8 = (gbyte*)dst;
            const uint32_t px[4] = {p0, p1, p2, p3};
#pragma unroll
            for (int k = 0; k < 4; ++k)
                if (x + k < width) {
                    d8[3 * k] = static_cast<uint8_t>(px[k]);
                    d8[3 * k + 1] = static_cast<uint8_t>(px[k] >> 8);
                    d8[3 * k + 2] = static_cast<uint8_t>(px[k] >> 16);
                }
        }
    } else if constexpr (kFull) {
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 v = {p0, p1, p2, p3};
        typedef __attribute__((address_space(1))) u32x4 gvec;
        if constexpr (kVariant & kVarPlainStores)
            *(gvec*)dst = v;
        else
            __builtin_nontemporal_store(v, (gvec*)dst);
    } else {
        if (x + 0 < width) dst[0] = p0;
        if (x + 1 < width) dst[1] = p1;
        if (x + 2 < width) dst[2] = p2;
        if (x + 3 < width) dst[3] = p3;
    }
}

// Colour stage of one task (samples are int16, row-major, in the block slots;
// luma level-shifted by +128 by its IDCT, chroma raw).
// Each lane owns 4 px x 2 rows.  4:2:0: one chroma row serves both pixel rows
// (nearest 2x2 replication, src/decoder.cpp:474-483), chroma terms are computed
// once per chroma sample; 4 iterations cover the 128x16 strip and every wave
// store instruction writes two 512-byte row segments.  4:4:4: the same lane
// shape over the 128x8 strip, chroma per pixel (src/decoder.cpp:457-471).
// Pixel math is packed: two pixels per int16x2 VGPR (pixels2).  Row addresses:
// row 4*it + h of the strip is wave-uniform; lanes 32-63 sit two rows lower,
// which is folded into their 32-bit lane offset.
template <bool kCheck, int kVariant, bool kFull>
__device__ __forceinline__ void emit_row4(uint8_t* __restrict__ row, uint32_t loff, int xa, int width, uint32_t y01,
                                          uint32_t y23, const ChromaPair& p01, const ChromaPair& p23,
                                          const ChromaTerms* c0, const ChromaTerms* c1, const ChromaTerms* c2,
                                          const ChromaTerms* c3)
{
    uint32_t q0, q1, q2, q3;
    pixels2<kCheck>(y01, p01, c0, c1, q0, q1);
    pixels2<kCheck>(y23, p23, c2, c3, q2, q3);
    store4<kFull, kVariant>(row, loff, xa, width, q0, q1, q2, q3);
}

// kStride / u0: this wave converts colour units u0, u0 + kStride, ... of the
// strip (the latency kernel spreads a task's units over its waves; the
// persistent kernel converts all of them: kStride 1, u0 0).
template <int kSampling, bool kFull, int kVariant, int kStride = 1>
__device__ __forceinline__ void colour_stage(const char* __restrict__ slots, int lane, uint8_t* __restrict__ out,
                                             int pitch, int width, int height, int y_base, int x_base, int u0 = 0)
{
    const int cg = lane & 31;     // 4-pixel column group within the 128-px strip
    const int x0 = cg * 4;
    const int xa = x_base + x0;
    constexpr int kPx = kOutBytes<kVariant>;   // output bytes per pixel
    const int ylane = 2 * (lane >> 5);   // this half-wave's row offset
    const uint32_t loff = static_cast<uint32_t>(x0 * kPx) + static_cast<uint32_t>(ylane) * static_cast<uint32_t>(pitch);
    uint8_t* const strip = out + static_cast<int64_t>(y_base) * pitch + static_cast<int64_t>(x_base) * kPx;
    if constexpr (kSampling == 1) {
        const int m = cg >> 2;        // MCU within strip
        const int xm = x0 & 15;       // x within MCU: 0,4,8,12
#pragma unroll
        for (int k = 0; k < (4 + kStride - 1) / kStride; ++k) {
            const int it = u0 + k * kStride;
            if (kStride > 1 && it >= 4) break;
            const int p = it * 2 + (lane >> 5);   // row pair 0..7 within the MCU row
            const int y0 = 2 * p;
            const char* yblk = slots + (m * 6 + (y0 >> 3) * 2 + (xm >> 3)) * kSlotBytes + (xm & 7) * 2;
            const int2 ya = *reinterpret_cast<const int2*>(yblk + (y0 & 7) * 16);
            const int2 yb = *reinterpret_cast<const int2*>(yblk + ((y0 + 1) & 7) * 16);
            const int coff = p * 16 + (xm >> 1) * 2;
            const uint32_t cu = *reinterpret_cast<const uint32_t*>(slots + (m * 6 + 4) * kSlotBytes + coff);
            const uint32_t cv = *reinterpret_cast<const uint32_t*>(slots + (m * 6 + 5) * kSlotBytes + coff);
            uint8_t* row0 = strip + static_cast<int64_t>(4 * it) * pitch;   // wave-uniform
            if constexpr ((kVariant & kAblNoCsc) != 0) {
                store4<kFull, kVariant>(row0, loff, xa, width, ya.x, ya.y, cu, cv);
                store4<kFull, kVariant>(row0 + pitch, loff, xa, width, yb.x, yb.y, cu, cv);
                continue;
            }
            const ChromaTerms c0 = chroma_terms<0>(cu, cv);
            const ChromaTerms c1 = chroma_terms<1>(cu, cv);
            const ChromaPair p0 = pair_of(c0, c0), p1 = pair_of(c1, c1);
            const int ya0 = y_base + y0;
            if (__builtin_amdgcn_ballot_w64((p0.flagged | p1.flagged) != 0)) {   // wave-uniform, rare
                if (kFull || ya0 < height)
                    emit_row4<true, kVariant, kFull>(row0, loff, xa, width, ya.x, ya.y, p0, p1, &c0, &c0, &c1, &c1);
                if (kFull || ya0 + 1 < height)
                    emit_row4<true, kVariant, kFull>(row0 + pitch, loff, xa, width, yb.x, yb.y, p0, p1, &c0, &c0, &c1,
                                                     &c1);
            } else {
                if (kFull || ya0 < height)
                    emit_row4<false, kVariant, kFull>(row0, loff, xa, width, ya.x, ya.y, p0, p1, &c0, &c0, &c1, &c1);
                if (kFull || ya0 + 1 < height)
                    emit_row4<false, kVariant, kFull>(row0 + pitch, loff, xa, width, yb.x, yb.y, p0, p1, &c0, &c0,
                                                      &c1, &c1);
            }
        }
    } else if constexpr (kSampling == 0) {
        const int m = cg >> 1;        // MCU within strip (16 x 8 px)
        const int xm = x0 & 7;        // 0 or 4
#pragma unroll
        for (int k = 0; k < (4 + kStride - 1) / kStride; ++k) {
            const int u = u0 + k * kStride;       // unit = (row pair it, row h)
            if (kStride > 1 && u >= 4) break;
            const int it = u >> 1, h = u & 1;
            const int p = it * 2 + (lane >> 5);   // row pair 0..3
            {
                const int y = 2 * p + h;
                const char* base = slots + m * 3 * kSlotBytes + y * 16 + xm * 2;
                const int2 sy = *reinterpret_cast<const int2*>(base);
                const uint2 su = *reinterpret_cast<const uint2*>(base + kSlotBytes);
                const uint2 sv = *reinterpret_cast<const uint2*>(base + 2 * kSlotBytes);
                if constexpr ((kVariant & kAblNoCsc) != 0) {
                    store4<kFull, kVariant>(strip + static_cast<int64_t>(4 * it + h) * pitch, loff, xa, width, sy.x,
                                            sy.y, su.x ^ sv.x, su.y ^ sv.y);
                    continue;
                }
                const ChromaTerms c0 = chroma_terms<0>(su.x, sv.x);
                const ChromaTerms c1 = chroma_terms<1>(su.x, sv.x);
                const ChromaTerms c2 = chroma_terms<0>(su.y, sv.y);
                const ChromaTerms c3 = chroma_terms<1>(su.y, sv.y);
                const ChromaPair p01 = pair_of(c0, c1), p23 = pair_of(c2, c3);
                const int ya = y_base + y;
                uint8_t* row = strip + static_cast<int64_t>(4 * it + h) * pitch;   // wave-uniform
                if (kFull || ya < height) {
                    if (__builtin_amdgcn_ballot_w64((p01.flagged | p23.flagged) != 0))
                        emit_row4<true, kVariant, kFull>(row, loff, xa, width, sy.x, sy.y, p01, p23, &c0, &c1, &c2,
                                                         &c3);
                    else
                        emit_row4<false, kVariant, kFull>(row, loff, xa, width, sy.x, sy.y, p01, p23, &c0, &c1, &c2,
                                                          &c3);
                }
            }
        }
    } else if constexpr (kSampling == 2) {
        // 4:2:2 (extension): 192x8 strip of 12 MCUs (Y0 Y1 Cb Cr, 16x8 px);
        // units of 4 px x 1 row, 48 per row, 6 per lane; each chroma sample
        // serves 2 horizontally adjacent pixels (nearest replication, as the
        // reference's 4:2:0 path does in both directions, src/decoder.cpp:474-483).
        (void)loff;
#pragma unroll 2
        for (int k = 0; k < (6 + kStride - 1) / kStride; ++k) {
            const int it = u0 + k * kStride;
            if (kStride > 1 && it >= 6) break;
            const int u = it * 64 + lane;
            const int y = u / 48;
            const int cu4 = u - y * 48;       // unit within the row
            const int m = cu4 >> 2;
            const int xm = (cu4 & 3) * 4;     // x within MCU: 0,4,8,12
            const int2 sy = *reinterpret_cast<const int2*>(slots + (4 * m + (xm >> 3)) * kSlotBytes + y * 16 +
                                                           (xm & 7) * 2);
            const int coff = y * 16 + xm;     // chroma samples xm/2, xm/2+1
            const uint32_t cu = *reinterpret_cast<const uint32_t*>(slots + (4 * m + 2) * kSlotBytes + coff);
            const uint32_t cv = *reinterpret_cast<const uint32_t*>(slots + (4 * m + 3) * kSlotBytes + coff);
            const ChromaTerms c0 = chroma_terms<0>(cu, cv);
            const ChromaTerms c1 = chroma_terms<1>(cu, cv);
            const ChromaPair p0 = pair_of(c0, c0), p1 = pair_of(c1, c1);
            const uint32_t lo = static_cast<uint32_t>(y) * static_cast<uint32_t>(pitch) +
                                static_cast<uint32_t>(cu4 * 4 * kPx);
            const int xu = x_base + cu4 * 4;
            const bool flagged = __builtin_amdgcn_ballot_w64((p0.flagged | p1.flagged) != 0) != 0;
            if (kFull || y_base + y < height) {
                if (flagged)
                    emit_row4<true, kVariant, kFull>(strip, lo, xu, width, sy.x, sy.y, p0, p1, &c0, &c0, &c1, &c1);
                else
                    emit_row4<false, kVariant, kFull>(strip, lo, xu, width, sy.x, sy.y, p0, p1, &c0, &c0, &c1, &c1);
            }
        }
    } else if constexpr (kSampling == 4) {
        // 4:1:1 (extension, Y H4V1): 256x8 strip of 8 MCUs (Y0-Y3 Cb Cr,
        // 32x8 px); units of 4 px x 1 row, 64 per row (one per lane), 8 rows;
        // each chroma sample serves 4 horizontally adjacent pixels (nearest
        // replication).
        (void)loff;
#pragma unroll 2
        for (int k = 0; k < (8 + kStride - 1) / kStride; ++k) {
            const int y = u0 + k * kStride;   // row of the strip
            if (kStride > 1 && y >= 8) break;
            const int m = lane >> 3;
            const int xm = (lane & 7) * 4;    // x within MCU: 0..28
            const int2 sy = *reinterpret_cast<const int2*>(slots + (6 * m + (xm >> 3)) * kSlotBytes + y * 16 +
                                                           (xm & 7) * 2);
            const int coff = y * 16 + (xm >> 2) * 2;
            const uint32_t cu = *reinterpret_cast<const unsigned short*>(slots + (6 * m + 4) * kSlotBytes + coff);
            const uint32_t cv = *reinterpret_cast<const unsigned short*>(slots + (6 * m + 5) * kSlotBytes + coff);
            const ChromaTerms c0 = chroma_terms<0>(cu, cv);
            const ChromaPair p0 = pair_of(c0, c0);
            const uint32_t lo = static_cast<uint32_t>(y) * static_cast<uint32_t>(pitch) +
                                static_cast<uint32_t>(lane * 4 * kPx);
            const int xu = x_base + lane * 4;
            if (kFull || y_base + y < height) {
                if (__builtin_amdgcn_ballot_w64(p0.flagged != 0))
                    emit_row4<true, kVariant, kFull>(strip, lo, xu, width, sy.x, sy.y, p0, p0, &c0, &c0, &c0, &c0);
                else
                    emit_row4<false, kVariant, kFull>(strip, lo, xu, width, sy.x, sy.y, p0, p0, &c0, &c0, &c0, &c0);
            }
        }
    } else if constexpr (kSampling == 5) {
        // 4:4:0 (extension, Y H1V2): 96x16 strip of 12 MCUs (Y0 above Y1, Cb,
        // Cr; 8x16 px); units of 4 px x 2 rows (pixel rows 2p, 2p+1 share
        // chroma row p: nearest vertical replication), 24 per row pair, 3 per
        // lane.  The chroma terms are computed once per chroma sample, as at
        // 4:2:0 (round 2 computed them for each pixel row: 6 units per lane).
        (void)loff;
#pragma unroll 1
        for (int k = 0; k < (3 + kStride - 1) / kStride; ++k) {
            const int it = u0 + k * kStride;
            if (kStride > 1 && it >= 3) break;
            const int u = it * 64 + lane;
            const int p = u / 24;              // chroma row = pixel rows 2p, 2p+1
            const int cu4 = u - p * 24;        // unit within the row pair
            const int m = cu4 >> 1;
            const int xm = (cu4 & 1) * 4;      // x within MCU: 0 or 4
            const int y0 = 2 * p;
            const char* yblk = slots + (4 * m + (y0 >> 3)) * kSlotBytes + (y0 & 7) * 16 + xm * 2;
            const int2 sya = *reinterpret_cast<const int2*>(yblk);
            const int2 syb = *reinterpret_cast<const int2*>(yblk + 16);   // row y0 + 1 (same block: y0 even)
            const int coff = p * 16 + xm * 2;
            const uint2 su = *reinterpret_cast<const uint2*>(slots + (4 * m + 2) * kSlotBytes + coff);
            const uint2 sv = *reinterpret_cast<const uint2*>(slots + (4 * m + 3) * kSlotBytes + coff);
            const ChromaTerms c0 = chroma_terms<0>(su.x, sv.x);
            const ChromaTerms c1 = chroma_terms<1>(su.x, sv.x);
            const ChromaTerms c2 = chroma_terms<0>(su.y, sv.y);
            const ChromaTerms c3 = chroma_terms<1>(su.y, sv.y);
            const ChromaPair p01 = pair_of(c0, c1), p23 = pair_of(c2, c3);
            const uint32_t lo = static_cast<uint32_t>(y0) * static_cast<uint32_t>(pitch) +
                                static_cast<uint32_t>(cu4 * 4 * kPx);
            const int xu = x_base + cu4 * 4;
            const int ya = y_base + y0;
            if (__builtin_amdgcn_ballot_w64((p01.flagged | p23.flagged) != 0)) {   // wave-uniform, rare
                if (kFull || ya < height)
                    emit_row4<true, kVariant, kFull>(strip, lo, xu, width, sya.x, sya.y, p01, p23, &c0, &c1, &c2, &c3);
                if (kFull || ya + 1 < height)
                    emit_row4<true, kVariant, kFull>(strip, lo + static_cast<uint32_t>(pitch), xu, width, syb.x,
                                                     syb.y, p01, p23, &c0, &c1, &c2, &c3);
            } else {
                if (kFull || ya < height)
                    emit_row4<false, kVariant, kFull>(strip, lo, xu, width, sya.x, sya.y, p01, p23, &c0, &c1, &c2,
                                                      &c3);
                if (kFull || ya + 1 < height)
                    emit_row4<false, kVariant, kFull>(strip, lo + static_cast<uint32_t>(pitch), xu, width, syb.x,
                                                      syb.y, p01, p23, &c0, &c1, &c2, &c3);
            }
        }
    } else {
        // gray (extension): 384x8 strip of 48 one-block MCUs; units of 4 px x
        // 1 row, 96 per row, 12 per lane; R = G = B = clamp(Y + 128), the
        // reference's conversion with U = V = 0 (src/decoder.cpp:367-370).
        (void)loff;
#pragma unroll
        for (int k = 0; k < (12 + kStride - 1) / kStride; ++k) {
            const int it = u0 + k * kStride;
            if (kStride > 1 && it >= 12) break;
            const int u = it * 64 + lane;
            const int y = u / 96;
            const int cu4 = u - y * 96;
            const int2 sy = *reinterpret_cast<const int2*>(slots + (cu4 >> 1) * kSlotBytes + y * 16 + (cu4 & 1) * 8);
            const uint32_t g01 = sat_pk_u8(static_cast<uint32_t>(sy.x));   // bytes g0 g1
            const uint32_t g23 = sat_pk_u8(static_cast<uint32_t>(sy.y));
            const uint32_t lo = static_cast<uint32_t>(y) * static_cast<uint32_t>(pitch) +
                                static_cast<uint32_t>(cu4 * 4 * kPx);
            if (kFull || y_base + y < height)
                store4<kFull, kVariant>(strip, lo, x_base + cu4 * 4, width, perm(g01, g01, 0x0c000000u),
                                        perm(g01, g01, 0x0c010101u), perm(g23, g23, 0x0c000000u),
                                        perm(g23, g23, 0x0c010101u));
        }
    }
}

// Task-local block (= LDS slot) transformed by lane group g in round i.  The
// mapping keeps each round's component uniform across the wave (dequant table
// and luma level shift): 4:4:4 / 4:2:0 / gray blocks are MCU-interleaved with
// a period dividing 6, so 6g + i works; 4:2:2 MCUs are (Y0, Y1, Cb, Cr), so
// rounds 0-2 take the 24 luma blocks, rounds 3-5 the 12 Cb then 12 Cr blocks.
// The IDCT rounds depend only on the MCU's block order: 4:1:1 MCUs (Y0-Y3,
// Cb, Cr) are transformed like 4:2:0 ones, 4:4:0 MCUs (Y0, Y1, Cb, Cr) like
// 4:2:2 ones.
constexpr int round_class(int s) { return s == 4 ? 1 : s == 5 ? 2 : s; }

template <int kSampling0, int kSampling = round_class(kSampling0)>
__device__ __forceinline__ int round_block(int i, int g)
{
    if constexpr (kSampling == 2) {
        if (i < 3) {
            const int idx = i * 8 + g;          // luma block idx of the strip
            return 4 * (idx >> 1) + (idx & 1);
        }
        const int idx = (i - 3) * 8 + g;        // 0-11 Cb, 12-23 Cr
        return idx < 12 ? 4 * idx + 2 : 4 * (idx - 12) + 3;
    } else {
        return 6 * g + i;
    }
}

// Component (0 = Y, 1 = Cb, 2 = Cr) of round i's blocks; -1 where it differs
// between lane groups (4:2:2 round 4: groups 0-3 Cb, 4-7 Cr).
template <int kSampling0, int kSampling = round_class(kSampling0)>
__device__ __forceinline__ constexpr int round_component(int i)
{
    return kSampling == 1 ? (i < 4 ? 0 : i - 3)
         : kSampling == 0 ? (i % 3)
         : kSampling == 3 ? 0
         : (i < 3 ? 0 : i == 3 ? 1 : i == 5 ? 2 : -1);
}

// Component (0 = Y, 1 = Cb, 2 = Cr) of task-local block b (MCU-major).
template <int kSampling0, int kSampling = round_class(kSampling0)>
__device__ __forceinline__ int block_component(int b)
{
    if constexpr (kSampling == 0) {
        return b % 3;
    } else if constexpr (kSampling == 1) {
        const int j = b % 6;
        return j < 4 ? 0 : j - 3;
    } else if constexpr (kSampling == 2) {
        const int j = b & 3;
        return j < 2 ? 0 : j - 1;
    } else {
        return 0;
    }
}

// Round i transforms luma blocks (runtime form of round_component(i) == 0).
template <int kSampling0, int kSampling = round_class(kSampling0)>
__device__ __forceinline__ bool round_is_luma(int i)
{
    return kSampling == 1 ? i < 4 : kSampling == 0 ? i % 3 == 0 : kSampling == 2 ? i < 3 : true;
}

// One round's row-pass inputs, kFmt 0: int16 zigzag coefficients staged in
// the LDS slots, gathered as the row pass's operand pairs and dequantised two
// at a time (v_pk_mul_lo_u16: the low 16 bits of the product, which is the
// reference's int on the legal domain, where dequantised coefficients fit
// int16 -- idct8_row_pk).  q[c][k]: this lane's row of component c's table as
// the pairs (q0,q4), (q1,q7), (q3,q5), (q2,q6) (load_qrow_pk).
template <int kSampling>
__device__ __forceinline__ RowPk load_round_pk(const char* __restrict__ slots, int lane, int i, const int (&zoff)[8],
                                               const uint32_t (&q)[3][4])
{
    const int g = lane >> 3;
    const int b = round_block<kSampling>(i, g);
    const int comp = round_component<kSampling>(i);
    const char* blk = slots + b * kSlotBytes;
    auto pair = [&](int ca, int cb, int k) {
        const s16x2 c = {*reinterpret_cast<const short*>(blk + zoff[ca]),
                         *reinterpret_cast<const short*>(blk + zoff[cb])};
        // a mixed round (4:2:2 round 4) selects the table per lane
        const uint32_t qq = comp >= 0 ? q[comp < 0 ? 0 : comp][k] : (g < 4 ? q[1][k] : q[2][k]);
        return c * __builtin_bit_cast(s16x2, qq);   // dequant (src/decoder.cpp:340)
    };
    RowPk p;
    p.p04 = pair(0, 4, 0);
    p.p17 = pair(1, 7, 1);
    p.p35 = pair(3, 5, 2);
    p.p26 = pair(2, 6, 3);
    return p;
}

// kVarD16 kernels (the runtime launches them on sramecc+ devices only, where
// d16 LDS loads zero the other half): shapes whose round blocks are 6g + i
// with a wave-uniform component (4:4:4, 4:2:0, 4:1:1, grayscale), staged
// int16 (kFmt 0).  Instantiated for 4:4:4 (hjd_runtime.hip).
template <int kSampling, int kFmt, int kVariant>
constexpr bool kD16Gather = (kVariant & kVarD16) != 0 && kFmt == 0 &&
                            (round_class(kSampling) == 0 || round_class(kSampling) == 1 || round_class(kSampling) == 3);

// load_round_pk for kD16Gather shapes, round kI: each pair's second
// coefficient is loaded straight into the high half of its word with
// ds_read_u16_d16_hi, which on MI355X (sramecc+) zeroes the low half
// (profiles/r03_d16_probe.txt), so the pair is (first | second): one v_or_b32
// (a full-rate op on gfx950) instead of a v_perm_b32.  LLVM does not emit the
// d16 LDS loads for this target, so they are inline asm: all four are issued
// before the four compiler-visible ds_read_u16 of the same round, and DS
// operations of a wave complete in order, so the compiler's own wait for
// each low-half load also covers the high-half load issued before it.
template <int kSampling, int kI>
__device__ __forceinline__ RowPk load_round_pk_d16(const char* __restrict__ slots, uint32_t slots_lds, int lane,
                                                   const int (&zoff)[8], const uint32_t (&q)[3][4])
{
    constexpr int comp = round_component<kSampling>(kI);
    static_assert(comp >= 0, "wave-uniform component");
    constexpr int kOff = kI * kSlotBytes;
    const int blk_off = 6 * (lane >> 3) * kSlotBytes;   // round_block = 6g + kI
    constexpr int kHi[4] = {4, 7, 5, 6}, kLo[4] = {0, 1, 3, 2};
    uint32_t w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const uint32_t a = slots_lds + static_cast<uint32_t>(blk_off + zoff[kHi[k]]);
        asm volatile("ds_read_u16_d16_hi %0, %1 offset:%2" : "=v"(w[k]) : "v"(a), "i"(kOff) : "memory");
    }
    const char* blk = slots + blk_off + kOff;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] |= *reinterpret_cast<const unsigned short*>(blk + zoff[kLo[k]]);
    RowPk p;   // dequant (src/decoder.cpp:340)
    p.p04 = __builtin_bit_cast(s16x2, w[0]) * __builtin_bit_cast(s16x2, q[comp][0]);
    p.p17 = __builtin_bit_cast(s16x2, w[1]) * __builtin_bit_cast(s16x2, q[comp][1]);
    p.p35 = __builtin_bit_cast(s16x2, w[2]) * __builtin_bit_cast(s16x2, q[comp][2]);
    p.p26 = __builtin_bit_cast(s16x2, w[3]) * __builtin_bit_cast(s16x2, q[comp][3]);
    return p;
}

template <int kSampling>
__device__ __forceinline__ RowPk load_round_pk_d16_at(int i, const char* __restrict__ slots, uint32_t slots_lds,
                                                      int lane, const int (&zoff)[8], const uint32_t (&q)[3][4])
{
    switch (i) {   // i is a constant in the unrolled round loop
    case 0: return load_round_pk_d16<kSampling, 0>(slots, slots_lds, lane, zoff, q);
    case 1: return load_round_pk_d16<kSampling, 1>(slots, slots_lds, lane, zoff, q);
    case 2: return load_round_pk_d16<kSampling, 2>(slots, slots_lds, lane, zoff, q);
    case 3: return load_round_pk_d16<kSampling, 3>(slots, slots_lds, lane, zoff, q);
    case 4: return load_round_pk_d16<kSampling, 4>(slots, slots_lds, lane, zoff, q);
    default: return load_round_pk_d16<kSampling, 5>(slots, slots_lds, lane, zoff, q);
    }
}

// One round's row-pass inputs, kFmt 1: int32 natural rows (already
// dequantised: the idct.h format) read straight from global memory.
template <int kSampling>
__device__ __forceinline__ void load_round_i32(int lane, int i, const int* __restrict__ src32, int nblk, int (&v)[8])
{
    const int g = lane >> 3, r = lane & 7;
    const int b = round_block<kSampling>(i, g);
    int4 lo = make_int4(0, 0, 0, 0), hi = lo;
    if (b < nblk) {   // lanes past the strip's last block compute on zeros
        const int4* p = reinterpret_cast<const int4*>(src32 + b * 64 + r * 8);
        lo = p[0];
        hi = p[1];
    }
    v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
    v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
}

// Row r of the natural-order table qt_pool[t*64 ..] as the load_round_pk pairs.
__device__ __forceinline__ void load_qrow_pk(const int* __restrict__ qt_pool, int t, int r, uint32_t (&q)[4])
{
    const int4* qp = reinterpret_cast<const int4*>(qt_pool + t * 64 + r * 8);
    const int4 a = qp[0], b = qp[1];   // DQT entries are <= 65535
    q[0] = (a.x & 0xffff) | (b.x << 16);   // q0, q4
    q[1] = (a.y & 0xffff) | (b.w << 16);   // q1, q7
    q[2] = (a.w & 0xffff) | (b.y << 16);   // q3, q5
    q[3] = (a.z & 0xffff) | (b.z << 16);   // q2, q6
}

// IDCT of the task's 48 blocks (6 rounds).  kFmt 0: int16 zigzag staged in the
// LDS slots; kFmt 1: int32 natural rows read straight from global memory.
// Samples end up as int16 row-major in the block slots (luma as Y + 128).  The next round's
// coefficient gathers are issued before this round's column math, so their
// LDS latency overlaps it.
template <int kSampling, int kFmt, int kVariant = 0>
__device__ __forceinline__ void idct_stage(char* __restrict__ slots, char* __restrict__ rowbuf, int lane,
                                           const int (&zoff)[8], const uint32_t (&q)[3][4],
                                           const int* __restrict__ src32, int nblk,
                                           uint32_t slots_lds = 0)
{
    const int g = lane >> 3, r = lane & 7;
    RowPk pk;
    int v[8];
    if constexpr (kD16Gather<kSampling, kFmt, kVariant>)
        pk = load_round_pk_d16_at<kSampling>(0, slots, slots_lds, lane, zoff, q);
    else if constexpr (kFmt == 0)
        pk = load_round_pk<kSampling>(slots, lane, 0, zoff, q);
    else
        load_round_i32<kSampling>(lane, 0, src32, nblk, v);
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const int b = round_block<kSampling>(i, g);
        if constexpr (kFmt == 0)
            idct8_row_pk(pk, v);
        else
            idct8<false>(v);
        int c8[8];
        {
            int4* dst = reinterpret_cast<int4*>(rowbuf + g * kRowBufBlock + r * kRowStride);
            dst[0] = make_int4(v[0], v[1], v[2], v[3]);
            dst[1] = make_int4(v[4], v[5], v[6], v[7]);
            wave_lds_sync();
            const char* col = rowbuf + g * kRowBufBlock + r * 4;
#pragma unroll
            for (int k = 0; k < 8; ++k) c8[k] = *reinterpret_cast<const int*>(col + k * kRowStride);
        }
        if (i + 1 < 6) {
            if constexpr (kD16Gather<kSampling, kFmt, kVariant>)
                pk = load_round_pk_d16_at<kSampling>(i + 1, slots, slots_lds, lane, zoff, q);
            else if constexpr (kFmt == 0)
                pk = load_round_pk<kSampling>(slots, lane, i + 1, zoff, q);
            else
                load_round_i32<kSampling>(lane, i + 1, src32, nblk, v);
        }
        if (round_component<kSampling>(i) == 0)
            idct8_col_hi<kLumaLevel>(c8);   // luma leaves the IDCT level-shifted (Ys = Y + 128)
        else
            idct8_col_hi(c8);
        {
            char* blk = slots + b * kSlotBytes + r * 2;   // column r; the samples are the words' high halves
#pragma unroll
            for (int k = 0; k < 8; ++k)
                *reinterpret_cast<short*>(blk + k * 16) = static_cast<short>(static_cast<uint32_t>(c8[k]) >> 16);
        }
        wave_lds_sync();
    }
}

// Logical position of workgroup `bid` in the task order.  The hardware deals
// consecutive workgroups to the 8 XCDs in turn, so in launch order adjacent
// strips land in 8 different L2s.  Instead each XCD's groups cover one
// contiguous eighth of the grid: XCD x = bid % 8 takes positions
// x*q + min(x, rem) + bid/8 (+1.8 % at 4:2:0, +2.9 % at 4:4:4 same-box,
// profiles/r02_xcd_order_ab.json; runs of 4..1024 groups per XCD and several
// concurrent regions per XCD measured no better).
__device__ __forceinline__ uint32_t group_order(uint32_t bid, uint32_t ngroups)
{
    const uint32_t x = bid & 7, k = bid >> 3, q = ngroups >> 3, rem = ngroups & 7;
    return x * q + min(x, rem) + k;
}

// The fused kernel.  Persistent grid; wave w owns the contiguous task range
// [w*T/W, (w+1)*T/W) so its frame changes rarely and the frame record stays in
// SGPRs; the next task's coefficients are prefetched into VGPRs while the
// current one is transformed.
template <int kSampling, int kFmt, int kVariant>
__global__ __launch_bounds__(kGroupThreads, KLayout::min_waves) void decode_kernel(const void* __restrict__ coefs,
                                                              const int* __restrict__ qt_pool,
                                                              const FrameDev* __restrict__ frames, int nframes,
                                                              int64_t total_tasks, uint8_t* __restrict__ out,
                                                              int64_t chunk, int64_t rem)
{
    using L = KLayout;
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerGroup * L::wave_lds];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    char* slots = lds + wave * L::wave_lds;
    // LDS byte address of this wave's slots (inline-asm DS loads, kVarD16)
    const uint32_t slots_lds = static_cast<uint32_t>(reinterpret_cast<size_t>(lds)) + wave * L::wave_lds;
    char* rowbuf = slots + kTaskBlocks * kSlotBytes;   // transpose buffer
    const int r = lane & 7;

    // this wave's task sequence: t_begin, t_begin + t_step, ... (< t_end)
    // chunk / rem: the split of the task list over the grid, computed on the
    // host (launch_decode) so no wave spends a 64-bit division on it:
    // default order, total_tasks = chunk * (grid * 4 waves) + rem;
    // wg-interleave, ceil(total_tasks / 4) quads = chunk * grid + rem.
    int64_t t_begin, t_end, t_step;
    if constexpr ((kVariant & kVarWgInterleave) != 0) {
        const int64_t qb = static_cast<int64_t>(blockIdx.x) * chunk + min<int64_t>(blockIdx.x, rem);
        const int64_t qe = qb + chunk + (blockIdx.x < rem ? 1 : 0);
        t_begin = qb * kWavesPerGroup + wave;
        t_end = min<int64_t>(qe * kWavesPerGroup, total_tasks);
        t_step = kWavesPerGroup;
    } else {
        const int64_t gw = static_cast<int64_t>(group_order(blockIdx.x, gridDim.x)) * kWavesPerGroup + wave;
        t_begin = gw * chunk + min(gw, rem);
        t_end = t_begin + chunk + (gw < rem ? 1 : 0);
        t_step = 1;
    }
    if (t_begin >= t_end) return;

    int zoff[8];
#pragma unroll
    for (int c = 0; c < 8; ++c)
        zoff[c] = (kVariant & kAblGatherBroadcast) != 0 ? 2 * zz_of_natural(c) : 2 * zz_of_natural(r * 8 + c);

    uint32_t q[3][4];   // this lane's row of each component's qtable, 16-bit pairs
    int q_tables[3] = {-1, -1, -1};
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < 4; ++k) q[c][k] = 0;

    FrameCursor pc;   // frame of the task being prefetched
    cursor_seek(pc, frames, nframes, total_tasks, t_begin);

    int4 pre[6];      // prefetch registers (kFmt 0): 6 x 16 B per lane = 6 KiB per wave
    auto prefetch = [&](const TaskGeom& g) {
        const int4* src = reinterpret_cast<const int4*>(static_cast<const short*>(coefs) + g.blk0 * 64);
        if (g.nblk == kTaskBlocks) {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                // non-temporal: read once (+2.5 % 4:2:0, +1.2 % 4:4:4 same-box, profiles/r02_ntload_ab.json)
                typedef int i32x4 __attribute__((ext_vector_type(4)));
                const i32x4 t = __builtin_nontemporal_load(reinterpret_cast<const i32x4*>(src) + lane + 64 * k);
                pre[k] = make_int4(t.x, t.y, t.z, t.w);
            }
        } else {
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int j = lane + 64 * k;   // 16-byte chunk index within the task
                pre[k] = (j < g.nblk * 8) ? src[j] : make_int4(0, 0, 0, 0);
            }
        }
    };
    if constexpr (kFmt == 0) {
        prefetch(task_geom<kSampling>(pc, t_begin));
        // the first task's table rows load beside its coefficients, so a wave
        // start waits for one memory round trip, not two
        q_tables[0] = pc.qt0; q_tables[1] = pc.qt1; q_tables[2] = pc.qt2;
#pragma unroll
        for (int c = 0; c < 3; ++c) load_qrow_pk(qt_pool, q_tables[c], r, q[c]);
        __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0): see the edge-strip drain below
    }

    for (int64_t task = t_begin, next_task; task >= 0; task = next_task) {
        next_task = task + t_step < t_end ? task + t_step : -1;   // -1: this is the wave's last task
        const FrameCursor cc = pc;
        const TaskGeom tg = task_geom<kSampling>(cc, task);
        if constexpr (kFmt == 0) {
            if (cc.qt0 != q_tables[0] || cc.qt1 != q_tables[1] || cc.qt2 != q_tables[2]) {
                q_tables[0] = cc.qt0; q_tables[1] = cc.qt1; q_tables[2] = cc.qt2;
#pragma unroll
                for (int c = 0; c < 3; ++c) load_qrow_pk(qt_pool, q_tables[c], r, q[c]);
            }
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                const int j = lane + 64 * k;
                *reinterpret_cast<int4*>(slots + (j >> 3) * kSlotBytes + (j & 7) * 16) = pre[k];
            }
            wave_lds_sync();
            if (next_task >= 0) {   // the next task's loads fly during this task
                while (next_task >= pc.end) cursor_load(pc, frames, nframes, total_tasks, pc.idx + 1);
                prefetch(task_geom<kSampling>(pc, next_task));
            }
        } else {
            if (next_task >= 0)
                while (next_task >= pc.end) cursor_load(pc, frames, nframes, total_tasks, pc.idx + 1);
        }

        constexpr int kRows = KGeom<kSampling>::kMcuH;
        constexpr int kStripW = KGeom<kSampling>::kStripW;
        uint8_t* fout = out + cc.out_base;
        const bool full = cc.vec_ok && tg.x_base + kStripW <= cc.width && tg.y_base + kRows <= cc.height;
        if constexpr ((kVariant & kAblNoIdct) == 0)
            idct_stage<kSampling, kFmt, kVariant>(slots, rowbuf, lane, zoff, q,
                                                  static_cast<const int*>(coefs) + tg.blk0 * 64, tg.nblk, slots_lds);

        if constexpr ((kVariant & kAblNoColour) != 0) {
            (void)fout;
        } else if (full)
            colour_stage<kSampling, true, kVariant>(slots, lane, fout, cc.pitch, cc.width, cc.height, tg.y_base, tg.x_base);
        else {
            colour_stage<kSampling, false, kVariant>(slots, lane, fout, cc.pitch, cc.width, cc.height, tg.y_base, tg.x_base);
            // Edge strips issue a data-dependent number of stores; drain them
            // here so the loop head's wait for the prefetched coefficients can
            // be a fixed vmcnt (the full path's stores may stay in flight).
            __builtin_amdgcn_s_waitcnt(0x0f70);   // vmcnt(0)
        }
        wave_lds_sync();
    }
}

// Latency variant for small launches (one FHD frame: ~1000 tasks, about one
// wave per SIMD for the persistent kernel, which then runs each task's six
// IDCT rounds and four colour units back to back).  One 384-thread workgroup
// per task: wave w stages and transforms round w's 8 blocks (its own transpose
// buffer), one workgroup barrier, then the waves share the strip's colour
// units.  Same device functions, same results; the critical path of a task
// is one round + one colour unit instead of six + four.
constexpr int kLatWaves = 6;
constexpr int kLatThreads = 64 * kLatWaves;
constexpr int kLatLds = kTaskBlocks * kSlotBytes + kLatWaves * 8 * kRowBufBlock;

template <int kSampling, int kFmt, int kVariant>
__global__ __launch_bounds__(kLatThreads) void decode_kernel_lat(const void* __restrict__ coefs,
                                                                const int* __restrict__ qt_pool,
                                                                const FrameDev* __restrict__ frames, int nframes,
                                                                int64_t total_tasks, uint8_t* __restrict__ out)
{
    __shared__ __attribute__((aligned(16))) char lds[kLatLds];
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // = this wave's IDCT round
    const int lane = threadIdx.x & 63;
    const int g = lane >> 3, r = lane & 7;
    char* slots = lds;
    char* rowbuf = lds + kTaskBlocks * kSlotBytes + wave * 8 * kRowBufBlock;
    const int64_t task = blockIdx.x;
    if (task >= total_tasks) return;
    FrameCursor cc;
    cursor_seek(cc, frames, nframes, total_tasks, task);
    const TaskGeom tg = task_geom<kSampling>(cc, task);

    const int b = round_block<kSampling>(wave, g);
    int v[8];
    if constexpr (kFmt == 0) {
        // this lane's row of its block's qtable (the block's component may
        // differ between lane groups in 4:2:2 round 4)
        const int comp = block_component<kSampling>(b);
        const int qt = comp == 0 ? cc.qt0 : (comp == 1 ? cc.qt1 : cc.qt2);
        const int4* qp = reinterpret_cast<const int4*>(qt_pool + qt * 64 + r * 8);
        const int4 qa = qp[0], qb = qp[1];
        const int qrow[8] = {qa.x, qa.y, qa.z, qa.w, qb.x, qb.y, qb.z, qb.w};
        // stage this round's 8 blocks: lane (g, r) moves 16-B chunk r of block b
        int4 v4 = make_int4(0, 0, 0, 0);
        if (b < tg.nblk)
            v4 = reinterpret_cast<const int4*>(static_cast<const short*>(coefs) + (tg.blk0 + b) * 64)[r];
        *reinterpret_cast<int4*>(slots + b * kSlotBytes + r * 16) = v4;
        wave_lds_sync();
        const char* blk = slots + b * kSlotBytes;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            const int coef = *reinterpret_cast<const short*>(blk + 2 * zz_of_natural(r * 8 + c));
            v[c] = mul24(coef, qrow[c]);   // dequant (src/decoder.cpp:340)
        }
    } else {
        int4 lo = make_int4(0, 0, 0, 0), hi = lo;
        if (b < tg.nblk) {
            const int4* p = reinterpret_cast<const int4*>(static_cast<const int*>(coefs) + (tg.blk0 + b) * 64 + r * 8);
            lo = p[0];
            hi = p[1];
        }
        v[0] = lo.x; v[1] = lo.y; v[2] = lo.z; v[3] = lo.w;
        v[4] = hi.x; v[5] = hi.y; v[6] = hi.z; v[7] = hi.w;
    }
    idct8<false>(v);
    {
        int4* dst = reinterpret_cast<int4*>(rowbuf + g * kRowBufBlock + r * kRowStride);
        dst[0] = make_int4(v[0], v[1], v[2], v[3]);
        dst[1] = make_int4(v[4], v[5], v[6], v[7]);
    }
    wave_lds_sync();
    int c8[8];
    {
        const char* col = rowbuf + g * kRowBufBlock + r * 4;
#pragma unroll
        for (int k = 0; k < 8; ++k) c8[k] = *reinterpret_cast<const int*>(col + k * kRowStride);
    }
    if (round_is_luma<kSampling>(wave))
        idct8_col_hi<kLumaLevel>(c8);
    else
        idct8_col_hi(c8);
    {
        char* blk = slots + b * kSlotBytes + r * 2;   // column r; the samples are the words' high halves
#pragma unroll
        for (int k = 0; k < 8; ++k)
            *reinterpret_cast<short*>(blk + k * 16) = static_cast<short>(static_cast<uint32_t>(c8[k]) >> 16);
    }
    __syncthreads();   // all 48 blocks' samples are in the slots

    constexpr int kRows = KGeom<kSampling>::kMcuH;
    constexpr int kStripW = KGeom<kSampling>::kStripW;
    uint8_t* fout = out + cc.out_base;
    if (cc.vec_ok && tg.x_base + kStripW <= cc.width && tg.y_base + kRows <= cc.height)
        colour_stage<kSampling, true, kVariant, kLatWaves>(slots, lane, fout, cc.pitch, cc.width, cc.height,
                                                            tg.y_base, tg.x_base, wave);
    else
        colour_stage<kSampling, false, kVariant, kLatWaves>(slots, lane, fout, cc.pitch, cc.width, cc.height,
                                                             tg.y_base, tg.x_base, wave);
}

// IDCT only, out of place (the reference's batch_idct): one wave = 8 blocks.
__global__ __launch_bounds__(kGroupThreads) void idct_blocks_kernel(const int* __restrict__ in,
                                                                   int* __restrict__ out, int64_t nblocks)
{
    __shared__ __attribute__((aligned(16))) char lds[kWavesPerGroup * 8 * kRowBufBlock];
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 3, r = lane & 7;
    char* rowbuf = lds + wave * 8 * kRowBufBlock;
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
        int4* dst = reinterpret_cast<int4*>(rowbuf + g * kRowBufBlock + r * kRowStride);
        dst[0] = make_int4(v[0], v[1], v[2], v[3]);
        dst[1] = make_int4(v[4], v[5], v[6], v[7]);
        wave_lds_sync();
        const char* col = rowbuf + g * kRowBufBlock + r * 4;
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = *reinterpret_cast<const int*>(col + k * kRowStride);
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
        out[i] = kMode == 0 ? pixel_bgrx(y[i], u[i], v[i]) : pixel_bgrx_f64(y[i], u[i], v[i]);
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
        out[i] = kMode == 0 ? pixel_bgrx(Y, U, V) : pixel_bgrx_f64(Y, U, V);
    }
}

}  // namespace hjd
