// hjd_device.hpp -- device-side arithmetic of the pixel back-end (gfx950).
//
// Everything here is bit-exact to the reference CPU path on the reference's
// legal input domain (the domain on which src/cpuIDCT8x8.cpp is defined: no
// signed overflow and column outputs inside its iclp[-512..511] table).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace hjd {

// round(2048*sqrt(2)*cos(k*pi/16)): src/cpuIDCT8x8.cpp:6-11
constexpr int kC1 = 2841, kC2 = 2676, kC3 = 2408, kC5 = 1609, kC6 = 1108, kC7 = 565;

// 24-bit signed multiply (v_mul_i32_i24 / v_mad_i32_i24, full rate).  Exact
// (low 32 bits of the product) when both operands fit in 24 signed bits.  On
// the legal domain every operand that goes through it does: by Parseval the
// block's coefficient energy is bounded by its output energy (|out| <= 512 per
// sample => ||coef||_2 <= ~4.1e3), so stage-1/2 operands of the row pass are
// < 2^14 and of the column pass (row outputs, gain 8*sqrt(8)) < 2^18.
// The host build (the idct.h CPU entry points share this code) multiplies in
// plain 32-bit int, which is the same value on that domain.
__host__ __device__ __forceinline__ int mul24(int a, int b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __mul24(a, b);
#else
    return a * b;
#endif
}

// The stage-3 products 181*(a4 +- a5) can exceed 24 bits on the legal domain,
// so they use a full 32-bit multiply (low 32 bits = the reference's int math).
__host__ __device__ __forceinline__ int mul181(int x) { return x * 181; }

// min/max pairs lower to one v_med3_i32
template <int kLevel = 0>
__host__ __device__ __forceinline__ int clamp_sample(int v)
{
    return v < -256 + kLevel ? -256 + kLevel : (v > 255 + kLevel ? 255 + kLevel : v);
}
__device__ __forceinline__ int clamp_u8(int v) { return min(max(v, 0), 255); }

// One 8-point pass on natural-order values v[0..7] (in place).
// kCol = false: row pass, src/cpuIDCT8x8.cpp:36-80 (x<<11, +128 on DC, >>8 out).
// kCol = true:  column pass, src/cpuIDCT8x8.cpp:82-127 (x<<8, +8192 on DC,
//               (+4)>>3 on stage-1/2 products, >>14 out, clamp [-256,255] --
//               the CPU clamp, not the OpenCL kernel's [-256,256] at
//               src/idct8x8.cl:116).
// The reference's DC-only short-cuts (:40-45, :86-92) give exactly the values
// of the full butterfly, so the kernel always runs the full butterfly.
// kLevel (column pass only): added to every output before the clamp, folded
// into the DC rounding constant ((r + kLevel*2^14) >> 14 == (r >> 14) + kLevel),
// so the luma level shift of the colour stage costs nothing.
template <bool kCol, int kLevel = 0>
__host__ __device__ __forceinline__ void idct8(int (&v)[8])
{
    constexpr int kIn = kCol ? 8 : 11;
    constexpr int kRnd = kCol ? 4 : 0;
    constexpr int kSh = kCol ? 3 : 0;

    static_assert(kCol || kLevel == 0, "level shift is a column-pass option");
    int e0 = (v[0] << kIn) + (kCol ? 8192 + (kLevel << 14) : 128);
    int e1 = v[4] << kIn;

    // odd part
    int t = mul24(kC7, v[1] + v[7]) + kRnd;
    int o4 = (t + mul24(kC1 - kC7, v[1])) >> kSh;
    int o5 = (t - mul24(kC1 + kC7, v[7])) >> kSh;
    t = mul24(kC3, v[5] + v[3]) + kRnd;
    int o6 = (t - mul24(kC3 - kC5, v[5])) >> kSh;
    int o7 = (t - mul24(kC3 + kC5, v[3])) >> kSh;

    // even part
    int e8 = e0 + e1;
    e0 -= e1;
    t = mul24(kC6, v[2] + v[6]) + kRnd;
    int e2 = (t - mul24(kC2 + kC6, v[6])) >> kSh;
    int e3 = (t + mul24(kC2 - kC6, v[2])) >> kSh;

    int a1 = o4 + o6, a4 = o4 - o6;
    int a6 = o5 + o7, a5 = o5 - o7;

    int f7 = e8 + e3, f8 = e8 - e3;
    int f3 = e0 + e2, f0 = e0 - e2;
    int g2 = (mul181(a4 + a5) + 128) >> 8;
    int g4 = (mul181(a4 - a5) + 128) >> 8;

    int r0 = f7 + a1, r1 = f3 + g2, r2 = f0 + g4, r3 = f8 + a6;
    int r4 = f8 - a6, r5 = f0 - g4, r6 = f3 - g2, r7 = f7 - a1;
    if constexpr (kCol) {
        v[0] = clamp_sample<kLevel>(r0 >> 14); v[1] = clamp_sample<kLevel>(r1 >> 14);
        v[2] = clamp_sample<kLevel>(r2 >> 14); v[3] = clamp_sample<kLevel>(r3 >> 14);
        v[4] = clamp_sample<kLevel>(r4 >> 14); v[5] = clamp_sample<kLevel>(r5 >> 14);
        v[6] = clamp_sample<kLevel>(r6 >> 14); v[7] = clamp_sample<kLevel>(r7 >> 14);
    } else {
        v[0] = r0 >> 8; v[1] = r1 >> 8; v[2] = r2 >> 8; v[3] = r3 >> 8;
        v[4] = r4 >> 8; v[5] = r5 >> 8; v[6] = r6 >> 8; v[7] = r7 >> 8;
    }
}

// The column pass of idct8<true, kLevel> with each result in the HIGH int16
// of its word (the low half is junk): the kernel stores it with
// ds_write_b16_d16_hi, so no output needs its own shift.  Every value from the
// even part's DC on is carried at 4x scale (r' = 4r, exact in int32: |r| <
// 2^23 on the legal domain, and the sums are mod 2^32 anyway), so hi16(r') =
// floor(r' / 2^16) = r >> 14, and the clamp is a med3 against bounds scaled
// the same way.  The stage-1/2 products keep the reference's (+4) >> 3 at
// unit scale and are scaled after it (x4 in the final add chains); the
// stage-3 terms 4 * floor((181 s + 128) / 256) = ((181 s + 128) >> 6) & ~3.
// Outside the legal domain the reference itself is undefined (iclp is read
// out of bounds once (r >> 14) leaves [-512, 511], and its int math can
// overflow), so no output is specified there.  This form's own limit: the 4x
// sums wrap once |r| > 2^29 (an unclamped sample beyond about +-32768, far
// outside [-512, 511]), where idct8<true> wrapped only past 2^31; such a
// sample may then clamp to the opposite bound.  Likewise the int16 path
// dequantises with 16-bit products (v_pk_mul_lo_u16) and the row pass takes
// 24-bit operands.  The kernel is bit-exact wherever the reference is defined
// (tests/test_idct_forms.py, the clamp-edge vectors of test_gpu_parity.py).
template <int kLevel = 0>
__host__ __device__ __forceinline__ void idct8_col_hi(int (&v)[8])
{
    int e0 = v[0] * 1024 + (8192 + (kLevel << 14)) * 4;
    const int e1 = v[4] * 1024;
    int t = mul24(kC7, v[1] + v[7]) + 4;
    const int o4 = (t + mul24(kC1 - kC7, v[1])) >> 3;
    const int o5 = (t - mul24(kC1 + kC7, v[7])) >> 3;
    t = mul24(kC3, v[5] + v[3]) + 4;
    const int o6 = (t - mul24(kC3 - kC5, v[5])) >> 3;
    const int o7 = (t - mul24(kC3 + kC5, v[3])) >> 3;
    const int e8 = e0 + e1;
    e0 -= e1;
    t = mul24(kC6, v[2] + v[6]) + 4;
    const int e2 = ((t - mul24(kC2 + kC6, v[6])) >> 3) * 4;
    const int e3 = ((t + mul24(kC2 - kC6, v[2])) >> 3) * 4;
    const int a1 = (o4 + o6) * 4, a4 = o4 - o6;
    const int a6 = (o5 + o7) * 4, a5 = o5 - o7;
    const int f7 = e8 + e3, f8 = e8 - e3;
    const int f3 = e0 + e2, f0 = e0 - e2;
    const int g2 = ((mul181(a4 + a5) + 128) >> 6) & ~3;
    const int g4 = ((mul181(a4 - a5) + 128) >> 6) & ~3;
    constexpr int lo = (-256 + kLevel) * 65536, hi = (255 + kLevel) * 65536 + 65535;
    auto clampw = [](int x) { return x < lo ? lo : (x > hi ? hi : x); };
    v[0] = clampw(f7 + a1); v[1] = clampw(f3 + g2); v[2] = clampw(f0 + g4); v[3] = clampw(f8 + a6);
    v[4] = clampw(f8 - a6); v[5] = clampw(f0 - g4); v[6] = clampw(f3 - g2); v[7] = clampw(f7 - a1);
}

// ---- row pass on packed int16 pairs (the pixel kernel's hot form) -----------
typedef short s16x2 __attribute__((ext_vector_type(2)));

// v_dot2_i32_i16: a.x*b.x + a.y*b.y + c (no clamp; 32-bit wrap like C int
// math).  b is an SGPR constant pair (const_pair).  Written as asm: the
// compiler otherwise selects the accumulate-in-place v_dot2c form and seeds
// each accumulator with a v_mov.
template <int kC>
__host__ __device__ __forceinline__ int sdot2(s16x2 a, s16x2 b)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int r;
    if constexpr (kC == 0) {
        asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(r) : "v"(a), "s"(b));
    } else {
        asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(kC));
    }
    return r;
#else
    return static_cast<int>(a.x) * b.x + static_cast<int>(a.y) * b.y + kC;
#endif
}

// a.x*b.x + a.y*b.y + c with c in a VGPR (an accumulation chain of dot2s).
__host__ __device__ __forceinline__ int sdot2acc(s16x2 a, s16x2 b, int c)
{
#if defined(__HIP_DEVICE_COMPILE__)
    int r;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(r) : "v"(a), "s"(b), "v"(c));
    return r;
#else
    return static_cast<int>(a.x) * b.x + static_cast<int>(a.y) * b.y + c;
#endif
}

// Dequantised row coefficients as int16 pairs (v0,v4), (v1,v7), (v3,v5), (v2,v6):
// the operand pairs of the row pass's rotations.
struct RowPk {
    s16x2 p04, p17, p35, p26;
};

// The row pass of src/cpuIDCT8x8.cpp:36-80 (idctrow) on packed pairs.  Every
// stage-1/2 value of the reference's row pass is an exact sum of two products
// (it has no intermediate shifts), e.g. x4 = W7*(x4+x5) + (W1-W7)*x4 =
// W1*b1 + W7*b7, so each is one v_dot2_i32_i16 of a coefficient pair with a
// constant pair -- the same integers as idct8<false>.  On the legal domain the
// dequantised coefficients are int16 (Parseval: |coef| <= ||coef||_2 <= ~4.1e3,
// see mul24) and no sum overflows int32.
// A constant int16 pair held in an SGPR: the dot2 products then issue as one
// VOP3P v_dot2_i32_i16 (SGPR constant, inline 0 accumulator) instead of the
// literal-operand v_dot2c form, which needs a v_mov to seed its accumulator.
__host__ __device__ __forceinline__ s16x2 const_pair(int lo, int hi)
{
    uint32_t k = (static_cast<uint32_t>(lo) & 0xffffu) | (static_cast<uint32_t>(hi) << 16);
#if defined(__HIP_DEVICE_COMPILE__)
    asm("" : "+s"(k));
#endif
    return __builtin_bit_cast(s16x2, k);
}

__host__ __device__ __forceinline__ void idct8_row_pk(const RowPk& p, int (&v)[8])
{
    const s16x2 k0p = const_pair(2048, 2048), k0m = const_pair(2048, -2048);
    const s16x2 k4 = const_pair(kC1, kC7), k5 = const_pair(kC7, -kC1);
    const s16x2 k6 = const_pair(kC3, kC5), k7 = const_pair(-kC5, kC3);
    const s16x2 k3 = const_pair(kC2, kC6), k2 = const_pair(kC6, -kC2);
    const s16x2 k6n = const_pair(-kC3, -kC5), k7n = const_pair(kC5, -kC3);
    const s16x2 k3n = const_pair(-kC2, -kC6), k2n = const_pair(-kC6, kC2);
    const int e8 = sdot2<128>(p.p04, k0p);   // (b0 << 11) + 128 + (b4 << 11)
    const int e0 = sdot2<128>(p.p04, k0m);   // (b0 << 11) + 128 - (b4 << 11)
    const int o4 = sdot2<0>(p.p17, k4);
    const int o5 = sdot2<0>(p.p17, k5);
    // the stage-2 sums and differences accumulate onto the stage-1 products:
    // one dot2 each instead of a dot2 per product plus an add per sum
    // (o6 = (b3,b5).k6, o7 = (b3,b5).k7, e3 = (b2,b6).k3, e2 = (b2,b6).k2)
    const int a1 = sdot2acc(p.p35, k6, o4), a4 = sdot2acc(p.p35, k6n, o4);   // o4 +- o6
    const int a6 = sdot2acc(p.p35, k7, o5), a5 = sdot2acc(p.p35, k7n, o5);   // o5 +- o7
    const int f7 = sdot2acc(p.p26, k3, e8), f8 = sdot2acc(p.p26, k3n, e8);   // e8 +- e3
    const int f3 = sdot2acc(p.p26, k2, e0), f0 = sdot2acc(p.p26, k2n, e0);   // e0 +- e2
    const int g2 = (mul181(a4 + a5) + 128) >> 8;
    const int g4 = (mul181(a4 - a5) + 128) >> 8;
    v[0] = (f7 + a1) >> 8; v[1] = (f3 + g2) >> 8; v[2] = (f0 + g4) >> 8; v[3] = (f8 + a6) >> 8;
    v[4] = (f8 - a6) >> 8; v[5] = (f0 - g4) >> 8; v[6] = (f3 - g2) >> 8; v[7] = (f7 - a1) >> 8;
}

// ---------------------------------------------------------------------------
// Colour conversion.  Reference (src/decoder.cpp:367-370 + src/macro.h:121-145):
//   R = (int)(Y + 1.402*V + 128), G = (int)(Y - 0.34414*U - 0.71414*V + 128),
//   B = (int)(Y + 1.772*U + 128) in C double, each clamped to [0,255],
//   packed 0x00RRGGBB (bytes B,G,R,0).
//
// Exact-integer restatement used by the kernel (proved over all 2^27
// (Y,U,V) in [-256,255]^3 against the reference's hash by
// tests/test_oracle.py::test_integer_csc_formulation_is_exact, and the device
// code itself by the exhaustive device test in tests/test_gpu_parity.py):
//   * clamp(trunc(x)) == clamp(floor(x)) for every real x, and Y+128 is an
//     integer, so each channel is clamp(Y + 128 + floor(chroma term));
//   * the +128 level shift is folded into the luma IDCT (its DC rounding
//     constant, idct8<true, 128>): the colour stage receives Ys = Y + 128;
//   * every chroma term is produced in the HIGH int16 of a 32-bit word, so
//     one v_perm per channel assembles the int16 pair of two pixels:
//       floor(1.402 v)               = hi16(v * 91881)
//       floor(1.772 u)               = hi16(u * 116130), except at u = -250
//         (one below: -444; Ys + B <= 383 - 443 < 0 there, so B saturates
//         to 0 either way and the pixel is the same)
//       floor(-(17207u+35707v)/50000) = hi16(mulhi_i32(128*(-17207u-35707v), 43980466))
//     (43980466 = ceil(2^48 / 6.4e6)).  All four products are 24-bit
//     multiplies reading the packed sample through SDWA (no extraction); the third
//     is exact except where the division is exact with a negative quotient:
//     (U,V) = (-200,200) and (-100,100), the only grid points whose mulhi
//     has low half 0xffff (every other point's is <= 0xfffe).  There the
//     value is one below the floor; the reference itself is one below the
//     floor at (-200,200) for Y in [188,201] (its double rounding).  So the
//     flag marks a pixel whose G term needs +1 unless it is that corner at
//     those Y.  Callers take the corrected path only when some lane of the
//     wave has a flagged pixel.
// Chroma terms are computed once per chroma sample and shared by the 4 (4:2:0)
// pixels that replicate it.
// ---------------------------------------------------------------------------
constexpr int kLumaLevel = 128;    // Ys = Y + 128, folded into the luma IDCT
constexpr int kRK = 91881;         // floor(1.402 v) = (v * kRK) >> 16
constexpr int kBK = 116130;        // floor(1.772 u) = (u * kBK) >> 16 but at u = -250 (saturated)
constexpr int kGScale = 128;
constexpr int kGKu = -17207 * kGScale, kGKv = -35707 * kGScale;   // 24-bit signed
constexpr int kGMagic = 43980466;  // ceil(2^48 / (50000 * kGScale))
constexpr int kGCornerQ = -75;     // G term at (U,V) = (-200,200) before correction
constexpr int kGCornerYs0 = 188 + kLumaLevel;   // Y in [188,201]: the reference's rounding corner

// The three chroma terms of one sample, each in the high int16 of its word.
struct ChromaTerms {
    uint32_t r, g, b;
};

__host__ __device__ __forceinline__ int g_mulhi(int mc)
{
#if defined(__HIP_DEVICE_COMPILE__)
    return __mulhi(mc, kGMagic);
#else
    return static_cast<int>((static_cast<long long>(mc) * kGMagic) >> 32);
#endif
}

// 24-bit multiply of one sign-extended int16 half of a packed sample word by
// an SGPR constant: v_mul_i32_i24 with an SDWA source select, so the sample is
// never unpacked into its own register.
template <int kHalf>
__device__ __forceinline__ int mul24_half(uint32_t w, int k)
{
    int r;
    if constexpr (kHalf == 0)
        asm("v_mul_i32_i24_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD"
            : "=v"(r) : "v"(w), "s"(k));
    else
        asm("v_mul_i32_i24_sdwa %0, sext(%1), %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"
            : "=v"(r) : "v"(w), "s"(k));
    return r;
}

// Chroma terms of the (U,V) sample held in int16 half kHalf of the packed
// words uw, vw: four SDWA 24-bit multiplies (no sample is unpacked), one add
// and G's mulhi.
template <int kHalf>
__device__ __forceinline__ ChromaTerms chroma_terms(uint32_t uw, uint32_t vw)
{
    ChromaTerms t;
    t.r = static_cast<uint32_t>(mul24_half<kHalf>(vw, kRK));
    t.b = static_cast<uint32_t>(mul24_half<kHalf>(uw, kBK));
    t.g = static_cast<uint32_t>(g_mulhi(mul24_half<kHalf>(uw, kGKu) + mul24_half<kHalf>(vw, kGKv)));
    return t;
}

// G flag: the mulhi's low half is 0xffff only at the exact negative quotients
__device__ __forceinline__ bool g_flagged(const ChromaTerms& t) { return static_cast<uint16_t>(t.g) == 0xffffu; }

// ---- packed (2 x int16 per VGPR) pixel math ---------------------------------

__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, a) + __builtin_bit_cast(s16x2, b));
}

// v_sat_pk_u8_i16: two int16 lanes saturated to [0,255] and packed into bytes
// 0 (low lane) and 1 (high lane) -- the clamp255 of src/macro.h:121-126 for two
// pixels in one instruction.
__device__ __forceinline__ uint32_t sat_pk_u8(uint32_t a)
{
    uint32_t r;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(a));
    return r;
}

// v_perm_b32: result byte i = sel byte i of {S1 bytes 0-3 -> 0..3, S0 bytes -> 4..7, 0x0c -> 0}
__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel)
{
    return __builtin_amdgcn_perm(s0, s1, sel);
}
constexpr uint32_t kSelLoLo = 0x05040100u;   // (s1.lo16) | (s0.lo16 << 16)
constexpr uint32_t kSelHiHi = 0x07060302u;   // (s1.hi16) | (s0.hi16 << 16)

// The chroma terms of two pixels as int16 pairs: r = (r0, r1) (low half =
// first pixel), bg0 = (b0, g0) and bg1 = (b1, g1) -- the B and G terms of one
// pixel share a word, so each pixel's saturated B,G bytes come out of one
// v_sat_pk_u8_i16 already in BGRX order.
struct ChromaPair {
    uint32_t r, bg0, bg1;
    int flagged;      // either pixel's G term needs the corrected path
};

__device__ __forceinline__ ChromaPair pair_of(const ChromaTerms& c0, const ChromaTerms& c1)
{
    ChromaPair p;
    p.r = perm(c1.r, c0.r, kSelHiHi);
    p.bg0 = perm(c0.g, c0.b, kSelHiHi);
    p.bg1 = perm(c1.g, c1.b, kSelHiHi);
    p.flagged = static_cast<int>(g_flagged(c0)) | static_cast<int>(g_flagged(c1));
    return p;
}

// (ys.lo + c.lo, ys.lo + c.hi) and (ys.hi + c.lo, ys.hi + c.hi): one packed add
// whose op_sel broadcasts one luma half to both lanes.
__device__ __forceinline__ uint32_t pk_add16_ylo(uint32_t ys, uint32_t c)
{
    uint32_t r;
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1]" : "=v"(r) : "v"(ys), "v"(c));
    return r;
}
__device__ __forceinline__ uint32_t pk_add16_yhi(uint32_t ys, uint32_t c)
{
    uint32_t r;
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(r) : "v"(ys), "v"(c));
    return r;
}

// G-term correction of one flagged pixel (see the block comment above).
__device__ __forceinline__ short g_fix(const ChromaTerms& c, int ys)
{
    if (!g_flagged(c)) return 0;
    const bool corner = static_cast<int>(c.g) >> 16 == kGCornerQ && static_cast<unsigned>(ys - kGCornerYs0) < 14u;
    return corner ? 0 : 1;
}

// Two BGRX pixels from an int16 pair of level-shifted luma samples Ys = Y+128
// (low half first) and their chroma pair.  kCheck applies g_fix; callers take
// that path only when some lane of the wave has a flagged pixel.  3 packed
// adds, 3 saturating packs and 2 byte permutes per two pixels.
template <bool kCheck>
__device__ __forceinline__ void pixels2(uint32_t yspair, const ChromaPair& c, const ChromaTerms* c0,
                                        const ChromaTerms* c1, uint32_t& px0, uint32_t& px1)
{
    const uint32_t R = sat_pk_u8(pk_add16(yspair, c.r));   // bytes r0 r1
    uint32_t bg0 = pk_add16_ylo(yspair, c.bg0);            // (Ys0 + b0, Ys0 + g0)
    uint32_t bg1 = pk_add16_yhi(yspair, c.bg1);            // (Ys1 + b1, Ys1 + g1)
    if constexpr (kCheck) {   // +1 on the G lane (the high int16; a carry out of bit 31 is dropped)
        bg0 += static_cast<uint32_t>(g_fix(*c0, static_cast<short>(yspair))) << 16;
        bg1 += static_cast<uint32_t>(g_fix(*c1, static_cast<int>(yspair) >> 16)) << 16;
    }
    const uint32_t BG0 = sat_pk_u8(bg0), BG1 = sat_pk_u8(bg1);   // bytes b g
    px0 = perm(R, BG0, 0x0c040100u);                      // b0 g0 r0 0
    px1 = perm(R, BG1, 0x0c050100u);                      // b1 g1 r1 0
}

// Scalar form (one pixel, raw Y/U/V) on top of the same code, for the colour test hooks.
__device__ __forceinline__ uint32_t pixel_bgrx(int y, int u, int v)
{
    const ChromaTerms t = chroma_terms<0>(static_cast<uint32_t>(u), static_cast<uint32_t>(v));
    const uint32_t ys = static_cast<uint32_t>(y + kLumaLevel);
    const uint32_t yp = perm(ys, ys, kSelLoLo);
    uint32_t p0, p1;
    pixels2<true>(yp, pair_of(t, t), &t, &t, p0, p1);
    return p0;
}

// Literal fp64 form of src/decoder.cpp:369 (C evaluation order, no FMA
// contraction) -- kept as the cross-check arm of the exhaustive test.
__device__ __forceinline__ uint32_t pixel_bgrx_f64(int y, int u, int v)
{
#pragma clang fp contract(off)
    const double Y = y, U = u, V = v;
    const int r = static_cast<int>(Y + 1.402 * V + 128);
    const int g = static_cast<int>(Y - 0.34414 * U - 0.71414 * V + 128);
    const int b = static_cast<int>(Y + 1.772 * U + 128);
    return (static_cast<uint32_t>(clamp_u8(r)) << 16) | (static_cast<uint32_t>(clamp_u8(g)) << 8) |
           static_cast<uint32_t>(clamp_u8(b));
}

}  // namespace hjd
