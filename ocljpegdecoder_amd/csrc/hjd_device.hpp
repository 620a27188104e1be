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
__host__ __device__ __forceinline__ int clamp_sample(int v) { return v < -256 ? -256 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int clamp_u8(int v) { return min(max(v, 0), 255); }

// One 8-point pass on natural-order values v[0..7] (in place).
// kCol = false: row pass, src/cpuIDCT8x8.cpp:36-80 (x<<11, +128 on DC, >>8 out).
// kCol = true:  column pass, src/cpuIDCT8x8.cpp:82-127 (x<<8, +8192 on DC,
//               (+4)>>3 on stage-1/2 products, >>14 out, clamp [-256,255] --
//               the CPU clamp, not the OpenCL kernel's [-256,256] at
//               src/idct8x8.cl:116).
// The reference's DC-only short-cuts (:40-45, :86-92) give exactly the values
// of the full butterfly, so the kernel always runs the full butterfly.
template <bool kCol>
__host__ __device__ __forceinline__ void idct8(int (&v)[8])
{
    constexpr int kIn = kCol ? 8 : 11;
    constexpr int kRnd = kCol ? 4 : 0;
    constexpr int kSh = kCol ? 3 : 0;

    int e0 = (v[0] << kIn) + (kCol ? 8192 : 128);
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
        v[0] = clamp_sample(r0 >> 14); v[1] = clamp_sample(r1 >> 14);
        v[2] = clamp_sample(r2 >> 14); v[3] = clamp_sample(r3 >> 14);
        v[4] = clamp_sample(r4 >> 14); v[5] = clamp_sample(r5 >> 14);
        v[6] = clamp_sample(r6 >> 14); v[7] = clamp_sample(r7 >> 14);
    } else {
        v[0] = r0 >> 8; v[1] = r1 >> 8; v[2] = r2 >> 8; v[3] = r3 >> 8;
        v[4] = r4 >> 8; v[5] = r5 >> 8; v[6] = r6 >> 8; v[7] = r7 >> 8;
    }
}

// ---------------------------------------------------------------------------
// Colour conversion.  Reference (src/decoder.cpp:367-370 + src/macro.h:121-145):
//   R = (int)(Y + 1.402*V + 128), G = (int)(Y - 0.34414*U - 0.71414*V + 128),
//   B = (int)(Y + 1.772*U + 128) in C double, each clamped to [0,255],
//   packed 0x00RRGGBB (bytes B,G,R,0).
//
// Exact-integer restatement used by the kernel (proved by an exhaustive
// device test over all 2^27 (Y,U,V) in [-256,255]^3, tests/test_gpu_parity.py):
//   * clamp(trunc(x)) == clamp(floor(x)) for every real x;
//   * Y+128 is an integer, so floor(x) = Y + 128 + floor(chroma term);
//   * 1.402 = 701/500 and 1.772 = 443/250: for V,U != 0 the chroma term sits
//     >= 1/500 from an integer, far above fp32/fp64 rounding, so
//     floor(float(V)*1.402f) is exact (and exactly 0 for V == 0);
//   * G's term is -(17207U + 35707V)/50000; it is computed as an exact integer
//     floor division.  When the division is exact, the reference's double
//     rounding can land one below the integer: over the whole domain this
//     happens only for (U,V) = (-200,200) with Y in [188,201], where the
//     reference gives one less (enumerated in tests/test_oracle.py).
// Chroma terms are computed once per chroma sample and shared by the 4 (4:2:0)
// pixels that replicate it.
// ---------------------------------------------------------------------------
struct ChromaTerms {
    int rq, gq, bq;
    int special;
};

// Exact fixed-point floors (S = 20; K and the bias searched and proved over
// v,u in [-256,255] by tests/test_oracle.py::test_fixed_point_colour_terms):
//   floor(1.402 v) + 128 = (v*1470091 + (128<<20) + 1048) >> 20
//   floor(1.772 u) + 128 = (u*1858077 + (128<<20) + 2097) >> 20
// The +2^20/(2*den) bias keeps every case >= 1/1000 (R) or 1/500 (B) away
// from an integer, which also covers the exact multiples (u = +-250).
constexpr int kRK = 1470091, kRBias = (128 << 20) + 1048;
constexpr int kBK = 1858077, kBBias = (128 << 20) + 2097;

__host__ __device__ __forceinline__ int r_term(int v) { return (mul24(v, kRK) + kRBias) >> 20; }
__host__ __device__ __forceinline__ int b_term(int u) { return (mul24(u, kBK) + kBBias) >> 20; }

// floor(-(17207u + 35707v) / 50000) + 128, exactly, with one multiply-high:
// m' = -(17207u + 35707v) + 300*50000 lies in [1.5e6, 2.9e7] < 2^25, and
// floor(m'/50000) == mulhi(m', 2814749768) >> 15 for every m' < 2^25
// (2814749768 = ceil(2^47/50000); exhaustively checked in
// tests/test_oracle.py::test_fixed_point_colour_terms).  The offset's 300 is
// removed together with the +128 level shift (-172).  m' also identifies the
// double-rounding corner: (U,V) = (-200,200) is the only grid point with
// m' = 11,300,000.
constexpr int kGOffset = 15000000;
constexpr unsigned kGMagic = 2814749768u;
constexpr int kGSpecial = 11300000;

__host__ __device__ __forceinline__ int g_mprime(int u, int v) { return mul24(u, -17207) + mul24(v, -35707) + kGOffset; }

__host__ __device__ __forceinline__ int g_term_from_m(int mp)
{
#if defined(__HIP_DEVICE_COMPILE__)
    const unsigned hi = __umulhi(static_cast<unsigned>(mp), kGMagic);
#else
    const unsigned hi = static_cast<unsigned>((static_cast<unsigned long long>(static_cast<unsigned>(mp)) * kGMagic) >> 32);
#endif
    return static_cast<int>(hi >> 15) - 172;
}

__device__ __forceinline__ ChromaTerms chroma_terms(int u, int v)
{
    ChromaTerms t;
    t.rq = r_term(v);
    t.bq = b_term(u);
    const int mp = g_mprime(u, v);
    t.gq = g_term_from_m(mp);
    t.special = mp == kGSpecial;
    return t;
}

// ---- packed (2 x int16 per VGPR) pixel math ---------------------------------
typedef short s16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ uint32_t pk_add16(uint32_t a, uint32_t b)
{
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, a) + __builtin_bit_cast(s16x2, b));
}

__device__ __forceinline__ uint32_t pk_clamp_u8(uint32_t a)
{
    s16x2 x = __builtin_bit_cast(s16x2, a);
    x = __builtin_elementwise_max(x, (s16x2){0, 0});
    x = __builtin_elementwise_min(x, (s16x2){255, 255});
    return __builtin_bit_cast(uint32_t, x);
}

// v_sat_pk_u8_i16: two int16 lanes saturated to [0,255] and packed into bytes
// 0 (low lane) and 1 (high lane) -- the clamp255 of src/macro.h:121-126 for two
// pixels in one instruction (replaces a packed max + min).
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

// The chroma terms of two pixels as int16 pairs (low half = first pixel).
struct ChromaPair {
    uint32_t r, g, b;
    int special;      // either pixel's chroma is the (U,V) = (-200,200) corner
};

__device__ __forceinline__ ChromaPair pair_of(const ChromaTerms& c0, const ChromaTerms& c1)
{
    ChromaPair p;
    p.r = perm(c1.rq, c0.rq, kSelLoLo);
    p.g = perm(c1.gq, c0.gq, kSelLoLo);
    p.b = perm(c1.bq, c0.bq, kSelLoLo);
    p.special = c0.special | c1.special;
    return p;
}

// Two BGRX pixels from an int16 pair of Y samples (low half first) and their
// chroma pair.  kCheckSpecial adds the reference's double-rounding corner
// (G one lower for (U,V) = (-200,200), Y in [188,201]); callers take that path
// only when some lane of the wave needs it.
template <bool kCheckSpecial>
__device__ __forceinline__ void pixels2(uint32_t ypair, const ChromaPair& c, const ChromaTerms* c0,
                                        const ChromaTerms* c1, uint32_t& px0, uint32_t& px1)
{
    const uint32_t R = sat_pk_u8(pk_add16(ypair, c.r));   // bytes r0 r1
    uint32_t graw = pk_add16(ypair, c.g);
    if constexpr (kCheckSpecial) {
        const int y0 = static_cast<short>(ypair), y1 = static_cast<int>(ypair) >> 16;
        const short d0 = (c0->special && static_cast<unsigned>(y0 - 188) < 14u) ? 1 : 0;
        const short d1 = (c1->special && static_cast<unsigned>(y1 - 188) < 14u) ? 1 : 0;
        graw = __builtin_bit_cast(uint32_t, __builtin_bit_cast(s16x2, graw) - (s16x2){d0, d1});
    }
    const uint32_t G = sat_pk_u8(graw);                   // bytes g0 g1
    const uint32_t B = sat_pk_u8(pk_add16(ypair, c.b));   // bytes b0 b1
    const uint32_t T = perm(G, B, 0x05010400u);           // b0 g0 b1 g1
    px0 = perm(R, T, 0x0c040100u);                        // b0 g0 r0 0
    px1 = perm(R, T, 0x0c050302u);                        // b1 g1 r1 0
}

// Scalar form (one pixel) on top of the same code, for the colour test hooks.
__device__ __forceinline__ uint32_t pixel_bgrx(int y, const ChromaTerms& t)
{
    const uint32_t yp = perm(static_cast<uint32_t>(y), static_cast<uint32_t>(y), kSelLoLo);
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
