// VALU throughput probe (tuning tool, not product): cycles per wave64
// instruction per SIMD for the integer/packed ops the pixel kernel uses.
// 8 independent chains per lane, 256 WGs x 1024 threads (16 waves/CU... 4/SIMD), timed by events.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define N_ITER 4096
#define CHAIN 8

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t seed)
{
    uint32_t a[CHAIN];
    for (int i = 0; i < CHAIN; ++i) a[i] = seed + threadIdx.x * 7 + i * 13;
    const uint32_t k = seed | 1;
    for (int it = 0; it < N_ITER; ++it) {
#pragma unroll
        for (int i = 0; i < CHAIN; ++i) {
            uint32_t x = a[i];
            if constexpr (OP == 0) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 1) asm volatile("v_mad_i32_i24 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 2) asm volatile("v_mul_lo_u32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 3) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(x) : "v"(k), "v"(k + 255));
            if constexpr (OP == 4) asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 5) asm volatile("v_perm_b32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 6) asm volatile("v_cvt_f32_i32 %0, %0" : "+v"(x));
            if constexpr (OP == 7) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 8) asm volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 9) asm volatile("v_ashrrev_i32 %0, 3, %0" : "+v"(x));
            if constexpr (OP == 10) asm volatile("v_mul_i32_i24 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 11) asm volatile("v_cvt_flr_i32_f32 %0, %0" : "+v"(x));
            if constexpr (OP == 12) asm volatile("v_lshl_add_u32 %0, %0, 2, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 13) asm volatile("v_add3_u32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 14) asm volatile("v_dot2_i32_i16 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 15) asm volatile("v_pk_mul_lo_u16 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 16) asm volatile("v_pk_mad_i16 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 17) asm volatile("v_alignbit_b32 %0, %0, %1, %0" : "+v"(x) : "v"(k));
            if constexpr (OP == 18) asm volatile("v_bfe_u32 %0, %0, %1, 5" : "+v"(x) : "v"(k));
            if constexpr (OP == 19) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x) : "v"(k));
            if constexpr (OP == 20) asm volatile("v_mov_b32 %0, %1" : "+v"(x) : "v"(k + x));
            if constexpr (OP == 21) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(*reinterpret_cast<uint64_t*>(&a[i & ~1])));
            if constexpr (OP == 22) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_0" : "+v"(x) : "v"(k));
            if constexpr (OP == 23) asm volatile("v_or_b32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:DWORD" : "+v"(x) : "v"(k));
            if constexpr (OP == 24) asm volatile("v_add_u32_sdwa %0, sext(%0), %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD" : "+v"(x) : "v"(k));
            if constexpr (OP == 25) asm volatile("v_or_b32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 26) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 27) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x));
            if constexpr (OP == 28) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 29) asm volatile("v_max_i32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 30) asm volatile("v_mul_hi_i32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 31) asm volatile("v_mul_hi_i32_i24 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 32) asm volatile("v_sat_pk_u8_i16 %0, %0" : "+v"(x));
            if constexpr (OP == 33) asm volatile("v_cvt_pk_i16_i32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 34) asm volatile("v_lshl_or_b32 %0, %0, 16, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 35) asm volatile("v_or3_b32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 36) asm volatile("v_add_lshl_u32 %0, %0, %1, 2" : "+v"(x) : "v"(k));
            if constexpr (OP == 37) asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 38) asm volatile("v_dot2c_i32_i16 %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 39) asm volatile("v_mul_u32_u24 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 40) asm volatile("v_cmp_eq_u32 vcc, %0, %1\n v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k) : "vcc");
            if constexpr (OP == 41) asm volatile("v_cmp_eq_u32_sdwa vcc, %0, %1 src0_sel:WORD_0 src1_sel:DWORD\n v_add_u32 %0, %0, %1" : "+v"(x) : "v"(k) : "vcc");
            if constexpr (OP == 42) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[40:41]" : "+v"(x) : "v"(k));
            if constexpr (OP == 43) asm volatile("v_mov_b32_sdwa %0, %1 dst_sel:BYTE_2 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0" : "+v"(x) : "v"(k));
            if constexpr (OP == 44) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 45) asm volatile("v_ashrrev_i32_sdwa %0, 3, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:DWORD" : "+v"(x));
            if constexpr (OP == 46) asm volatile("v_pk_add_u16 %0, %0, %1 op_sel:[1,0] op_sel_hi:[1,1]" : "+v"(x) : "v"(k));
            if constexpr (OP == 47) asm volatile("v_mad_u32_u24 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 48) asm volatile("v_min3_i32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            if constexpr (OP == 49) asm volatile("v_bfi_b32 %0, %0, %1, %1" : "+v"(x) : "v"(k));
            a[i] = x;
        }
    }
    uint32_t s = 0;
    for (int i = 0; i < CHAIN; ++i) s ^= a[i];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP>
float run(uint32_t* out, int blocks, const char* name)
{
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 1u);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 3u);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // instructions per SIMD: blocks*4 waves spread over 256 CUs x 4 SIMDs
    const double waves_per_simd = blocks * 4.0 / (256 * 4);
    const double instr = waves_per_simd * N_ITER * CHAIN;
    const double clk = 2.1e9;   // approx; also print ns per instr
    printf("%-20s %8.3f ms  %.2f ns/instr/SIMD  ~%.2f cyc@2.1GHz\n", name, ms, ms * 1e6 / instr, ms * 1e-3 * clk / instr);
    return ms;
}

int main()
{
    uint32_t* out;
    const int blocks = 256 * 4;   // 4 WG/CU of 4 waves = 4 waves per SIMD
    (void)hipMalloc(&out, blocks * 256 * 4);
    run<0>(out, blocks, "v_add_u32");
    run<5>(out, blocks, "v_perm_b32");
    run<10>(out, blocks, "v_mul_i32_i24");
    run<19>(out, blocks, "v_cndmask_b32");
    run<22>(out, blocks, "v_mov_sdwa_w1pres");
    run<23>(out, blocks, "v_or_b32_sdwa");
    run<24>(out, blocks, "v_add_u32_sdwa");
    run<25>(out, blocks, "v_or_b32_e32");
    run<26>(out, blocks, "v_and_b32_e32");
    run<27>(out, blocks, "v_lshlrev_b32_e32");
    run<28>(out, blocks, "v_sub_u32_e32");
    run<29>(out, blocks, "v_max_i32_e32");
    run<30>(out, blocks, "v_mul_hi_i32");
    run<31>(out, blocks, "v_mul_hi_i32_i24");
    run<32>(out, blocks, "v_sat_pk_u8_i16");
    run<33>(out, blocks, "v_cvt_pk_i16_i32");
    run<34>(out, blocks, "v_lshl_or_b32");
    run<35>(out, blocks, "v_or3_b32");
    run<36>(out, blocks, "v_add_lshl_u32");
    run<37>(out, blocks, "v_add_u32_e64");
    run<38>(out, blocks, "v_dot2c_i32_i16");
    run<39>(out, blocks, "v_mul_u32_u24_e32");
    run<40>(out, blocks, "v_cmp+add (pair)");
    run<41>(out, blocks, "v_cmp_sdwa+add (pair)");
    run<42>(out, blocks, "v_cndmask sgpr-mask");
    run<43>(out, blocks, "v_mov_sdwa_b2pres");
    run<44>(out, blocks, "v_xor_b32_e32");
    run<45>(out, blocks, "v_ashrrev_sdwa");
    run<46>(out, blocks, "v_pk_add_u16 opsel");
    run<47>(out, blocks, "v_mad_u32_u24");
    run<48>(out, blocks, "v_min3_i32");
    run<49>(out, blocks, "v_bfi_b32");
    return 0;
}
