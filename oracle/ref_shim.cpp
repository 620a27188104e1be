// ref_shim.cpp -- TEST INFRASTRUCTURE ONLY.
//
// Thin C-ABI over the reference CPU path compiled *from its own sources* under
// /root/reference/src (see oracle/Makefile; nothing from the reference is copied
// into this repo).  Built into oracle/_ref/libref.so and used only by the golden
// fixture generator (tests/golden/make_golden.py), the oracle pinning tests and,
// optionally, bench.py's cpu_baseline leg.
//
// Capture: the Makefile links with -Wl,--wrap=_Z9Fast_IDCTPi so every call the
// reference's decode_mcu_data (src/decoder.cpp:448-452) makes to Fast_IDCT
// (src/cpuIDCT8x8.cpp:25) passes through __wrap_ below, which records the
// dequantised natural-order input block (jpg.mcu_data, src/jpeg.h:76) and the
// IDCT output, in the reference's own MCU-major order.
#include <stdio.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "stdafx.h"
#include "macro.h"
#include "jpeg.h"
#include "idct.h"

bool load_jpg(const char* filePath);                      // src/parser.cpp:272
bool decode_mcu_data(const JPG_DATA& jpg, FILE* const fp); // src/decoder.cpp:397
uint32_t YUV_to_RGB32(coef_t Y, coef_t U, coef_t V);     // src/decoder.cpp:367

static FILE* g_cap_in = nullptr;
static FILE* g_cap_out = nullptr;

extern "C" void __real__Z9Fast_IDCTPi(int* block);
extern "C" void __wrap__Z9Fast_IDCTPi(int* block)
{
    if (g_cap_in) fwrite(block, sizeof(int), 64, g_cap_in);
    __real__Z9Fast_IDCTPi(block);
    if (g_cap_out) fwrite(block, sizeof(int), 64, g_cap_out);
}

extern "C" {

void ref_init(void) { Initialize_Fast_IDCT(); }

void ref_fast_idct(int32_t* blk) { Fast_IDCT(blk); }

void ref_fast_idct_n(int32_t* blk, int64_t n)
{
    for (int64_t i = 0; i < n; i++) Fast_IDCT(blk + 64 * i);
}

uint32_t ref_yuv_to_rgb32(int32_t y, int32_t u, int32_t v) { return YUV_to_RGB32(y, u, v); }

void ref_yuv_to_rgb32_n(const int32_t* y, const int32_t* u, const int32_t* v, uint32_t* out, int64_t n)
{
    for (int64_t i = 0; i < n; i++) out[i] = YUV_to_RGB32(y[i], u[i], v[i]);
}

// Decode `path` with the reference (USE_CPU_ONLY).  The reference writes its
// BMP to "m:\\output.bmp" in the current directory (src/decoder.cpp:420); the
// caller chdir()s into a scratch directory first.  When capture paths are
// given, the IDCT input/output blocks are appended there.
int ref_load_jpg(const char* path, const char* cap_in, const char* cap_out)
{
    g_cap_in = cap_in ? fopen(cap_in, "wb") : nullptr;
    g_cap_out = cap_out ? fopen(cap_out, "wb") : nullptr;
    bool ok = load_jpg(path);
    if (g_cap_in) fclose(g_cap_in);
    if (g_cap_out) fclose(g_cap_out);
    g_cap_in = g_cap_out = nullptr;
    return ok ? 0 : -1;
}

// Run the reference's own pixel back-end, decode_mcu_data (src/decoder.cpp:397,
// USE_CPU_ONLY: Fast_IDCT per block + YUV_to_RGB32 + its BMP fwrite), on an
// int32 natural-order dequantised block buffer (jpg.mcu_data layout) that this
// function is allowed to overwrite (the reference IDCTs in place).  Only the
// JPG_DATA fields that decode_mcu_data reads are filled.  Writes
// "m:\\output.bmp" in the current directory.  Used as the reference CPU
// timing leg of bench.py.
int ref_decode_mcu_data(int32_t* mcu_data, int width, int height, int sampling)
{
    JPG_DATA jpg;
    memset(&jpg, 0, sizeof(jpg));
    jpg.frame_info.bit_depth = 8;
    jpg.frame_info.img_width = (uint16_t)width;
    jpg.frame_info.img_height = (uint16_t)height;
    jpg.frame_info.num_channels = 3;
    const uint8_t sy = sampling == 1 ? 0x22 : 0x11;
    jpg.frame_info.channel_info[0].sampling_factor = sy;
    jpg.frame_info.channel_info[1].sampling_factor = 0x11;
    jpg.frame_info.channel_info[2].sampling_factor = 0x11;
    jpg.blks_per_mcu[0] = sampling == 1 ? 4 : 1;
    jpg.blks_per_mcu[1] = 1;
    jpg.blks_per_mcu[2] = 1;
    jpg.tot_blks_per_mcu = jpg.blks_per_mcu[0] + 2;
    jpg.mcu_width = jpg.mcu_height = sampling == 1 ? 16 : 8;
    jpg.mcu_count_w = (width - 1) / jpg.mcu_width + 1;
    jpg.mcu_count_h = (height - 1) / jpg.mcu_height + 1;
    jpg.mcu_count = jpg.mcu_count_w * jpg.mcu_count_h;
    jpg.blk_count = jpg.mcu_count * jpg.tot_blks_per_mcu;
    jpg.color_space = sampling == 1 ? YUV411 : YUV444;
    jpg.mcu_data = reinterpret_cast<coef_t(*)[64]>(mcu_data);
    return decode_mcu_data(jpg, nullptr) ? 0 : -1;
}

}  // extern "C"
