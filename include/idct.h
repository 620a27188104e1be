/*
 * idct.h -- drop-in replacement for the reference's back-end header
 * (xinfushe/oclJPEGDecoder src/idct.h:4-18), implemented by libhjd.so on top of
 * the C ABI in hjd.h.  Same names, same C++ signatures (so the same mangled
 * symbols, e.g. _Z22clidct_allocate_memoryimmii), same bool/int results, so
 * src/decoder.cpp links against libhjd.so in place of src/oclDCT8x8.cpp +
 * OpenCL.
 *
 * Behaviour kept from the reference (src/oclDCT8x8.cpp):
 *   - int32 natural-order dequantised blocks in (jpg.mcu_data layout);
 *   - BGRX out, alpha byte 0, cropped to W x H, row pitch W*4;
 *   - functions return false/-1 and print to stderr, never throw;
 *   - Initialize_OpenCL_IDCT() tolerates "no device" (returns 1).
 * Behaviour fixed (documented in INTEGRATION.md):
 *   - clidct_transfer_data_to_device honours `offset` (the reference ignores it,
 *     src/oclDCT8x8.cpp:148-153);
 *   - the column clamp is [-256,255] as in the CPU path (the OpenCL kernel uses
 *     [-256,256], src/idct8x8.cl:116), so GPU output == CPU output;
 *   - the input buffer is never modified by clidct_run (the OpenCL kernel
 *     transforms it in place); clidct_retrieve_data_from_device still returns
 *     the IDCT'd blocks, as the reference's would after a run.
 * The four CPU entry points (Initialize_Fast_IDCT, Fast_IDCT, idctrow, idctcol)
 * are the reference's USE_CPU_ONLY back-end API; they run on the host and are
 * never used by the GPU entry points.
 */
#ifndef HJD_IDCT_H
#define HJD_IDCT_H

#include <stddef.h>

/* The reference's src/macro.h:114-119 defines this enum; a translation unit that
 * already includes that header defines HJD_HAVE_COLORSPACE to skip this copy. */
#ifndef HJD_HAVE_COLORSPACE
#define HJD_HAVE_COLORSPACE
enum ColorSpace { YUV444, YUV411, Other };
#endif

/* CPU back-end (src/cpuIDCT8x8.cpp) */
void Initialize_Fast_IDCT();
void Fast_IDCT(int* block);
void idctrow(int* blk);
void idctcol(int* blk);

/* GPU back-end (src/oclDCT8x8.cpp), MI355X/HIP implementation */
int Initialize_OpenCL_IDCT();
bool clidct_create();
bool clidct_allocate_memory(const int total_blocks, const size_t image_width, const size_t image_height,
                            const int mcu_width, const int mcu_height);
bool clidct_transfer_data_to_device(const int block_data_src[1][64], const int offset, const int count);
bool clidct_build(ColorSpace colorspace);
bool clidct_run(ColorSpace colorspace);
bool clidct_retrieve_data_from_device(int block_data_dest[1][64]);
bool clidct_retrieve_image_from_device(void* img_data_dest, const size_t img_width, const size_t img_height);
bool clidct_wait_for_completion();
bool clidct_clean_up();

#endif /* HJD_IDCT_H */
