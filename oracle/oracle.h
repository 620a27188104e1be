/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's pixel back-end (xinfushe/oclJPEGDecoder,
 * USE_CPU_ONLY build), used as the parity checker for the HIP path.
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may
 * load this library.  The product (ocljpegdecoder_amd/, libhjd.so) never
 * links or calls it.
 *
 * Parity is pinned (tests/test_oracle.py) against:
 *   - golden vectors produced by the reference itself compiled from
 *     /root/reference/src by oracle/Makefile (oracle/_ref/libref.so),
 *   - the sha256 values recorded in SURVEY.md s8(c) for the reference's
 *     only sample, test/JPEG_example_JPG_RIP_050.jpg,
 *   - the clamp-edge known answers of SURVEY.md s8(c).
 */
#ifndef HJD_ORACLE_H
#define HJD_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* standard JPEG zigzag: natural index of zigzag position k (zigzag.h:15-40) */
extern const int32_t oracle_zigzag[64];

/* 8x8 integer IDCT in place, int32 natural order (cpuIDCT8x8.cpp:25-127) */
void oracle_fast_idct(int32_t blk[64]);

/* zigzag + dequant: out[zz[k]] = coef_zz[k] * qt_zz[k] (decoder.cpp:338-342) */
void oracle_dequant_block(const int16_t coef_zz[64], const int32_t qt_zz[64], int32_t out_nat[64]);

/* YUV_to_RGB32 + RGBClamp32 (decoder.cpp:367-370, macro.h:121-145):
 * returns 0x00RRGGBB (little-endian bytes B,G,R,0) */
uint32_t oracle_yuv_to_bgrx(int32_t y, int32_t u, int32_t v);

/* bulk form of oracle_yuv_to_bgrx, for the exhaustive colour test */
void oracle_yuv_to_bgrx_n(const int32_t* y, const int32_t* u, const int32_t* v, uint32_t* out, int64_t n);

/* sampling codes shared with include/hjd.h.  ORACLE_YUV422 (Y H2V1) and
 * ORACLE_GRAY are extensions the reference rejects (decoder.cpp:58-69): the
 * same IDCT and colour arithmetic with nearest horizontal chroma replication,
 * gray as the conversion with U = V = 0.  Parity for them is unpinned by the
 * reference (it has no such path); tests pin the HIP path to this
 * restatement.  ORACLE_YUV411_H4V1 (Y H4V1) and ORACLE_YUV440 (Y H1V2) likewise,
 * with nearest replication along the subsampled axis. */
enum {
    ORACLE_YUV444 = 0, ORACLE_YUV420 = 1, ORACLE_YUV422 = 3, ORACLE_GRAY = 4, ORACLE_YUV411_H4V1 = 5,
    ORACLE_YUV440 = 6
};

/*
 * Whole frame from int16 quantised zigzag coefficients, MCU-major
 * (per MCU: Y blocks in HxV raster, then Cb, then Cr), MCUs in raster order.
 * qt[c] = 64 quantisation values of component c in file (zigzag) order.
 * out = W*H BGRX pixels, pitch out_pitch_px pixels (>= W).
 * Follows decoder.cpp:443-491 (MCU loop) after decoder.cpp:338-342.
 */
int oracle_decode_frame_q16(const int16_t* coefs, const int32_t* qt_y, const int32_t* qt_cb,
                            const int32_t* qt_cr, int width, int height, int sampling,
                            uint32_t* out, int out_pitch_px);

/* Same, from int32 natural-order dequantised blocks (jpg.mcu_data, jpeg.h:76). */
int oracle_decode_frame_i32(const int32_t* mcu_data, int width, int height, int sampling,
                            uint32_t* out, int out_pitch_px);

/* IDCT-only over n blocks (out-of-place; the reference's batch_idct path). */
void oracle_idct_blocks(const int32_t* in, int32_t* out, int64_t nblocks);

/*
 * CPU baseline: nframes identical-geometry frames on a
 * pthread pool, one frame per task.  Frame f reads
 * coefs + (f % ncoef_frames) * coef_stride; worker t writes into its own slot
 * out + t * out_stride (out must hold nthreads slots).  Returns 0 on success.
 */
int oracle_decode_batch_q16_mt(const int16_t* coefs, int64_t coef_stride, int ncoef_frames, const int32_t* qt_y,
                               const int32_t* qt_cb, const int32_t* qt_cr, int width, int height,
                               int sampling, uint32_t* out, int64_t out_stride, int nframes,
                               int nthreads);

#ifdef __cplusplus
}
#endif
#endif
