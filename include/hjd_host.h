/*
 * hjd_host.h -- host JPEG front end of the MI355X pixel back-end (C ABI).
 *
 * Baseline-JPEG marker parsing and Huffman (entropy) decoding on the CPU,
 * producing exactly the input of the fused kernel: int16 quantised
 * coefficients in zigzag order, MCU-major, with DC prediction applied
 * (src/decoder.cpp:221-346 of xinfushe/oclJPEGDecoder), plus the frame's
 * quantisation tables in file order.  Supports what the reference supports
 * (src/decoder.cpp:18-70): 8-bit samples, 3 components, 4:2:0 (H2V2,H1V1,H1V1)
 * or 4:4:4, restart intervals (DRI/RSTn).  Deliberate differences from the
 * reference parser, all of them fixes: 16-bit DQT entries are read big-endian
 * (src/parser.cpp:83-86 reads them native-endian); scan components are matched
 * to frame components by id (src/decoder.cpp:315 assumes equal order); APPn,
 * COM and other non-frame markers are skipped anywhere before SOS.
 *
 * Also: a stream object that pipelines host Huffman decoding (worker
 * threads), pinned host staging, hipMemcpyAsync H2D on a copy stream and the
 * fused kernel on a compute stream (double/triple buffering).
 */
#ifndef HJD_HOST_H
#define HJD_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "hjd.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hjd_jpeg_info {
    int32_t width;
    int32_t height;
    int32_t sampling;          /* HJD_YUV444 or HJD_YUV420 */
    int32_t restart_interval;  /* MCUs per restart interval, 0 = none */
    int32_t mcu_w;             /* MCU grid */
    int32_t mcu_h;
    int64_t nblocks;           /* coefficient blocks (64 int16 each) */
    int32_t qt[3][64];         /* quantisation table of each component, file (zigzag) order */
    int32_t qt_precision[3];   /* 0 = 8-bit DQT entries, 1 = 16-bit */
    int64_t scan_offset;       /* byte offset of the entropy-coded segment */
} hjd_jpeg_info;

/* Parse headers up to SOS.  Returns HJD_OK, or HJD_E_INVALID for malformed or
 * unsupported files (hjd_last_error() says why). */
int hjd_jpeg_parse(const uint8_t* data, size_t size, hjd_jpeg_info* info);

/* Parse + Huffman-decode one file into coefs (capacity in blocks). */
int hjd_jpeg_decode_coefs(const uint8_t* data, size_t size, hjd_jpeg_info* info, int16_t* coefs,
                          int64_t capacity_blocks);

/* Decode n files on `nthreads` host threads (0 = hardware concurrency);
 * status[i] receives each file's return code.  Returns HJD_OK if all
 * succeeded. */
int hjd_jpeg_decode_batch(const uint8_t* const* datas, const size_t* sizes, int n, int16_t* const* coefs,
                          int64_t capacity_blocks, int nthreads, int32_t* status);

/* ---- streaming decode (host Huffman || H2D || kernel) ------------------- */
typedef struct hjd_stream hjd_stream;

/* nslots pinned staging slots of max_blocks coefficient blocks each (>= 2;
 * 3 = triple buffering); nthreads host Huffman workers (0 = hw concurrency). */
int hjd_stream_create(hjd_ctx* ctx, int64_t max_blocks, int nslots, int nthreads, hjd_stream** out);
int hjd_stream_destroy(hjd_stream* s);

/* Queue one JPEG (the bytes must stay valid until hjd_stream_sync returns).
 * Its BGRX pixels are written to d_out (device memory, row pitch out_pitch
 * bytes) by the fused kernel once its coefficients reach the device. */
int hjd_stream_submit(hjd_stream* s, const uint8_t* data, size_t size, void* d_out, int32_t out_pitch);

/* Wait for every submitted image; returns the first error, if any.  stats (may
 * be NULL) receives {images, pixels, host_decode_ns, h2d_bytes, kernel_launches}. */
int hjd_stream_sync(hjd_stream* s, int64_t stats[5]);

#ifdef __cplusplus
}
#endif
#endif
