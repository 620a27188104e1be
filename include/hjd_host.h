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
    int32_t sampling;          /* HJD_YUV444, HJD_YUV420, HJD_YUV422 or HJD_GRAY */
    int32_t restart_interval;  /* MCUs per restart interval, 0 = none */
    int32_t mcu_w;             /* MCU grid */
    int32_t mcu_h;
    int64_t nblocks;           /* coefficient blocks (64 int16 each) */
    int32_t qt[3][64];         /* quantisation table of each component, file (zigzag) order */
    int32_t qt_precision[3];   /* 0 = 8-bit DQT entries, 1 = 16-bit */
    int64_t scan_offset;       /* byte offset of the (first) entropy-coded segment */
    int32_t process;           /* 0 = baseline (SOF0), 1 = extended sequential (SOF1), 2 = progressive (SOF2) */
    int32_t single_scan;       /* 1: one interleaved sequential scan holds the image (0: several scans, or progressive;
                                  the GPU entropy decoder takes every sequential file, process 0 or 1) */
} hjd_jpeg_info;

/* Besides the reference's single interleaved baseline scan, the host decoder
 * takes sequential files with several scans (SOF0/SOF1: non-interleaved or
 * partly interleaved components) and progressive files (SOF2: spectral
 * selection + successive approximation, EOB runs, restarts); the result is the
 * same coefficient layout.  For those, qt[] is final after decode (tables
 * latch at each component's first scan). */

/* Parse headers up to SOS.  Returns HJD_OK, or HJD_E_INVALID for malformed or
 * unsupported files (hjd_last_error() says why). */
int hjd_jpeg_parse(const uint8_t* data, size_t size, hjd_jpeg_info* info);

/* Parse + Huffman-decode one file into coefs (capacity in blocks). */
int hjd_jpeg_decode_coefs(const uint8_t* data, size_t size, hjd_jpeg_info* info, int16_t* coefs,
                          int64_t capacity_blocks);

/* The calling process's CPU share: the CPUs in its affinity mask, capped by
 * its cgroup's CPU quota, rounded up (the cgroup of /proc/self/cgroup and its
 * ancestors; v2 cpu.max or v1 cpu.cfs_quota_us / cpu.cfs_period_us; computed
 * once per process).  A container granted 16 CPUs of time on a 256-CPU host
 * gets 16, not 256.  The default thread count (nthreads = 0) of
 * hjd_jpeg_decode_batch; hjd_stream_create and hjd_gstream_create cap it by
 * the device's CPU slice (hjd_device_worker_cpus). */
int hjd_host_cpu_share(void);
/* hjd_host_cpu_share computed from the tree at `root` ("/proc/self/cgroup",
 * "/sys/fs/cgroup/..." under it; NULL = the real one, not cached): tests. */
int hjd_debug_cpu_share(const char* root);
/* The host CPUs the stream workers of HIP device `device` bind to: its NUMA
 * node's CPUs this process may use, split evenly among the node's visible
 * GPUs (hjd_debug_worker_cpus on the real topology).  Writes up to `capacity`
 * ids; *ncpus = how many (0: unknown topology, no binding). */
int hjd_device_worker_cpus(int device, int32_t* cpus, int capacity, int32_t* ncpus);

/* Decode n files on `nthreads` host threads (0 = hjd_host_cpu_share());
 * status[i] receives each file's return code.  Returns HJD_OK if all
 * succeeded. */
int hjd_jpeg_decode_batch(const uint8_t* const* datas, const size_t* sizes, int n, int16_t* const* coefs,
                          int64_t capacity_blocks, int nthreads, int32_t* status);

/* ---- streaming decode (host Huffman || H2D || kernel) ------------------- */
typedef struct hjd_stream hjd_stream;

/* nslots pinned staging slots of max_blocks coefficient blocks each (>= 2;
 * 3 = triple buffering); nthreads host Huffman workers (0 = hjd_host_cpu_share()
 * capped by the device's CPU slice, hjd_device_worker_cpus). */
int hjd_stream_create(hjd_ctx* ctx, int64_t max_blocks, int nslots, int nthreads, hjd_stream** out);
int hjd_stream_destroy(hjd_stream* s);

/* Queue one JPEG (the bytes must stay valid until hjd_stream_sync returns).
 * Its BGRX pixels are written to d_out (device memory, row pitch out_pitch
 * bytes) by the fused kernel once its coefficients reach the device. */
int hjd_stream_submit(hjd_stream* s, const uint8_t* data, size_t size, void* d_out, int32_t out_pitch);

/* Wait for every submitted image; returns the first error, if any.  stats (may
 * be NULL) receives {images, pixels, host_decode_ns, h2d_bytes, kernel_launches}. */
int hjd_stream_sync(hjd_stream* s, int64_t stats[5]);
/* Cumulative GPU-side busy time of the stream's jobs, complete as of the last
 * hjd_stream_sync: the sum of every upload's duration on the copy stream and
 * of every fused-kernel launch on the compute stream (HIP timing events).
 * Divided by a wall-clock interval it is the fraction of the time the host
 * Huffman workers kept the copy engine / the kernel fed. */
int hjd_stream_busy(hjd_stream* s, int64_t* h2d_busy_ns, int64_t* kernel_busy_ns);

/* Host CPUs of one GPU's worker pool (both stream kinds bind their workers to
 * them; HJD_NUMA=0 disables the binding): the GPUs on the same NUMA node, in
 * PCI bus-id order, split that node's CPUs into equal contiguous slices; with
 * fewer CPUs than GPUs they share the node.  This hook computes the split for
 * GPU `bus` among `gpus` from a sysfs tree at `sysfs_root` ("" or NULL: the
 * real one; a test passes a fake topology), optionally intersected with this
 * process's affinity.  Writes up to `capacity` CPU ids; *ncpus = how many
 * (0: unknown topology, no binding). */
int hjd_debug_worker_cpus(const char* sysfs_root, const char* bus, const char* const* gpus, int ngpus,
                          int only_allowed, int32_t* cpus, int capacity, int32_t* ncpus);
/* Pixel format of subsequent submits: HJD_OUT_BGRX (default) or HJD_OUT_BGR24
 * (d_out 4-byte aligned, pitch >= 3*width); jobs already queued keep theirs. */
int hjd_stream_set_output_format(hjd_stream* s, int out_format);

/* ---- GPU entropy decoding ----------------------
 * Replaces the single-threaded scan decode of the reference
 * (src/decoder.cpp:221-365) with a parallel one on the GPU.  The host only
 * parses headers and copies each scan into pinned memory without byte
 * stuffing / RST markers (memcpy speed); the Huffman decode runs on the GPU as
 * a self-synchronising parallel decode verified from the frame start, so its
 * coefficients are identical to hjd_jpeg_decode_coefs on every valid file
 * (DESIGN.md s10).  The fused pixel kernel follows on the same stream. */
typedef struct hjd_gdec hjd_gdec;

/* Capacity: max_frames JPEGs per call whose coefficient blocks total at most
 * max_blocks.  max_scan_bytes = the total size of the files of a call (the
 * sum of sizes[]) is always enough, wherever the files lie in memory.  The
 * sum of their entropy-coded bytes is enough too: pinned files then take the
 * host destuff path where their raw scans (stuffing, restart markers and the
 * bytes after EOI included) would not fit, unless HJD_DESTUFF=device, which
 * reports the overflow.
 * sub_bits = bits per parallel subsequence (0 = default 1024; >= 32). */
int hjd_gdec_create(hjd_ctx* ctx, int max_frames, int64_t max_scan_bytes, int64_t max_blocks, int sub_bits,
                    hjd_gdec** out);
int hjd_gdec_destroy(hjd_gdec* g);

/* Decode n JPEGs to BGRX in device memory (d_outs[i], row pitch pitches[i];
 * 16-byte aligned).  Asynchronous on `stream` (hipStream_t, NULL = default);
 * the input bytes may be reused as soon as the call returns (for pinned input,
 * which the DMA reads in place, the call returns once those uploads have
 * landed; the kernels stay asynchronous).  A later call on
 * the same object waits (on the host) for this call's uploads and is ordered
 * (on the device) after its kernels, whatever stream it uses; hjd_gdec_sync
 * reports the statuses of the most recent call. */
int hjd_gdec_decode(hjd_gdec* g, const uint8_t* const* datas, const size_t* sizes, int n, void* const* d_outs,
                    const int32_t* pitches, void* stream);

/* Entropy decode only: int16 quantised zigzag coefficients (the HJD_IN_Q16_ZIGZAG
 * layout), frame i at block block_offsets[i] of d_coefs (16-byte aligned). */
int hjd_gdec_decode_coefs(hjd_gdec* g, const uint8_t* const* datas, const size_t* sizes, int n, int16_t* d_coefs,
                          int64_t* block_offsets, void* stream);

/* Wait for the last call.  status[i] (may be NULL): 0 = ok, else
 * HJD_GDEC_CORRUPT / HJD_GDEC_COUNT bits (HJD_GDEC_SEQUENTIAL is informational).
 * Returns HJD_E_INVALID if any frame's entropy data was corrupt. */
int hjd_gdec_sync(hjd_gdec* g, int32_t* status);

/* Pixel format of the following hjd_gdec_decode calls: HJD_OUT_BGRX (default)
 * or HJD_OUT_BGR24 (include/hjd.h; 3-byte pixels, d_outs 4-byte aligned,
 * pitches >= 3*width, multiple of 4). */
int hjd_gdec_set_output_format(hjd_gdec* g, int out_format);
/* Bytes of the most recent decode call: scan bytes the host CPU read + wrote
 * (0 when every scan was destuffed on the GPU) and bytes moved host -> device. */
int hjd_gdec_last_bytes(hjd_gdec* g, int64_t* host_scan_bytes, int64_t* h2d_bytes);

#define HJD_GDEC_SEQUENTIAL 1   /* verification needed the sequential path (round-based sync) or a
                                   serial chain repair (speculative sync: the decoder then moves its
                                   next calls to a longer lead-in) */
#define HJD_GDEC_CORRUPT 2      /* invalid Huffman data on the decoded chain */
#define HJD_GDEC_COUNT 4        /* fewer blocks than the frame needs */

/* ---- GPU-entropy stream: JPEG bytes in, BGRX in HBM out -----------------
 * Like hjd_stream, but the Huffman decode runs on the GPU: worker threads only
 * parse + destuff each JPEG into the pinned staging of the open batch (up to
 * max_frames JPEGs / max_scan_bytes / max_blocks per batch); nslots (2..16)
 * batches rotate on their own HIP streams so uploads overlap kernels. */
typedef struct hjd_gstream hjd_gstream;
int hjd_gstream_create(hjd_ctx* ctx, int max_frames, int64_t max_scan_bytes, int64_t max_blocks, int nslots,
                       int nthreads, hjd_gstream** out);
int hjd_gstream_destroy(hjd_gstream* s);
/* Queue one JPEG (bytes valid until hjd_gstream_sync returns); pixels go to
 * d_out (device, row pitch out_pitch bytes, 16-byte aligned).  submit and sync
 * may be called from several threads (they are serialised internally). */
int hjd_gstream_submit(hjd_gstream* s, const uint8_t* data, size_t size, void* d_out, int32_t out_pitch);
/* D2H sink (SURVEY.md s8(e) "D2H-on", s8(f) rank 4): same, but the pixels are
 * copied back into host memory h_out (row pitch out_pitch bytes; pinned memory
 * keeps the copy asynchronous) once the frame is decoded. */
int hjd_gstream_submit_host(hjd_gstream* s, const uint8_t* data, size_t size, void* h_out, int32_t out_pitch);
/* Flush and wait; returns the first error.  stats (may be NULL):
 * {images, pixels, host_prep_ns, h2d_bytes, batches}. */
int hjd_gstream_sync(hjd_gstream* s, int64_t stats[5]);
/* Pixel format of the stream's outputs (device and host sinks alike):
 * HJD_OUT_BGRX (default) or HJD_OUT_BGR24; with BGR24 the D2H sink moves
 * 3 bytes per pixel.  Only between hjd_gstream_sync and the next submit
 * (HJD_E_STATE otherwise). */
int hjd_gstream_set_output_format(hjd_gstream* s, int out_format);
/* Scan bytes the host CPU has read + written so far (destuffing into pinned
 * staging: 2 per scan byte; a frame whose bytes are pinned host memory is
 * destuffed on the GPU and costs 0: only its header is parsed on the host). */
int hjd_gstream_host_bytes(hjd_gstream* s, int64_t* host_scan_bytes);

/* Pin (page-lock) a caller's host range so the GPU can DMA from it: JPEG bytes
 * in pinned memory (this, or hipHostMalloc) reach the device raw and are
 * destuffed there (HJD_DESTUFF=auto, the default; "host" / "device" force one
 * path).  The range must stay registered while frames submitted from it are in
 * flight (until hjd_gstream_sync / hjd_gdec_sync). */
int hjd_host_register(void* ptr, size_t size);
/* Host-side stream preparation alone, no GPU (measurement hook for the
 * multi-GPU host ceiling, one call = one per-GPU pool): nthreads threads on
 * NUMA node `node` (-1: unbound) prepare `frames` JPEGs read in order from an
 * arena of arena_bytes (datas replicated) into a staging ring of ring_bytes.
 * mode 0 host destuff, 1 header + tables only (the GPU-destuff path), 2 plain
 * memcpy of each file.  Calls sharing `barrier` (parties > 1) start their timed
 * phase together.  out: wall ns, summed thread CPU ns, JPEG bytes, frames. */
int hjd_debug_host_prep(const uint8_t* const* datas, const size_t* sizes, int n, int mode, int nthreads, int node,
                        int64_t frames, int64_t arena_bytes, int64_t ring_bytes, int32_t* barrier, int parties,
                        int64_t out[4]);
int hjd_host_unregister(void* ptr);

/* The 54-byte header of the reference's output BMP (src/decoder.cpp:372-394):
 * 32 bpp, top-down; the file is this header followed by the W*H*4 BGRX bytes. */
int hjd_bmp_header(int32_t width, int32_t height, uint8_t header[54]);
/* The 24-bpp counterpart (SURVEY.md s8(f) rank 4 "RGB24 writer"): top-down,
 * rows padded to 4 bytes; the file is this header followed by the rows of an
 * HJD_OUT_BGR24 image at pitch (3*W+3)&~3. */
int hjd_bmp_header_bgr24(int32_t width, int32_t height, uint8_t header[54]);

/* Test hook: the reader of the host decoder's single-scan files, process-wide.
 * 0 (default) the de-stuffed reader wherever the scan admits it, 1 the
 * byte-wise reader always (the cross-check); -1 queries.  Returns the previous
 * mode. */
int hjd_debug_host_reader(int mode);
/* Test hook (no GPU): runs the same parallel algorithm on the host, one frame,
 * and writes its coefficients.  Not a decode path. */
/* Destuff step alone (test hooks): the host routine, and the device kernels on
 * one raw scan of n bytes with nseg restart intervals expected (out: >= n+64
 * bytes; status: kStatusCorrupt bit 2 for malformed scans). */
int hjd_debug_destuff_host(const uint8_t* scan, size_t n, uint8_t* out, size_t cap, uint32_t* seg_end, int max_seg,
                           int* nseg, int64_t* out_bytes);
int hjd_debug_destuff_gpu(hjd_ctx* ctx, const uint8_t* scan, size_t n, int nseg, uint8_t* out, size_t cap,
                          uint32_t* seg_end, int64_t* out_bytes, uint32_t* status);
int hjd_debug_entropy_emulate(const uint8_t* data, size_t size, int sub_bits, int16_t* coefs, int64_t capacity_blocks,
                              int32_t* status);
/* Test hook (no GPU): the sync kernels' step decode (AC step tables, several
 * units per lookup) against the unit-by-unit decode, from guessed and true
 * entries of the first scan; *runs compared, *mismatches in exit state or
 * statistics. */
int hjd_debug_entropy_sync_check(const uint8_t* data, size_t size, int sub_bits, int64_t* runs, int64_t* mismatches);

#ifdef __cplusplus
}
#endif
#endif
