/*
 * hjd.h -- C ABI of the MI355X (gfx950) JPEG pixel back-end.
 *
 * Hot path (one fused HIP kernel): zigzag + dequant -> 8x8 integer IDCT ->
 * chroma upsample (nearest, 2x2) -> YCbCr->RGB (JFIF, truncating) -> BGRX store,
 * bit-exact to the reference CPU path (src/cpuIDCT8x8.cpp + src/decoder.cpp:367-491
 * of xinfushe/oclJPEGDecoder).  Plain C types only; every device pointer is a
 * HIP device address, every `stream` a hipStream_t (NULL = default stream).
 *
 * The reference's own entry points (src/idct.h:4-18) are provided with their
 * original C++ signatures by include/idct.h on top of this ABI.
 *
 * Errors: functions return HJD_OK (0) or a negative HJD_E_* code and never
 * throw; hjd_last_error() returns a description of the last failure on the
 * calling thread.
 */
#ifndef HJD_H
#define HJD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HJD_ABI_VERSION 1

enum hjd_status {
    HJD_OK = 0,
    HJD_E_INVALID = -1,   /* bad argument / unsupported geometry */
    HJD_E_NO_DEVICE = -2, /* no HIP device (or index out of range) */
    HJD_E_HIP = -3,       /* a HIP runtime call failed */
    HJD_E_NOMEM = -4,     /* host or device allocation failed */
    HJD_E_STATE = -5      /* call out of sequence (e.g. run before upload) */
};

/* Chroma sampling.  0..2 are numerically equal to the reference's ColorSpace
 * enum (src/macro.h:114-119: YUV444 = 0, YUV411 = 1 (really H2V2 4:2:0),
 * Other = 2).  HJD_YUV422 (Y H2V1, chroma H1V1) and HJD_GRAY (one component)
 * are extensions the reference rejects (src/decoder.cpp:58-69; SURVEY.md
 * s8(f) rank 4): the same IDCT and the same colour arithmetic with nearest
 * (horizontal) chroma replication, and R = G = B = clamp(Y + 128) for gray
 * (the reference's formula with U = V = 0).  HJD_YUV411_H4V1 (true 4:1:1:
 * Y H4V1, chroma H1V1; not the reference's "YUV411", which is H2V2) and
 * HJD_YUV440 (Y H1V2) are further extensions with nearest replication along
 * the subsampled axis. */
enum hjd_sampling {
    HJD_YUV444 = 0, HJD_YUV420 = 1, HJD_OTHER = 2, HJD_YUV422 = 3, HJD_GRAY = 4, HJD_YUV411_H4V1 = 5, HJD_YUV440 = 6
};

/* Output pixel format. */
enum hjd_out_format {
    /* 4 bytes per pixel: B, G, R, 0 (the reference's RGB32 buffer and its
     * 32-bpp BMP rows, src/decoder.cpp:367-395). */
    HJD_OUT_BGRX = 0,
    /* 3 bytes per pixel: B, G, R (a 24-bpp BMP row; extension, SURVEY.md
     * s8(f) rank 4).  Same values as BGRX without the pad byte; the kernel
     * writes 25 % fewer bytes. */
    HJD_OUT_BGR24 = 1
};

/* Kernel selection of a plan (hjd_plan_set_kernel).  Both kernels produce
 * identical pixels; AUTO takes the latency kernel (one workgroup per 48-block
 * task, six waves sharing it) for launches of few tasks -- a single frame --
 * and the persistent streaming kernel for batches. */
enum hjd_kernel_mode { HJD_KERNEL_AUTO = 0, HJD_KERNEL_PERSISTENT = 1, HJD_KERNEL_LATENCY = 2 };

/* Coefficient input format. */
enum hjd_input_format {
    /* int16 quantised coefficients in zigzag order, exactly as Huffman decoding
     * produces them (src/decoder.cpp:221-260); dequant + de-zigzag happen in
     * the kernel load (src/decoder.cpp:338-342). 128 B per block. */
    HJD_IN_Q16_ZIGZAG = 0,
    /* int32 dequantised coefficients in natural order: the reference's
     * jpg.mcu_data layout (src/jpeg.h:76) accepted by
     * clidct_transfer_data_to_device. 256 B per block. */
    HJD_IN_I32_NATURAL = 1
};

/*
 * One frame of a batch.  Blocks are MCU-major in raster MCU order; per MCU the
 * Y blocks in HxV raster order, then Cb, then Cr (src/decoder.cpp:286-344).
 * MCU grid: ceil(W/8)xceil(H/8) (4:4:4, 3 blocks; gray, 1 block),
 * ceil(W/16)xceil(H/16) (4:2:0, 6 blocks), ceil(W/16)xceil(H/8) (4:2:2,
 * 4 blocks), ceil(W/32)xceil(H/8) (4:1:1, 6 blocks) or ceil(W/8)xceil(H/16)
 * (4:4:0, 4 blocks).
 */
typedef struct hjd_frame {
    uint64_t coef_offset; /* first block's offset in the coef buffer, in BLOCKS */
    uint64_t out_offset;  /* byte offset of pixel (0,0) in the output buffer */
    int32_t width;        /* visible pixels (output is cropped to W x H) */
    int32_t height;
    int32_t out_pitch;    /* bytes per output row, >= 4*width (BGR24: 3*width), multiple of 4 */
    int32_t sampling;     /* enum hjd_sampling (not HJD_OTHER) */
    int32_t qt_index[3];  /* per component (Y, Cb, Cr): index into the qtable set */
    int32_t out_format;   /* HJD_OUT_BGRX (0) or HJD_OUT_BGR24; the same for all frames of a plan */
} hjd_frame;

typedef struct hjd_ctx hjd_ctx;
typedef struct hjd_plan hjd_plan;

/* ---- library / device ---- */
int hjd_abi_version(void);
const char* hjd_last_error(void);
int hjd_device_count(int* count);

/* Context = one device + one stream of work.  Not thread-safe; use one context
 * per host thread (or per GPU). */
int hjd_ctx_create(int device, hjd_ctx** out);
int hjd_ctx_destroy(hjd_ctx* ctx);
int hjd_ctx_device(const hjd_ctx* ctx);

/* ---- sizes ---- */
int hjd_frame_blocks(int width, int height, int sampling, int64_t* nblocks);

/*
 * Plan: validates a batch of frames, computes the work decomposition and
 * uploads the frame table and de-zigzagged quantisation tables to the device
 * (synchronously, outside any timed region).  qtables: nq tables of 64 values
 * each in FILE (zigzag) order, as DQT stores them (src/parser.cpp:65-89);
 * ignored (may be NULL) for HJD_IN_I32_NATURAL.
 */
int hjd_plan_create(hjd_ctx* ctx, const hjd_frame* frames, int nframes, int input_format,
                    const int32_t* qtables, int nq, hjd_plan** out);
int hjd_plan_destroy(hjd_plan* plan);
/* Tuning hook: kernel variant bits (0 = default).  bit 0: plain instead of
 * non-temporal output stores; bit 1: workgroup-interleaved task order.
 * Results are identical for every variant. */
int hjd_plan_set_variant(hjd_plan* plan, int variant);
int hjd_plan_set_kernel(hjd_plan* plan, int mode);   /* hjd_kernel_mode */
/* Pin the persistent kernel's task chunk without hjd_plan_autotune: exactly
 * `tasks` consecutive tasks per wave (1..4096, no occupancy floor; 0 restores
 * the shape default, which never drops below ~4 waves per SIMD).  Applies to
 * launches that take the persistent kernel: an HJD_KERNEL_AUTO plan small
 * enough for the latency kernel keeps it.  Identical pixels either way. */
int hjd_plan_set_chunk(hjd_plan* plan, int tasks);
int64_t hjd_plan_tasks(const hjd_plan* plan);      /* work items (strips) */
int64_t hjd_plan_pixels(const hjd_plan* plan);     /* visible pixels */
int64_t hjd_plan_coef_bytes(const hjd_plan* plan); /* algorithmic input bytes */

/*
 * Enqueue the fused decode of every frame of the plan on `stream` (async).
 * d_coefs: coefficient buffer (int16 or int32 per the plan's format);
 * d_out: output buffer (frames at their out_offset).  Both 16-byte aligned.
 * grid_blocks: grid size in 256-thread workgroups; 0 = default (short task
 * chunks per wave over many more groups than are resident, which keeps the
 * resident waves inside a narrow window of the batch).
 * The input is never modified (the reference kernel's in-place IDCT,
 * src/idct8x8.cl:136-155, is not reproduced).
 */
int hjd_plan_launch(hjd_plan* plan, const void* d_coefs, void* d_out, void* stream, int grid_blocks);

/*
 * Adapt the plan's launch to this device (synchronous, setup time): times
 * every candidate launch shape -- chunks of 1, 2, 4, 8 or 16 tasks per wave,
 * each with nt or plain output stores (BGRX) -- with the plan's own buffers,
 * `rounds`
 * interleaved rounds (0 = 2) of one warm and two timed launches each, and
 * keeps the fastest for the plan's later launches with grid_blocks = 0.
 * Every candidate writes identical pixels (d_out holds a valid decode on
 * return unless the choice came from the cache, below).  Plans the latency
 * kernel serves are left unchanged.  Optional
 * outputs: the chosen tasks per wave (0 = unchanged) and the variant bits.
 */
int hjd_plan_autotune(hjd_plan* plan, const void* d_coefs, void* d_out, void* stream, int rounds,
                      int32_t* tasks_per_wave, int32_t* variant);
/* hjd_plan_autotune's choice is cached per process (device x sampling x
 * input format x output format x the other variant bits x frame count x
 * task count):
 * a later plan of the same key takes it with no launch (and d_out is then NOT
 * written).  HJD_AUTOTUNE_CACHE=0 disables the cache; this empties it. */
int hjd_autotune_cache_clear(void);

/* The launch shape a plan's next hjd_plan_launch(grid_blocks = 0) uses. */
typedef struct hjd_launch_shape {
    int32_t kernel;             /* HJD_KERNEL_PERSISTENT or HJD_KERNEL_LATENCY */
    int32_t tasks_per_wave;     /* persistent: the chunk asked for (pinned, tuned or the shape default) */
    int32_t max_tasks_per_wave; /* persistent: the most tasks one wave takes with that grid */
    int32_t grid;               /* workgroups (latency: one per task) */
    int32_t variant;            /* variant bits */
    int32_t autotune_launches;  /* kernel launches the last hjd_plan_autotune made (0: none or cached) */
    int32_t autotune_cached;    /* 1: the last hjd_plan_autotune reused a cached choice */
} hjd_launch_shape;
int hjd_plan_launch_shape(const hjd_plan* plan, hjd_launch_shape* out);

/* IDCT only (the reference's batch_idct, src/idct8x8.cl:157-166), out of
 * place: int32 natural-order dequantised blocks -> int32 samples [-256,255]. */
int hjd_idct_blocks(hjd_ctx* ctx, const int32_t* d_in, int32_t* d_out, int64_t nblocks, void* stream);

/* The idct.h shim (include/idct.h) keeps its context, stream, grow-only device
 * buffers, plan cache and pinned staging alive across images: the reference
 * caller's clidct_clean_up (src/decoder.cpp:518-521) ends one image only.
 * This frees all of it (HJD_COMPAT_TEARDOWN=1 does so after every image, as
 * src/oclDCT8x8.cpp:316-341 did). */
int hjd_compat_release(void);

/* ---- test / measurement hooks (same device code as the fused kernel) ---- */
/* Colour stage alone over n (Y,U,V) triples: out[i] = BGRX.  mode 0 = the
 * kernel's exact-integer formulation, 1 = literal fp64 formulation. */
int hjd_debug_csc(hjd_ctx* ctx, const int32_t* d_y, const int32_t* d_u, const int32_t* d_v,
                  uint32_t* d_out, int64_t n, int mode, void* stream);
/* Exhaustive colour check: evaluates every (Y,U,V) in [-256,255]^3 on the
 * device and writes the 2^27 BGRX words to d_out (512 MiB). */
int hjd_debug_csc_exhaustive(hjd_ctx* ctx, uint32_t* d_out, int mode, void* stream);

/* Same-run measurement of the fused kernel's stages (bench.py): launch the
 * plan's persistent kernel with stages skipped.  Outputs are WRONG by design
 * (timing only).  stages: 80 = memory only (coefficient loads, staging, LDS
 * reads and BGRX stores kept; no IDCT, no colour math), 4 = no stores,
 * 16 = no IDCT, 64 = no colour math, 20 = no IDCT and no stores, 8 = no colour
 * stage, 24 = neither IDCT nor colour stage, 256 = every lane gathers row 0
 * of its block (the product's instructions without the zigzag gather's LDS
 * bank conflicts).  4:2:0 / 4:4:4, int16 zigzag
 * input, BGRX output only.  grid_blocks as hjd_plan_launch (0 = the plan's launch shape,
 * hjd_plan_autotune's if it ran). */
int hjd_debug_plan_launch_stages(hjd_plan* plan, int stages, const void* d_coefs, void* d_out, void* stream,
                                 int grid_blocks);

/* The box's streaming ceiling for a read:write byte mix (bench.py's
 * frac_of_box_ceiling): units of read_kib KiB read + write_kib KiB written
 * (16 B per lane, coalesced), units_per_wave consecutive units per wave, one
 * launch over min(src_bytes / read_kib KiB, dst_bytes / write_kib KiB) units.
 * flags bit 0: non-temporal loads and stores; bit 1: XCD-contiguous group
 * order (the fused kernel's); bit 2: pipelined (the next unit's loads issued
 * before this unit's stores, as the fused kernel prefetches its next task);
 * bit 3: image-row stores (the fused kernel's store geometry: dst as 3840-px
 * BGRX rows, pitch 15360 B, each unit one 512-B-wide strip of 2*write_kib
 * rows, two row segments per wave store instruction).  Mixes (KiB): 6:8 (4:2:0 task), 6:4 (4:4:4
 * task), 0:8, 6:0, 4:4, 3:4.  *units_out = units moved (bytes = units *
 * (read_kib + write_kib) KiB).  dst_bytes >= 1 KiB. */
int hjd_debug_rw_mix(hjd_ctx* ctx, const void* d_src, void* d_dst, int64_t src_bytes, int64_t dst_bytes,
                     int read_kib, int write_kib, int units_per_wave, int flags, void* stream, int64_t* units_out);

/* Clock probe: one wave on `stream` samples the shader clock counter and the
 * 100-MHz real-time counter every interval_ticks (>= 100) real-time ticks,
 * nsamples times: d_out[2i] = real-time ticks, d_out[2i+1] = shader cycles
 * (2 * nsamples uint64 words).  Launched beside a kernel on another stream,
 * consecutive samples give the clock the chip holds under that load
 * (delta cycles / delta ticks * 100 MHz).  Ends after nsamples intervals. */
int hjd_debug_clock_probe(hjd_ctx* ctx, uint64_t* d_out, int nsamples, int interval_ticks, void* stream);

/* The 4:4:4 kernels' d16 gather (ds_read_u16_d16_hi) is valid only where that
 * load zeroes the low half of its destination.  *probe_zeroes: the one-wave
 * hardware probe's answer for `device` (hjd_ctx_create runs it; a completed
 * run is cached per device, a failed one reads 0 and is retried; HJD_D16_PROBE=
 * fail forces 0); *selected: whether the 4:4:4 launches take the d16 kernels
 * (the cached probe passed, and HJD_D16 is not 0). */
int hjd_debug_d16_gather(int device, int* probe_zeroes, int* selected);

#ifdef __cplusplus
}
#endif
#endif
