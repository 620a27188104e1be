/*
 * oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Plain-C restatement of the reference CPU pixel path:
 *   zigzag + dequant ........ src/decoder.cpp:338-342, src/zigzag.h:15-40
 *   8x8 integer IDCT ........ src/cpuIDCT8x8.cpp:13-127 (Chen-Wang, MPEG-2 ref style)
 *   MCU pixel assembly ...... src/decoder.cpp:443-491 (4:4:4 :457-471, 4:2:0 :474-483)
 *   colour conversion ....... src/decoder.cpp:367-370 (fp64, truncation toward 0)
 *   clamp / pack ............ src/macro.h:121-126 (clamp255), :141-145 (RGBClamp32)
 * Written from the reference's behaviour, not copied; pinned by tests/test_oracle.py.
 */
#include "oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

const int32_t oracle_zigzag[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* butterfly constants: round(2048*sqrt(2)*cos(k*pi/16)), cpuIDCT8x8.cpp:6-11 */
enum { C1 = 2841, C2 = 2676, C3 = 2408, C5 = 1609, C6 = 1108, C7 = 565 };

/* iclp[] of cpuIDCT8x8.cpp:13-23: clamp to [-256,255]; callers stay in [-512,511] */
static inline int32_t clip_sample(int32_t v) { return v < -256 ? -256 : (v > 255 ? 255 : v); }

/*
 * One 8-point pass.  `s` is the element stride (1 = row, 8 = column).
 * Row pass (cpuIDCT8x8.cpp:36-80): inputs scaled <<11 (DC gets +128 for the
 * final rounding), no stage-1/2 pre-shift, outputs >>8.
 * Column pass (cpuIDCT8x8.cpp:82-127): inputs scaled <<8 (DC +8192),
 * stage-1/2 products rounded with (+4)>>3, outputs >>14 then clipped.
 * The reference's all-AC-zero short-cuts (:40-45, :86-92) produce the same
 * values as the full butterfly on the legal domain; they are kept here so the
 * restatement mirrors the reference's control flow exactly.
 */
static void pass8(int32_t* p, int s, int col)
{
    int32_t b0 = p[0], b1 = p[s], b2 = p[2 * s], b3 = p[3 * s];
    int32_t b4 = p[4 * s], b5 = p[5 * s], b6 = p[6 * s], b7 = p[7 * s];
    int i;

    if (!(b1 | b2 | b3 | b4 | b5 | b6 | b7)) {
        int32_t dc = col ? clip_sample((b0 + 32) >> 6) : (b0 << 3);
        for (i = 0; i < 8; i++) p[i * s] = dc;
        return;
    }

    const int sh_in = col ? 8 : 11;
    const int32_t rnd = col ? 4 : 0;
    int32_t e0 = (b0 << sh_in) + (col ? 8192 : 128);
    int32_t e1 = b4 << sh_in;

    /* odd part, stage 1 */
    int32_t t = C7 * (b1 + b7) + rnd;
    int32_t o4 = t + (C1 - C7) * b1;
    int32_t o5 = t - (C1 + C7) * b7;
    t = C3 * (b5 + b3) + rnd;
    int32_t o6 = t - (C3 - C5) * b5;
    int32_t o7 = t - (C3 + C5) * b3;
    if (col) { o4 >>= 3; o5 >>= 3; o6 >>= 3; o7 >>= 3; }

    /* even part, stage 2 */
    int32_t e8 = e0 + e1;
    e0 -= e1;
    t = C6 * (b2 + b6) + rnd;
    int32_t e2 = t - (C2 + C6) * b6;
    int32_t e3 = t + (C2 - C6) * b2;
    if (col) { e2 >>= 3; e3 >>= 3; }
    int32_t a1 = o4 + o6;
    int32_t a4 = o4 - o6;
    int32_t a6 = o5 + o7;
    int32_t a5 = o5 - o7;

    /* stage 3 */
    int32_t f7 = e8 + e3;
    int32_t f8 = e8 - e3;
    int32_t f3 = e0 + e2;
    int32_t f0 = e0 - e2;
    int32_t g2 = (181 * (a4 + a5) + 128) >> 8;
    int32_t g4 = (181 * (a4 - a5) + 128) >> 8;

    /* stage 4 */
    int32_t r[8] = {f7 + a1, f3 + g2, f0 + g4, f8 + a6, f8 - a6, f0 - g4, f3 - g2, f7 - a1};
    if (col) {
        for (i = 0; i < 8; i++) p[i * s] = clip_sample(r[i] >> 14);
    } else {
        for (i = 0; i < 8; i++) p[i * s] = r[i] >> 8;
    }
}

void oracle_fast_idct(int32_t blk[64])
{
    int i;
    for (i = 0; i < 8; i++) pass8(blk + 8 * i, 1, 0);
    for (i = 0; i < 8; i++) pass8(blk + i, 8, 1);
}

void oracle_dequant_block(const int16_t coef_zz[64], const int32_t qt_zz[64], int32_t out_nat[64])
{
    int k;
    for (k = 0; k < 64; k++) out_nat[oracle_zigzag[k]] = (int32_t)coef_zz[k] * qt_zz[k];
}

static inline uint32_t clamp_u8(int32_t n) { return n < 0 ? 0u : (n > 255 ? 255u : (uint32_t)n); }

uint32_t oracle_yuv_to_bgrx(int32_t y, int32_t u, int32_t v)
{
    /* C semantics of decoder.cpp:369: int -> double, left-to-right, (int) truncates */
    const double Y = (double)y, U = (double)u, V = (double)v;
    const int32_t r = (int32_t)(Y + 1.402 * V + 128);
    const int32_t g = (int32_t)(Y - 0.34414 * U - 0.71414 * V + 128);
    const int32_t b = (int32_t)(Y + 1.772 * U + 128);
    return (clamp_u8(r) << 16) | (clamp_u8(g) << 8) | clamp_u8(b);
}

void oracle_yuv_to_bgrx_n(const int32_t* y, const int32_t* u, const int32_t* v, uint32_t* out, int64_t n)
{
    int64_t i;
    for (i = 0; i < n; i++) out[i] = oracle_yuv_to_bgrx(y[i], u[i], v[i]);
}

void oracle_idct_blocks(const int32_t* in, int32_t* out, int64_t nblocks)
{
    int64_t b;
    for (b = 0; b < nblocks; b++) {
        memcpy(out + 64 * b, in + 64 * b, 64 * sizeof(int32_t));
        oracle_fast_idct(out + 64 * b);
    }
}

/* One MCU of already-IDCT'd blocks -> pixels (decoder.cpp:454-484). */
static void put_mcu(const int32_t (*m)[64], int sampling, int mx, int my, int width, int height,
                    uint32_t* out, int pitch)
{
    int x, y;
    if (sampling == ORACLE_YUV444) {
        for (y = 0; y < 8; y++) {
            int py = my * 8 + y;
            if (py >= height) break;
            for (x = 0; x < 8; x++) {
                int px = mx * 8 + x;
                if (px >= width) break;
                int pos = y * 8 + x;
                out[(int64_t)py * pitch + px] = oracle_yuv_to_bgrx(m[0][pos], m[1][pos], m[2][pos]);
            }
        }
    } else if (sampling == ORACLE_YUV422) {
        /* extension (the reference rejects H2V1): nearest horizontal chroma
         * replication, the 4:2:0 rule of decoder.cpp:474-483 in x only */
        for (y = 0; y < 8; y++) {
            int py = my * 8 + y;
            if (py >= height) break;
            for (x = 0; x < 16; x++) {
                int px = mx * 16 + x;
                if (px >= width) break;
                int Y = m[x >> 3][(y << 3) | (x & 7)];
                int c = (y << 3) + (x >> 1);
                out[(int64_t)py * pitch + px] = oracle_yuv_to_bgrx(Y, m[2][c], m[3][c]);
            }
        }
    } else if (sampling == ORACLE_YUV411_H4V1) {
        /* extension: 32x8 MCU (Y0..Y3 side by side), one chroma sample per 4 px */
        for (y = 0; y < 8; y++) {
            int py = my * 8 + y;
            if (py >= height) break;
            for (x = 0; x < 32; x++) {
                int px = mx * 32 + x;
                if (px >= width) break;
                int Y = m[x >> 3][(y << 3) | (x & 7)];
                int c = (y << 3) + (x >> 2);
                out[(int64_t)py * pitch + px] = oracle_yuv_to_bgrx(Y, m[4][c], m[5][c]);
            }
        }
    } else if (sampling == ORACLE_YUV440) {
        /* extension: 8x16 MCU (Y0 above Y1), one chroma row per 2 pixel rows */
        for (y = 0; y < 16; y++) {
            int py = my * 16 + y;
            if (py >= height) break;
            for (x = 0; x < 8; x++) {
                int px = mx * 8 + x;
                if (px >= width) break;
                int Y = m[y >> 3][((y & 7) << 3) | x];
                int c = ((y >> 1) << 3) + x;
                out[(int64_t)py * pitch + px] = oracle_yuv_to_bgrx(Y, m[2][c], m[3][c]);
            }
        }
    } else if (sampling == ORACLE_GRAY) {
        /* extension: one component, the reference's conversion with U = V = 0 */
        for (y = 0; y < 8; y++) {
            int py = my * 8 + y;
            if (py >= height) break;
            for (x = 0; x < 8; x++) {
                int px = mx * 8 + x;
                if (px >= width) break;
                out[(int64_t)py * pitch + px] = oracle_yuv_to_bgrx(m[0][y * 8 + x], 0, 0);
            }
        }
    } else {
        for (y = 0; y < 16; y++) {
            int py = my * 16 + y;
            if (py >= height) break;
            for (x = 0; x < 16; x++) {
                int px = mx * 16 + x;
                if (px >= width) break;
                int Y = m[(y >> 3) * 2 + (x >> 3)][((y & 7) << 3) | (x & 7)];
                int c = ((y >> 1) << 3) + (x >> 1);
                out[(int64_t)py * pitch + px] = oracle_yuv_to_bgrx(Y, m[4][c], m[5][c]);
            }
        }
    }
}

static int frame_geometry(int width, int height, int sampling, int* mcw, int* mch, int* bpm, int* nluma)
{
    int mw, mh;
    if (width <= 0 || height <= 0) return -1;
    switch (sampling) {
    case ORACLE_YUV444: mw = 8; mh = 8; *bpm = 3; *nluma = 1; break;
    case ORACLE_YUV420: mw = 16; mh = 16; *bpm = 6; *nluma = 4; break;
    case ORACLE_YUV422: mw = 16; mh = 8; *bpm = 4; *nluma = 2; break;
    case ORACLE_GRAY: mw = 8; mh = 8; *bpm = 1; *nluma = 1; break;
    case ORACLE_YUV411_H4V1: mw = 32; mh = 8; *bpm = 6; *nluma = 4; break;
    case ORACLE_YUV440: mw = 8; mh = 16; *bpm = 4; *nluma = 2; break;
    default: return -1;
    }
    *mcw = (width - 1) / mw + 1; /* decoder.cpp:189-190 */
    *mch = (height - 1) / mh + 1;
    return 0;
}

int oracle_decode_frame_q16(const int16_t* coefs, const int32_t* qt_y, const int32_t* qt_cb,
                            const int32_t* qt_cr, int width, int height, int sampling,
                            uint32_t* out, int out_pitch_px)
{
    int mcw, mch, bpm, nluma, mx, my, b;
    if (frame_geometry(width, height, sampling, &mcw, &mch, &bpm, &nluma)) return -1;
    const int32_t* qt[6];
    for (b = 0; b < bpm; b++) qt[b] = b < nluma ? qt_y : (b == nluma ? qt_cb : qt_cr);
    int32_t m[6][64];
    const int16_t* src = coefs;
    for (my = 0; my < mch; my++) {
        for (mx = 0; mx < mcw; mx++) {
            for (b = 0; b < bpm; b++, src += 64) {
                oracle_dequant_block(src, qt[b], m[b]);
                oracle_fast_idct(m[b]);
            }
            put_mcu((const int32_t(*)[64])m, sampling, mx, my, width, height, out, out_pitch_px);
        }
    }
    return 0;
}

int oracle_decode_frame_i32(const int32_t* mcu_data, int width, int height, int sampling,
                            uint32_t* out, int out_pitch_px)
{
    int mcw, mch, bpm, nluma, mx, my, b;
    if (frame_geometry(width, height, sampling, &mcw, &mch, &bpm, &nluma)) return -1;
    int32_t m[6][64];
    const int32_t* src = mcu_data;
    for (my = 0; my < mch; my++) {
        for (mx = 0; mx < mcw; mx++) {
            for (b = 0; b < bpm; b++, src += 64) {
                memcpy(m[b], src, sizeof(m[b]));
                oracle_fast_idct(m[b]);
            }
            put_mcu((const int32_t(*)[64])m, sampling, mx, my, width, height, out, out_pitch_px);
        }
    }
    return 0;
}

/* ---- pthread pool for the CPU baseline: one frame per task ----
 * Frame f reads coefs + (f % ncoef_frames) * coef_stride; each worker writes
 * into its own output slot out + tid * out_stride (timing leg: the pixels of
 * frame f are not retained). */
typedef struct {
    const int16_t* coefs;
    int64_t coef_stride;
    int ncoef_frames;
    const int32_t *qy, *qcb, *qcr;
    int width, height, sampling;
    uint32_t* out;
    int64_t out_stride;
    int nframes;
    int next; /* guarded by mu */
    int err;
    pthread_mutex_t mu;
} batch_job;

typedef struct {
    batch_job* job;
    int tid;
} batch_worker_arg;

static void* batch_worker(void* arg)
{
    batch_worker_arg* a = (batch_worker_arg*)arg;
    batch_job* j = a->job;
    uint32_t* out = j->out + (int64_t)a->tid * j->out_stride;
    for (;;) {
        pthread_mutex_lock(&j->mu);
        int f = j->next++;
        pthread_mutex_unlock(&j->mu);
        if (f >= j->nframes) break;
        if (oracle_decode_frame_q16(j->coefs + (int64_t)(f % j->ncoef_frames) * j->coef_stride, j->qy, j->qcb,
                                    j->qcr, j->width, j->height, j->sampling, out, j->width))
            j->err = 1;
    }
    return NULL;
}

int oracle_decode_batch_q16_mt(const int16_t* coefs, int64_t coef_stride, int ncoef_frames, const int32_t* qt_y,
                               const int32_t* qt_cb, const int32_t* qt_cr, int width, int height,
                               int sampling, uint32_t* out, int64_t out_stride, int nframes,
                               int nthreads)
{
    batch_job j;
    int t;
    if (nthreads < 1) nthreads = 1;
    if (nthreads > 1024) nthreads = 1024;
    if (ncoef_frames < 1) ncoef_frames = 1;
    j.coefs = coefs; j.coef_stride = coef_stride; j.ncoef_frames = ncoef_frames;
    j.qy = qt_y; j.qcb = qt_cb; j.qcr = qt_cr;
    j.width = width; j.height = height; j.sampling = sampling;
    j.out = out; j.out_stride = out_stride;
    j.nframes = nframes; j.next = 0; j.err = 0;
    pthread_mutex_init(&j.mu, NULL);
    pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
    batch_worker_arg* args = (batch_worker_arg*)malloc(sizeof(batch_worker_arg) * (size_t)nthreads);
    if (!th || !args) { free(th); free(args); return -1; }
    for (t = 0; t < nthreads; t++) {
        args[t].job = &j;
        args[t].tid = t;
        pthread_create(&th[t], NULL, batch_worker, &args[t]);
    }
    for (t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
    free(th);
    free(args);
    pthread_mutex_destroy(&j.mu);
    return j.err ? -1 : 0;
}
