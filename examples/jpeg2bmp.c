/*
 * jpeg2bmp.c -- the C ABI end to end, no Python: JPEG files -> BMP files on
 * GPU 0.  The Huffman decode runs on the GPU (hjd_gdec, include/hjd_host.h),
 * then the fused dequant + IDCT + colour kernel writes BGRX into device
 * memory, which is copied back and written as the reference program's 32-bpp
 * BMP (src/decoder.cpp:372-395).  Sequential files, with one scan or several,
 * take the GPU entropy decoder; progressive files, which it does not take, go
 * through the host Huffman decoder and a plan.
 *
 *   make -C examples && examples/jpeg2bmp out_dir a.jpg [b.jpg ...]
 */
#include <hip/hip_runtime_api.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hjd.h"
#include "hjd_host.h"

#define CHECK(call)                                                                 \
    do {                                                                            \
        int rc_ = (call);                                                           \
        if (rc_ != HJD_OK) {                                                        \
            fprintf(stderr, "%s failed (%d): %s\n", #call, rc_, hjd_last_error());  \
            return 1;                                                               \
        }                                                                           \
    } while (0)

#define HIP_CHECK(call)                                                             \
    do {                                                                            \
        hipError_t e_ = (call);                                                     \
        if (e_ != hipSuccess) {                                                     \
            fprintf(stderr, "%s failed: %s\n", #call, hipGetErrorString(e_));       \
            return 1;                                                               \
        }                                                                           \
    } while (0)

static uint8_t* read_file(const char* path, size_t* size)
{
    FILE* f = fopen(path, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    uint8_t* buf = (uint8_t*)malloc(n > 0 ? (size_t)n : 1);
    if (buf && fread(buf, 1, (size_t)n, f) != (size_t)n) {
        free(buf);
        buf = NULL;
    }
    fclose(f);
    *size = (size_t)n;
    return buf;
}

/* Host Huffman + the fused kernel through a one-frame plan. */
static int decode_host_path(hjd_ctx* ctx, const uint8_t* data, size_t size, const hjd_jpeg_info* info,
                            void* d_out, int32_t pitch)
{
    int16_t* coefs = (int16_t*)malloc((size_t)info->nblocks * 64 * sizeof(int16_t));
    hjd_jpeg_info full;
    void* d_coefs = NULL;
    hjd_plan* plan = NULL;
    if (!coefs) return 1;
    CHECK(hjd_jpeg_decode_coefs(data, size, &full, coefs, info->nblocks));
    HIP_CHECK(hipMalloc(&d_coefs, (size_t)full.nblocks * 128));
    HIP_CHECK(hipMemcpy(d_coefs, coefs, (size_t)full.nblocks * 128, hipMemcpyHostToDevice));
    hjd_frame fr;
    memset(&fr, 0, sizeof(fr));
    fr.width = full.width;
    fr.height = full.height;
    fr.sampling = full.sampling;
    fr.out_pitch = pitch;
    fr.qt_index[0] = 0;
    fr.qt_index[1] = 1;
    fr.qt_index[2] = 2;
    CHECK(hjd_plan_create(ctx, &fr, 1, HJD_IN_Q16_ZIGZAG, &full.qt[0][0], 3, &plan));
    CHECK(hjd_plan_launch(plan, d_coefs, d_out, NULL, 0));
    HIP_CHECK(hipDeviceSynchronize());
    CHECK(hjd_plan_destroy(plan));
    HIP_CHECK(hipFree(d_coefs));
    free(coefs);
    return 0;
}

int main(int argc, char** argv)
{
    if (argc < 3) {
        fprintf(stderr, "usage: %s out_dir file.jpg...\n", argv[0]);
        return 2;
    }
    hjd_ctx* ctx = NULL;
    CHECK(hjd_ctx_create(0, &ctx));
    for (int a = 2; a < argc; ++a) {
        size_t size = 0;
        uint8_t* data = read_file(argv[a], &size);
        if (!data) {
            fprintf(stderr, "cannot read %s\n", argv[a]);
            return 1;
        }
        hjd_jpeg_info info;
        CHECK(hjd_jpeg_parse(data, size, &info));
        const int32_t pitch = info.width * 4;
        const size_t bytes = (size_t)pitch * (size_t)info.height;
        void* d_out = NULL;
        HIP_CHECK(hipMalloc(&d_out, bytes));
        if (info.process != 2) {   /* sequential (one scan or several): GPU Huffman decode + fused kernel */
            hjd_gdec* gd = NULL;
            CHECK(hjd_gdec_create(ctx, 1, (int64_t)size, info.nblocks, 0, &gd));
            const uint8_t* datas[1] = {data};
            const size_t sizes[1] = {size};
            void* outs[1] = {d_out};
            const int32_t pitches[1] = {pitch};
            int32_t status = 0;
            CHECK(hjd_gdec_decode(gd, datas, sizes, 1, outs, pitches, NULL));
            CHECK(hjd_gdec_sync(gd, &status));
            CHECK(hjd_gdec_destroy(gd));
        } else if (decode_host_path(ctx, data, size, &info, d_out, pitch)) {
            return 1;
        }
        uint8_t* px = (uint8_t*)malloc(bytes);
        HIP_CHECK(hipMemcpy(px, d_out, bytes, hipMemcpyDeviceToHost));
        uint8_t header[54];
        CHECK(hjd_bmp_header(info.width, info.height, header));
        const char* base = strrchr(argv[a], '/');
        base = base ? base + 1 : argv[a];
        char path[4096];
        snprintf(path, sizeof(path), "%s/%s.bmp", argv[1], base);
        FILE* f = fopen(path, "wb");
        if (!f || fwrite(header, 1, 54, f) != 54 || fwrite(px, 1, bytes, f) != bytes) {
            fprintf(stderr, "cannot write %s\n", path);
            return 1;
        }
        fclose(f);
        printf("%s: %dx%d sampling %d process %d scans %s -> %s (%s Huffman)\n", argv[a], info.width, info.height,
               info.sampling, info.process, info.single_scan ? "1" : "several", path,
               info.process != 2 ? "GPU" : "host");
        free(px);
        HIP_CHECK(hipFree(d_out));
        free(data);
    }
    CHECK(hjd_ctx_destroy(ctx));
    return 0;
}
