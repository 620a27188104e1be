// idct_compat.hip -- the reference's src/idct.h entry points on the MI355X back-end.
//
// Host-side replacement for src/oclDCT8x8.cpp (OpenCL runtime, file-static state,
// one image at a time) with identical C++ signatures (include/idct.h).  The GPU
// functions drive the C ABI of hjd.h: one context + stream, an int32
// natural-order block buffer (the jpg.mcu_data layout the reference uploads,
// src/decoder.cpp:356), a cropped BGRX image, and a one-frame plan of the fused
// kernel (HJD_IN_I32_NATURAL).  Messages go to stderr and failures return
// false, as in the reference.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

#include "hjd.h"
#include "hjd_device.hpp"
#include "idct.h"

namespace {

int g_device = -1;                 // selected by Initialize_OpenCL_IDCT
hjd_ctx* g_ctx = nullptr;
hipStream_t g_stream = nullptr;
int32_t* g_blocks = nullptr;       // int32 [total_blocks][64], natural order, dequantised
int32_t* g_idct = nullptr;         // IDCT'd blocks (lazily, for retrieve_data)
uint32_t* g_image = nullptr;       // BGRX, W x H, pitch W*4
hjd_plan* g_plan = nullptr;
int g_total_blocks = 0;
size_t g_width = 0, g_height = 0;
int g_mcu_w = 0, g_mcu_h = 0;
int g_built = -1;                  // colour space of the built plan
bool g_idct_valid = false;

bool report(const char* what)
{
    fprintf(stderr, "%s failed (%s)\n", what, hjd_last_error());
    return false;
}

bool hip_ok(hipError_t e, const char* what)
{
    if (e == hipSuccess) return true;
    fprintf(stderr, "%s failed (%s)\n", what, hipGetErrorString(e));
    return false;
}

}  // namespace

// ---- CPU back-end (src/cpuIDCT8x8.cpp API; same butterfly as the kernel) ----
void Initialize_Fast_IDCT() {}   // no clip table needed: the clamp is arithmetic

void idctrow(int* blk)
{
    int v[8];
    for (int i = 0; i < 8; ++i) v[i] = blk[i];
    hjd::idct8<false>(v);
    for (int i = 0; i < 8; ++i) blk[i] = v[i];
}

void idctcol(int* blk)
{
    int v[8];
    for (int i = 0; i < 8; ++i) v[i] = blk[8 * i];
    hjd::idct8<true>(v);
    for (int i = 0; i < 8; ++i) blk[8 * i] = v[i];
}

void Fast_IDCT(int* block)
{
    for (int i = 0; i < 8; ++i) idctrow(block + 8 * i);
    for (int i = 0; i < 8; ++i) idctcol(block + i);
}

// ---- GPU back-end (src/oclDCT8x8.cpp API) ----------------------------------
int Initialize_OpenCL_IDCT()
{
    puts("[ ] Initializing HIP environment");
    int n = 0;
    if (hjd_device_count(&n) != HJD_OK) {
        report("hjd_device_count");
        return -1;
    }
    for (int i = 0; i < n; ++i) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, i) == hipSuccess)
            printf("Device #%d: Name: %s (%s), Compute Units: %d, Local Memory Size: %zu\n", i + 1, prop.name,
                   prop.gcnArchName, prop.multiProcessorCount, static_cast<size_t>(prop.sharedMemPerBlock));
    }
    if (n > 0) {
        g_device = 0;
        printf("[ ] HIP device selected.\n");
        return 0;
    }
    printf("[X] No HIP device.\n");
    return 1;
}

bool clidct_create()
{
    if (g_device < 0 && Initialize_OpenCL_IDCT() != 0) return false;
    if (g_ctx) return true;
    if (hjd_ctx_create(g_device, &g_ctx) != HJD_OK) return report("hjd_ctx_create");
    if (!hip_ok(hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking), "hipStreamCreate")) return false;
    return true;
}

bool clidct_allocate_memory(const int total_blocks, const size_t image_width, const size_t image_height,
                            const int mcu_width, const int mcu_height)
{
    if (!g_ctx) {
        fprintf(stderr, "clidct_allocate_memory: no context (call clidct_create first)\n");
        return false;
    }
    if (total_blocks <= 0 || image_width == 0 || image_height == 0) {
        fprintf(stderr, "clidct_allocate_memory: invalid arguments\n");
        return false;
    }
    (void)hipFree(g_blocks); (void)hipFree(g_idct); (void)hipFree(g_image);
    g_blocks = nullptr; g_idct = nullptr; g_image = nullptr;
    if (!hip_ok(hipMalloc(&g_blocks, static_cast<size_t>(total_blocks) * 64 * sizeof(int32_t)), "hipMalloc(blocks)"))
        return false;
    if (!hip_ok(hipMalloc(&g_image, image_width * image_height * 4), "hipMalloc(image)")) return false;
    g_total_blocks = total_blocks;
    g_width = image_width;
    g_height = image_height;
    g_mcu_w = mcu_width;
    g_mcu_h = mcu_height;
    g_built = -1;
    g_idct_valid = false;
    return true;
}

bool clidct_transfer_data_to_device(const int block_data_src[1][64], const int offset, const int count)
{
    if (!g_blocks || offset < 0 || count < 0 || offset + count > g_total_blocks) {
        fprintf(stderr, "clidct_transfer_data_to_device: invalid range %d+%d of %d blocks\n", offset, count,
                g_total_blocks);
        return false;
    }
    const size_t bytes = static_cast<size_t>(count) * 64 * sizeof(int32_t);
    if (!hip_ok(hipMemcpyAsync(g_blocks + static_cast<size_t>(offset) * 64, block_data_src, bytes,
                               hipMemcpyHostToDevice, g_stream), "hipMemcpyAsync(H2D)"))
        return false;
    g_idct_valid = false;
    printf("[ ] Writing %zu bytes to device...\n", bytes);
    return hip_ok(hipStreamSynchronize(g_stream), "hipStreamSynchronize");
}

bool clidct_build(ColorSpace colorspace)
{
    if (!g_ctx || !g_blocks) {
        fprintf(stderr, "clidct_build: no memory allocated\n");
        return false;
    }
    if (g_plan) { hjd_plan_destroy(g_plan); g_plan = nullptr; }
    g_built = colorspace;
    if (colorspace == Other) return true;   // IDCT only (the reference's batch_idct)
    const int sampling = colorspace == YUV411 ? HJD_YUV420 : HJD_YUV444;
    const int want = sampling == HJD_YUV420 ? 16 : 8;
    if (g_mcu_w != want || g_mcu_h != want) {
        fprintf(stderr, "clidct_build: MCU %dx%d does not match colour space %d\n", g_mcu_w, g_mcu_h, colorspace);
        return false;
    }
    int64_t need = 0;
    if (hjd_frame_blocks(static_cast<int>(g_width), static_cast<int>(g_height), sampling, &need) != HJD_OK)
        return report("hjd_frame_blocks");
    if (need != g_total_blocks) {
        fprintf(stderr, "clidct_build: %d blocks allocated, image needs %lld\n", g_total_blocks,
                static_cast<long long>(need));
        return false;
    }
    hjd_frame f;
    memset(&f, 0, sizeof(f));
    f.width = static_cast<int32_t>(g_width);
    f.height = static_cast<int32_t>(g_height);
    f.out_pitch = static_cast<int32_t>(g_width * 4);
    f.sampling = sampling;
    if (hjd_plan_create(g_ctx, &f, 1, HJD_IN_I32_NATURAL, nullptr, 0, &g_plan) != HJD_OK)
        return report("hjd_plan_create");
    return true;
}

bool clidct_run(ColorSpace colorspace)
{
    if (!g_ctx || !g_blocks || g_built < 0) {
        fprintf(stderr, "clidct_run: program not built\n");
        return false;
    }
    if (colorspace != g_built) {
        fprintf(stderr, "clidct_run: colour space %d differs from the built one (%d)\n", colorspace, g_built);
        return false;
    }
    if (colorspace == Other) {
        if (!g_idct && !hip_ok(hipMalloc(&g_idct, static_cast<size_t>(g_total_blocks) * 256), "hipMalloc(idct)"))
            return false;
        if (hjd_idct_blocks(g_ctx, g_blocks, g_idct, g_total_blocks, g_stream) != HJD_OK)
            return report("hjd_idct_blocks");
        g_idct_valid = true;
        return true;
    }
    if (hjd_plan_launch(g_plan, g_blocks, g_image, g_stream, 0) != HJD_OK) return report("hjd_plan_launch");
    g_idct_valid = false;
    return true;
}

bool clidct_wait_for_completion() { return g_stream && hip_ok(hipStreamSynchronize(g_stream), "hipStreamSynchronize"); }

bool clidct_retrieve_data_from_device(int block_data_dest[1][64])
{
    if (!g_blocks) return false;
    if (!g_idct_valid) {   // after a fused run the reference's buffer holds IDCT'd blocks
        if (!g_idct && !hip_ok(hipMalloc(&g_idct, static_cast<size_t>(g_total_blocks) * 256), "hipMalloc(idct)"))
            return false;
        if (hjd_idct_blocks(g_ctx, g_blocks, g_idct, g_total_blocks, g_stream) != HJD_OK)
            return report("hjd_idct_blocks");
        g_idct_valid = true;
    }
    const size_t bytes = static_cast<size_t>(g_total_blocks) * 256;
    if (!hip_ok(hipMemcpyAsync(block_data_dest, g_idct, bytes, hipMemcpyDeviceToHost, g_stream), "hipMemcpyAsync(D2H)"))
        return false;
    printf("[ ] Retrieving %zu bytes from device...\n", bytes);
    return hip_ok(hipStreamSynchronize(g_stream), "hipStreamSynchronize");
}

bool clidct_retrieve_image_from_device(void* img_data_dest, const size_t img_width, const size_t img_height)
{
    if (!g_image || img_width > g_width || img_height > g_height || !img_data_dest) {
        fprintf(stderr, "clidct_retrieve_image_from_device: invalid region %zux%zu of %zux%zu\n", img_width,
                img_height, g_width, g_height);
        return false;
    }
    if (!hip_ok(hipMemcpy2DAsync(img_data_dest, img_width * 4, g_image, g_width * 4, img_width * 4, img_height,
                                 hipMemcpyDeviceToHost, g_stream), "hipMemcpy2DAsync(D2H)"))
        return false;
    printf("[ ] Retrieving %zu bytes from device...\n", img_width * 4 * img_height);
    return hip_ok(hipStreamSynchronize(g_stream), "hipStreamSynchronize");
}

bool clidct_clean_up()
{
    if (g_stream) (void)hipStreamSynchronize(g_stream);
    if (g_plan) { hjd_plan_destroy(g_plan); g_plan = nullptr; }
    (void)hipFree(g_blocks); (void)hipFree(g_idct); (void)hipFree(g_image);
    g_blocks = nullptr; g_idct = nullptr; g_image = nullptr;
    if (g_stream) { (void)hipStreamDestroy(g_stream); g_stream = nullptr; }
    if (g_ctx) { hjd_ctx_destroy(g_ctx); g_ctx = nullptr; }
    g_total_blocks = 0; g_width = g_height = 0; g_built = -1; g_idct_valid = false;
    return true;
}
