// idct_compat.hip -- the reference's src/idct.h entry points on the MI355X back-end.
//
// Host-side replacement for src/oclDCT8x8.cpp (OpenCL runtime, file-static state,
// one image at a time) with identical C++ signatures (include/idct.h).  The GPU
// functions drive the C ABI of hjd.h: one context + stream, an int32
// natural-order block buffer (the jpg.mcu_data layout the reference uploads,
// src/decoder.cpp:356), a cropped BGRX image, and a one-frame plan of the fused
// kernel (HJD_IN_I32_NATURAL).  Messages go to stderr and failures return
// false, as in the reference.
//
// Lifecycle.  The reference caller runs create/allocate/build ... clean_up once
// PER IMAGE (src/decoder.cpp:202-216, :518-521), and the OpenCL back-end tears
// everything down each time (src/oclDCT8x8.cpp:316-341).  Here clidct_clean_up
// ends the image only: the context, the stream, the device buffers (grow-only),
// the plan cache (keyed by width, height, colour space) and the pinned staging
// buffers live on, so the second image of a process allocates nothing unless it
// is larger.  HJD_COMPAT_TEARDOWN=1 restores the reference's full release;
// hjd_compat_release() (hjd.h) frees everything explicitly.
//
// Host<->device copies.  The caller's buffers are pageable (jpg.mcu_data is a
// plain new[], src/decoder.cpp:193).  HJD_COMPAT_COPY selects how they move:
//   pageable (default) hipMemcpyAsync straight from / to the caller's buffer;
//   register hipHostRegister the caller's buffer for the copy;
//   staged   memcpy through two pinned 8 MiB chunks while the DMA engine moves
//            the other one.
// Measured on the MI355X box with the reference program at 4K
// (profiles/r02_dropin_timing.json, steady-state images): pageable H2D 30-33
// GB/s and D2H 55 GB/s; register is within noise of it; staged is slowest (one
// host thread's memcpy: 21-26 GB/s H2D, 8-23 GB/s D2H), so pageable is the default.
// HJD_COMPAT_STATS=1 prints one line per image to stderr: allocations, stage
// times and an FNV-1a hash of the retrieved image (tests/test_dropin.py).
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "hjd.h"
#include "hjd_device.hpp"
#include "idct.h"

namespace {

using clk = std::chrono::steady_clock;

enum CopyMode { kPageable = 0, kStaged = 1, kRegister = 2 };
constexpr size_t kChunk = size_t(8) << 20;   // pinned staging chunk (two of them)
constexpr int kPlanCache = 8;

struct CachedPlan {
    hjd_plan* plan = nullptr;
    size_t w = 0, h = 0;
    int cs = -1;
    uint64_t last_use = 0;
};

// Process-lifetime state (the reference keeps the same in file statics,
// src/oclDCT8x8.cpp:11-23, but rebuilds it per image).
struct Compat {
    int device = -1;                   // selected by Initialize_OpenCL_IDCT
    hjd_ctx* ctx = nullptr;
    hipStream_t stream = nullptr;
    hipEvent_t ev_run0 = nullptr, ev_run1 = nullptr, ev_chunk[2] = {nullptr, nullptr};
    void* pinned[2] = {nullptr, nullptr};
    // device buffers, grow-only
    int32_t* blocks = nullptr;  size_t blocks_cap = 0;   // int32 [n][64] natural, dequantised
    int32_t* idct = nullptr;    size_t idct_cap = 0;     // IDCT'd blocks (lazily, retrieve_data)
    uint32_t* image = nullptr;  size_t image_cap = 0;    // BGRX, W x H, pitch W*4
    CachedPlan plans[kPlanCache];
    uint64_t use_clock = 0;
    // the current image
    hjd_plan* plan = nullptr;
    int total_blocks = 0;
    size_t width = 0, height = 0;
    int mcu_w = 0, mcu_h = 0;
    int built = -1;                    // colour space of the built plan
    bool idct_valid = false;
    bool run_timed = false;
    // per-image statistics (HJD_COMPAT_STATS)
    int image_no = 0;
    int allocs = 0;                    // device/pinned buffer allocations made for this image (growth)
    int plans_built = 0;               // plan-cache misses for this image
    double h2d_ms = 0, d2h_ms = 0, alloc_ms = 0;
    size_t h2d_bytes = 0, d2h_bytes = 0;
    uint64_t fnv = 0;
    int copy_mode = kPageable;
    bool stats = false, teardown = false, env_read = false;
} g;

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

double ms_since(clk::time_point t0)
{
    return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

void read_env()
{
    if (g.env_read) return;
    g.env_read = true;
    const char* m = getenv("HJD_COMPAT_COPY");
    if (m && !strcmp(m, "staged")) g.copy_mode = kStaged;
    else if (m && !strcmp(m, "register")) g.copy_mode = kRegister;
    else g.copy_mode = kPageable;
    const char* st = getenv("HJD_COMPAT_STATS");
    g.stats = st && *st && strcmp(st, "0");
    const char* td = getenv("HJD_COMPAT_TEARDOWN");
    g.teardown = td && *td && strcmp(td, "0");
}

// Grow-only device buffer.
template <typename T>
bool ensure(T*& p, size_t& cap, size_t bytes, const char* what)
{
    if (bytes <= cap) return true;
    if (p) { (void)hipStreamSynchronize(g.stream); (void)hipFree(p); p = nullptr; cap = 0; }
    if (!hip_ok(hipMalloc(&p, bytes), what)) return false;
    cap = bytes;
    ++g.allocs;
    return true;
}

bool ensure_pinned()
{
    for (int i = 0; i < 2; ++i) {
        if (g.pinned[i]) continue;
        if (!hip_ok(hipHostMalloc(&g.pinned[i], kChunk, hipHostMallocDefault), "hipHostMalloc(staging)")) return false;
        ++g.allocs;
    }
    return true;
}

// Host (pageable) -> device, blocking on return.
bool copy_h2d(void* dst, const void* src, size_t bytes)
{
    if (bytes == 0) return true;
    if (g.copy_mode == kPageable) {
        if (!hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, g.stream), "hipMemcpyAsync(H2D)"))
            return false;
        return hip_ok(hipStreamSynchronize(g.stream), "hipStreamSynchronize");
    }
    if (g.copy_mode == kRegister) {
        void* hs = const_cast<void*>(src);
        if (!hip_ok(hipHostRegister(hs, bytes, hipHostRegisterDefault), "hipHostRegister")) return false;
        bool ok = hip_ok(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, g.stream), "hipMemcpyAsync(H2D)") &&
                  hip_ok(hipStreamSynchronize(g.stream), "hipStreamSynchronize");
        (void)hipHostUnregister(hs);
        return ok;
    }
    if (!ensure_pinned()) return false;
    // staged: the host fills chunk b while the DMA engine drains chunk b^1
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    bool pending[2] = {false, false};
    int b = 0;
    for (size_t off = 0; off < bytes; off += kChunk, b ^= 1) {
        const size_t n = bytes - off < kChunk ? bytes - off : kChunk;
        if (pending[b] && !hip_ok(hipEventSynchronize(g.ev_chunk[b]), "hipEventSynchronize")) return false;
        memcpy(g.pinned[b], s + off, n);
        if (!hip_ok(hipMemcpyAsync(d + off, g.pinned[b], n, hipMemcpyHostToDevice, g.stream), "hipMemcpyAsync(H2D)") ||
            !hip_ok(hipEventRecord(g.ev_chunk[b], g.stream), "hipEventRecord"))
            return false;
        pending[b] = true;
    }
    return hip_ok(hipStreamSynchronize(g.stream), "hipStreamSynchronize");
}

// Device -> host (pageable), 2-D (rows of `row` bytes at pitches dpitch/spitch), blocking.
bool copy_d2h_2d(void* dst, size_t dpitch, const void* src, size_t spitch, size_t row, size_t rows)
{
    if (row == 0 || rows == 0) return true;
    if (g.copy_mode == kPageable || g.copy_mode == kRegister) {
        void* hd = dst;
        const size_t total = dpitch * (rows - 1) + row;
        if (g.copy_mode == kRegister &&
            !hip_ok(hipHostRegister(hd, total, hipHostRegisterDefault), "hipHostRegister"))
            return false;
        bool ok = hip_ok(hipMemcpy2DAsync(dst, dpitch, src, spitch, row, rows, hipMemcpyDeviceToHost, g.stream),
                         "hipMemcpy2DAsync(D2H)") &&
                  hip_ok(hipStreamSynchronize(g.stream), "hipStreamSynchronize");
        if (g.copy_mode == kRegister) (void)hipHostUnregister(hd);
        return ok;
    }
    if (!ensure_pinned()) return false;
    // staged: DMA rows into chunk b while the host copies chunk b^1 out
    const size_t rows_per = kChunk / row;
    if (rows_per == 0) {
        fprintf(stderr, "clidct_retrieve_image_from_device: row of %zu bytes exceeds the staging chunk\n", row);
        return false;
    }
    const char* s = static_cast<const char*>(src);
    char* d = static_cast<char*>(dst);
    size_t done_rows[2] = {0, 0}, first_row[2] = {0, 0};
    int b = 0;
    auto drain = [&](int k) -> bool {
        if (!done_rows[k]) return true;
        if (!hip_ok(hipEventSynchronize(g.ev_chunk[k]), "hipEventSynchronize")) return false;
        const char* p = static_cast<const char*>(g.pinned[k]);
        if (dpitch == row) memcpy(d + first_row[k] * dpitch, p, done_rows[k] * row);
        else
            for (size_t r = 0; r < done_rows[k]; ++r) memcpy(d + (first_row[k] + r) * dpitch, p + r * row, row);
        done_rows[k] = 0;
        return true;
    };
    for (size_t r0 = 0; r0 < rows; r0 += rows_per, b ^= 1) {
        const size_t n = rows - r0 < rows_per ? rows - r0 : rows_per;
        if (!drain(b)) return false;     // chunk b's previous rows leave before it is reused
        if (!hip_ok(hipMemcpy2DAsync(g.pinned[b], row, s + r0 * spitch, spitch, row, n, hipMemcpyDeviceToHost,
                                     g.stream), "hipMemcpy2DAsync(D2H)") ||
            !hip_ok(hipEventRecord(g.ev_chunk[b], g.stream), "hipEventRecord"))
            return false;
        first_row[b] = r0;
        done_rows[b] = n;
        if (!drain(b ^ 1)) return false; // the other chunk overlaps this DMA
    }
    return drain(0) && drain(1);
}

uint64_t fnv1a(const void* p, size_t n)
{
    const unsigned char* c = static_cast<const unsigned char*>(p);
    uint64_t h = 1469598103934665603ull;
    for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
    return h;
}

void release_all()
{
    if (g.stream) (void)hipStreamSynchronize(g.stream);
    for (auto& c : g.plans) {
        if (c.plan) hjd_plan_destroy(c.plan);
        c = CachedPlan();
    }
    g.plan = nullptr;
    (void)hipFree(g.blocks); (void)hipFree(g.idct); (void)hipFree(g.image);
    g.blocks = nullptr; g.idct = nullptr; g.image = nullptr;
    g.blocks_cap = g.idct_cap = g.image_cap = 0;
    for (int i = 0; i < 2; ++i) {
        if (g.pinned[i]) (void)hipHostFree(g.pinned[i]);
        g.pinned[i] = nullptr;
        if (g.ev_chunk[i]) (void)hipEventDestroy(g.ev_chunk[i]);
        g.ev_chunk[i] = nullptr;
    }
    if (g.ev_run0) (void)hipEventDestroy(g.ev_run0);
    if (g.ev_run1) (void)hipEventDestroy(g.ev_run1);
    g.ev_run0 = g.ev_run1 = nullptr;
    if (g.stream) { (void)hipStreamDestroy(g.stream); g.stream = nullptr; }
    if (g.ctx) { hjd_ctx_destroy(g.ctx); g.ctx = nullptr; }
}

}  // namespace

extern "C" int hjd_compat_release(void)
{
    release_all();
    g.total_blocks = 0; g.width = g.height = 0; g.built = -1; g.idct_valid = false;
    return HJD_OK;
}

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
    read_env();
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
        g.device = 0;
        printf("[ ] HIP device selected.\n");
        return 0;
    }
    printf("[X] No HIP device.\n");
    return 1;
}

bool clidct_create()
{
    read_env();
    if (g.device < 0 && Initialize_OpenCL_IDCT() != 0) return false;
    ++g.image_no;
    g.allocs = 0;
    g.plans_built = 0;
    g.h2d_ms = g.d2h_ms = g.alloc_ms = 0;
    g.h2d_bytes = g.d2h_bytes = 0;
    g.fnv = 0;
    g.run_timed = false;
    if (g.ctx) return true;            // kept from the previous image
    if (hjd_ctx_create(g.device, &g.ctx) != HJD_OK) return report("hjd_ctx_create");
    if (!hip_ok(hipStreamCreateWithFlags(&g.stream, hipStreamNonBlocking), "hipStreamCreate")) return false;
    for (int i = 0; i < 2; ++i)
        if (!hip_ok(hipEventCreateWithFlags(&g.ev_chunk[i], hipEventDisableTiming), "hipEventCreate")) return false;
    if (!hip_ok(hipEventCreate(&g.ev_run0), "hipEventCreate") || !hip_ok(hipEventCreate(&g.ev_run1), "hipEventCreate"))
        return false;
    return true;
}

bool clidct_allocate_memory(const int total_blocks, const size_t image_width, const size_t image_height,
                            const int mcu_width, const int mcu_height)
{
    if (!g.ctx) {
        fprintf(stderr, "clidct_allocate_memory: no context (call clidct_create first)\n");
        return false;
    }
    if (total_blocks <= 0 || image_width == 0 || image_height == 0) {
        fprintf(stderr, "clidct_allocate_memory: invalid arguments\n");
        return false;
    }
    const auto t0 = clk::now();
    if (!ensure(g.blocks, g.blocks_cap, static_cast<size_t>(total_blocks) * 64 * sizeof(int32_t), "hipMalloc(blocks)") ||
        !ensure(g.image, g.image_cap, image_width * image_height * 4, "hipMalloc(image)"))
        return false;
    g.alloc_ms += ms_since(t0);
    g.total_blocks = total_blocks;
    g.width = image_width;
    g.height = image_height;
    g.mcu_w = mcu_width;
    g.mcu_h = mcu_height;
    g.built = -1;
    g.plan = nullptr;
    g.idct_valid = false;
    return true;
}

bool clidct_transfer_data_to_device(const int block_data_src[1][64], const int offset, const int count)
{
    if (!g.blocks || offset < 0 || count < 0 || offset + count > g.total_blocks) {
        fprintf(stderr, "clidct_transfer_data_to_device: invalid range %d+%d of %d blocks\n", offset, count,
                g.total_blocks);
        return false;
    }
    const size_t bytes = static_cast<size_t>(count) * 64 * sizeof(int32_t);
    const auto t0 = clk::now();
    if (!copy_h2d(g.blocks + static_cast<size_t>(offset) * 64, block_data_src, bytes)) return false;
    g.h2d_ms += ms_since(t0);
    g.h2d_bytes += bytes;
    g.idct_valid = false;
    printf("[ ] Writing %zu bytes to device...\n", bytes);
    return true;
}

bool clidct_build(ColorSpace colorspace)
{
    if (!g.ctx || !g.blocks) {
        fprintf(stderr, "clidct_build: no memory allocated\n");
        return false;
    }
    g.plan = nullptr;
    g.built = colorspace;
    if (colorspace == Other) return true;   // IDCT only (the reference's batch_idct)
    const int sampling = colorspace == YUV411 ? HJD_YUV420 : HJD_YUV444;
    const int want = sampling == HJD_YUV420 ? 16 : 8;
    if (g.mcu_w != want || g.mcu_h != want) {
        fprintf(stderr, "clidct_build: MCU %dx%d does not match colour space %d\n", g.mcu_w, g.mcu_h, colorspace);
        g.built = -1;
        return false;
    }
    int64_t need = 0;
    if (hjd_frame_blocks(static_cast<int>(g.width), static_cast<int>(g.height), sampling, &need) != HJD_OK)
        return report("hjd_frame_blocks");
    if (need != g.total_blocks) {
        fprintf(stderr, "clidct_build: %d blocks allocated, image needs %lld\n", g.total_blocks,
                static_cast<long long>(need));
        g.built = -1;
        return false;
    }
    // plan cache: the frame table depends only on (W, H, colour space)
    ++g.use_clock;
    CachedPlan* victim = &g.plans[0];
    for (auto& c : g.plans) {
        if (c.plan && c.w == g.width && c.h == g.height && c.cs == colorspace) {
            c.last_use = g.use_clock;
            g.plan = c.plan;
            return true;
        }
        if (!c.plan || (victim->plan && c.last_use < victim->last_use)) victim = &c;
    }
    hjd_frame f;
    memset(&f, 0, sizeof(f));
    f.width = static_cast<int32_t>(g.width);
    f.height = static_cast<int32_t>(g.height);
    f.out_pitch = static_cast<int32_t>(g.width * 4);
    f.sampling = sampling;
    hjd_plan* p = nullptr;
    if (hjd_plan_create(g.ctx, &f, 1, HJD_IN_I32_NATURAL, nullptr, 0, &p) != HJD_OK) return report("hjd_plan_create");
    ++g.plans_built;                   // a new geometry: the plan's device frame table
    if (victim->plan) hjd_plan_destroy(victim->plan);
    *victim = CachedPlan{p, g.width, g.height, colorspace, g.use_clock};
    g.plan = p;
    return true;
}

bool clidct_run(ColorSpace colorspace)
{
    if (!g.ctx || !g.blocks || g.built < 0) {
        fprintf(stderr, "clidct_run: program not built\n");
        return false;
    }
    if (colorspace != g.built) {
        fprintf(stderr, "clidct_run: colour space %d differs from the built one (%d)\n", colorspace, g.built);
        return false;
    }
    (void)hipEventRecord(g.ev_run0, g.stream);
    if (colorspace == Other) {
        if (!ensure(g.idct, g.idct_cap, static_cast<size_t>(g.total_blocks) * 256, "hipMalloc(idct)")) return false;
        if (hjd_idct_blocks(g.ctx, g.blocks, g.idct, g.total_blocks, g.stream) != HJD_OK)
            return report("hjd_idct_blocks");
        g.idct_valid = true;
    } else {
        if (hjd_plan_launch(g.plan, g.blocks, g.image, g.stream, 0) != HJD_OK) return report("hjd_plan_launch");
        g.idct_valid = false;
    }
    (void)hipEventRecord(g.ev_run1, g.stream);
    g.run_timed = true;
    return true;
}

bool clidct_wait_for_completion()
{
    return g.stream && hip_ok(hipStreamSynchronize(g.stream), "hipStreamSynchronize");
}

bool clidct_retrieve_data_from_device(int block_data_dest[1][64])
{
    if (!g.blocks) return false;
    if (!g.idct_valid) {   // after a fused run the reference's buffer holds IDCT'd blocks
        if (!ensure(g.idct, g.idct_cap, static_cast<size_t>(g.total_blocks) * 256, "hipMalloc(idct)")) return false;
        if (hjd_idct_blocks(g.ctx, g.blocks, g.idct, g.total_blocks, g.stream) != HJD_OK)
            return report("hjd_idct_blocks");
        g.idct_valid = true;
    }
    const size_t bytes = static_cast<size_t>(g.total_blocks) * 256;
    const auto t0 = clk::now();
    if (!copy_d2h_2d(block_data_dest, 256, g.idct, 256, 256, static_cast<size_t>(g.total_blocks)))
        return false;
    g.d2h_ms += ms_since(t0);
    g.d2h_bytes += bytes;
    printf("[ ] Retrieving %zu bytes from device...\n", bytes);
    return true;
}

bool clidct_retrieve_image_from_device(void* img_data_dest, const size_t img_width, const size_t img_height)
{
    if (!g.image || img_width > g.width || img_height > g.height || !img_data_dest) {
        fprintf(stderr, "clidct_retrieve_image_from_device: invalid region %zux%zu of %zux%zu\n", img_width,
                img_height, g.width, g.height);
        return false;
    }
    const auto t0 = clk::now();
    if (!copy_d2h_2d(img_data_dest, img_width * 4, g.image, g.width * 4, img_width * 4, img_height)) return false;
    g.d2h_ms += ms_since(t0);
    g.d2h_bytes += img_width * 4 * img_height;
    if (g.stats) g.fnv = fnv1a(img_data_dest, img_width * 4 * img_height);
    printf("[ ] Retrieving %zu bytes from device...\n", img_width * 4 * img_height);
    return true;
}

bool clidct_clean_up()
{
    if (g.stream) (void)hipStreamSynchronize(g.stream);
    if (g.stats) {
        float kms = 0.f;
        if (g.run_timed) (void)hipEventElapsedTime(&kms, g.ev_run0, g.ev_run1);
        static const char* modes[] = {"pageable", "staged", "register"};
        fprintf(stderr,
                "[hjd-compat] image=%d size=%zux%zu blocks=%d allocs=%d plans_built=%d alloc_ms=%.3f h2d_ms=%.3f h2d_GBps=%.2f "
                "kernel_ms=%.3f d2h_ms=%.3f d2h_GBps=%.2f copy=%s fnv=%016llx\n",
                g.image_no, g.width, g.height, g.total_blocks, g.allocs, g.plans_built, g.alloc_ms, g.h2d_ms,
                g.h2d_ms > 0 ? g.h2d_bytes / g.h2d_ms / 1e6 : 0.0, kms, g.d2h_ms,
                g.d2h_ms > 0 ? g.d2h_bytes / g.d2h_ms / 1e6 : 0.0, modes[g.copy_mode],
                static_cast<unsigned long long>(g.fnv));
    }
    if (g.teardown) release_all();     // the reference's per-image teardown (src/oclDCT8x8.cpp:316-341)
    g.plan = nullptr;
    g.total_blocks = 0; g.width = g.height = 0; g.built = -1; g.idct_valid = false;
    return true;
}
