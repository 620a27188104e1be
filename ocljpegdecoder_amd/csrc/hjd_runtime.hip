// hjd_runtime.hip -- C-ABI runtime of the MI355X pixel back-end (include/hjd.h).
//
// Replaces the reference's OpenCL host runtime (src/oclDCT8x8.cpp:25-341):
// device selection, buffers, kernel selection per colour space and launch.
// Unlike the reference there is no file-static state here: contexts and plans
// are handles, so several images / frames / devices can be in flight.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdlib>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <tuple>
#include <new>
#include <string>
#include <vector>

#include "hjd.h"
#include "hjd_internal.h"
#include "hjd_kernels.hpp"

using hjd::FrameDev;
using hjd_internal::SamplingGeom;
using hjd_internal::sampling_geom;

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HJD_HIP(call)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (call);                                                              \
        if (e_ != hipSuccess)                                                                \
            return fail(HJD_E_HIP, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_),    \
                        __FILE__, __LINE__);                                                 \
    } while (0)

// JPEG zigzag: natural index of zigzag position k (src/zigzag.h:15-40).
constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

}  // namespace

int hjd_internal::set_error(int code, const char* fmt, ...)
{
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

struct hjd_ctx {
    int device = 0;
    int num_cu = 256;
};

struct hjd_plan {
    hjd_ctx* ctx = nullptr;
    int input_format = 0;
    int sampling = -1;          // common sampling of all frames (kernel template)
    int nframes = 0;
    int64_t tasks = 0;
    int64_t pixels = 0;
    int64_t coef_bytes = 0;
    FrameDev* d_frames = nullptr;
    int* d_qt = nullptr;        // natural-order tables [nq][64]
    int variant = 0;            // kernel variant bits (hjd_plan_set_variant)
    int out_format = HJD_OUT_BGRX;   // common output format of all frames
    int kernel_mode = HJD_KERNEL_AUTO;
    int tuned_grid = 0;         // hjd_plan_autotune's / hjd_plan_set_chunk's grid (0: the shape default)
    int tuned_per_wave = 0;     // its tasks per wave
    int autotune_launches = 0;  // kernel launches of the last hjd_plan_autotune
    int autotune_cached = 0;    // 1: that call reused a cached choice
};

constexpr int64_t kDefaultLatencyMaxTasks = 1024;   // measured: profiles/r01_latency_kernel.json

// Launches of at most this many tasks take the latency kernel (one workgroup
// per task) in HJD_KERNEL_AUTO mode; HJD_LAT_TASKS overrides it (tuning).
static int64_t latency_max_tasks()
{
    static const int64_t v = [] {
        const char* e = getenv("HJD_LAT_TASKS");
        return e ? static_cast<int64_t>(atoll(e)) : int64_t(kDefaultLatencyMaxTasks);
    }();
    return v;
}

// The 4:4:4 kernels gather coefficient pairs with ds_read_u16_d16_hi
// (hjd::kVarD16), which relies on d16 LDS loads zeroing the other half of
// the register.  MI355X as deployed (sramecc+) does that
// (profiles/r03_d16_probe.txt); a half-preserving part would corrupt the
// pairs.  So the variant is taken only where the one-wave hardware probe
// (hjd_probe.hip, run by hjd_ctx_create) completed and saw every lane's low
// half zeroed; the v_perm kernels are the fallback.  HJD_D16=0 forces the
// fallback (A/B); nothing forces the d16 kernels onto a part the probe did not
// pass.  Launches only read the cached answer.
bool hjd_internal::d16_gather_selected(int device)
{
    const char* e = getenv("HJD_D16");
    if (e && e[0] == '0') return false;
    return device >= 0 && hjd_internal::d16_probe_cached(device) == 1;
}
static bool device_d16_gather(int device) { return hjd_internal::d16_gather_selected(device); }

static int geometry(int width, int height, int sampling, int& mcu_w, int& mcu_h, int& bpm, int& tasks_mcus);
static int64_t default_per_wave(int sampling, int fmt);
static int grid_for_chunk(int64_t tasks, int64_t per_wave, bool occupancy_floor = true);

// launch_decode variant bits 8 and up: a stage-skipping measurement variant
// (hjd_debug_plan_launch_stages), stages << kStageShift | plan variant bits.
constexpr int kStageShift = 8;

int hjd_internal::ctx_num_cu(const hjd_ctx* ctx) { return ctx->num_cu; }

int64_t hjd_internal::make_frame_record(int width, int height, int sampling, int64_t coef_base, int64_t out_base,
                                        int pitch, const int qt_index[3], FrameRecord* rec, int out_format)
{
    int mw, mh, bpm, tasks_mcus;
    int rc = geometry(width, height, sampling, mw, mh, bpm, tasks_mcus);
    if (rc) return rc;
    static_assert(sizeof(FrameRecord) == sizeof(FrameDev), "record layout");
    FrameDev d;
    memset(&d, 0, sizeof(d));
    d.coef_base = coef_base;
    d.out_base = out_base;
    d.task_begin = 0;
    d.width = width;
    d.height = height;
    d.pitch = pitch;
    d.sampling = sampling;
    d.mcu_w = mw;
    d.strips = (mw + tasks_mcus - 1) / tasks_mcus;
    for (int c = 0; c < 3; ++c) d.qt[c] = qt_index ? qt_index[c] : 0;
    d.vec_ok = out_vector_ok(out_format, pitch, out_base) ? 1 : 0;
    memcpy(rec, &d, sizeof(d));
    return static_cast<int64_t>(d.strips) * mh;
}

int hjd_internal::launch_decode(int device, int num_cu, int sampling, int input_format, int variant,
                                const void* d_coefs, const int32_t* d_qt_nat, const FrameRecord* d_frames,
                                int nframes, int64_t tasks, void* d_out, void* stream, int grid_blocks, int out_format,
                                int kernel_mode)
{
    HJD_HIP(hipSetDevice(device));
    const int fmt = input_format == HJD_IN_Q16_ZIGZAG ? 0 : 1;
    (void)num_cu;
    SamplingGeom sg;
    if (!sampling_geom(sampling, &sg)) return set_error(HJD_E_INVALID, "unsupported sampling %d", sampling);
    const int grid = grid_blocks > 0 ? grid_blocks : grid_for_chunk(tasks, default_per_wave(sampling, fmt));
    if (out_format != HJD_OUT_BGRX && out_format != HJD_OUT_BGR24)
        return set_error(HJD_E_INVALID, "unknown output format %d", out_format);
    using K = void (*)(const void*, const int*, const FrameDev*, int, int64_t, uint8_t*);   // latency kernels
    using KP = void (*)(const void*, const int*, const FrameDev*, int, int64_t, uint8_t*, int64_t, int64_t);
    const bool latency = kernel_mode == HJD_KERNEL_LATENCY ||
                         (kernel_mode == HJD_KERNEL_AUTO && grid_blocks == 0 && tasks <= latency_max_tasks());
    // the task split of the persistent kernels (see decode_kernel): default
    // order over grid * 4 waves, wg-interleave over grid groups of 4-task quads
    const int64_t split_n = (variant & 2) ? static_cast<int64_t>(grid) : static_cast<int64_t>(grid) * hjd::kWavesPerGroup;
    const int64_t split_t = (variant & 2) ? (tasks + hjd::kWavesPerGroup - 1) / hjd::kWavesPerGroup : tasks;
    const int64_t chunk = split_t / split_n, rem = split_t % split_n;
    if (latency && (variant >> kStageShift) == 0) {   // [output format][sampling index][input format]
#define HJD_KL(V) hjd::decode_kernel_lat<0, 0, V>, hjd::decode_kernel_lat<0, 1, V>, \
                  hjd::decode_kernel_lat<1, 0, V>, hjd::decode_kernel_lat<1, 1, V>, \
                  hjd::decode_kernel_lat<2, 0, V>, hjd::decode_kernel_lat<2, 1, V>, \
                  hjd::decode_kernel_lat<3, 0, V>, hjd::decode_kernel_lat<3, 1, V>, \
                  hjd::decode_kernel_lat<4, 0, V>, hjd::decode_kernel_lat<4, 1, V>, \
                  hjd::decode_kernel_lat<5, 0, V>, hjd::decode_kernel_lat<5, 1, V>
        static const K kLat[24] = {HJD_KL(0), HJD_KL(hjd::kOutBgr24)};
#undef HJD_KL
        if (tasks > (int64_t(1) << 31) - 1) return set_error(HJD_E_INVALID, "too many tasks for the latency kernel");
        const K k = kLat[(out_format == HJD_OUT_BGR24 ? 12 : 0) + ((sg.index << 1) | fmt)];
        hipLaunchKernelGGL(k, dim3(static_cast<uint32_t>(tasks)), dim3(hjd::kLatThreads), 0,
                           static_cast<hipStream_t>(stream), d_coefs, d_qt_nat,
                           reinterpret_cast<const FrameDev*>(d_frames), nframes, tasks, static_cast<uint8_t*>(d_out));
        HJD_HIP(hipGetLastError());
        return HJD_OK;
    }
    if (out_format == HJD_OUT_BGR24) {   // [sampling index][input format], default variant
        static const KP kTable24[12] = {
            hjd::decode_kernel<0, 0, hjd::kOutBgr24>, hjd::decode_kernel<0, 1, hjd::kOutBgr24>,
            hjd::decode_kernel<1, 0, hjd::kOutBgr24>, hjd::decode_kernel<1, 1, hjd::kOutBgr24>,
            hjd::decode_kernel<2, 0, hjd::kOutBgr24>, hjd::decode_kernel<2, 1, hjd::kOutBgr24>,
            hjd::decode_kernel<3, 0, hjd::kOutBgr24>, hjd::decode_kernel<3, 1, hjd::kOutBgr24>,
            hjd::decode_kernel<4, 0, hjd::kOutBgr24>, hjd::decode_kernel<4, 1, hjd::kOutBgr24>,
            hjd::decode_kernel<5, 0, hjd::kOutBgr24>, hjd::decode_kernel<5, 1, hjd::kOutBgr24>};
        if ((variant & 3) != 0) return set_error(HJD_E_INVALID, "kernel variants are BGRX-only");
        KP k24 = kTable24[(sg.index << 1) | fmt];
        if (sampling == HJD_YUV444 && fmt == 0 && device_d16_gather(device))
            k24 = hjd::decode_kernel<0, 0, hjd::kOutBgr24 | hjd::kVarD16>;
        hipLaunchKernelGGL(k24, dim3(grid), dim3(hjd::kGroupThreads), 0,
                           static_cast<hipStream_t>(stream), d_coefs, d_qt_nat,
                           reinterpret_cast<const FrameDev*>(d_frames), nframes, tasks, static_cast<uint8_t*>(d_out),
                           chunk, rem);
        HJD_HIP(hipGetLastError());
        return HJD_OK;
    }
    if (fmt == 0 && (variant >> kStageShift) != 0) {   // stage-skipping measurement variants
        if (sg.index > 1) return hjd_internal::set_error(HJD_E_INVALID, "ablation variants are 4:4:4/4:2:0 only");
        constexpr int kStages[8] = {4, 8, 16, 20, 24, 64, 80, 256};
        const int stages = variant >> kStageShift;
        int si = -1;
        for (int i = 0; i < 8; ++i)
            if (kStages[i] == stages) si = i;
        if (si < 0) return hjd_internal::set_error(HJD_E_INVALID, "unknown ablation variant %d", stages);
#define HJD_ST(S, B) {hjd::decode_kernel<S, 0, 4 | (B)>, hjd::decode_kernel<S, 0, 8 | (B)>,                  \
                      hjd::decode_kernel<S, 0, 16 | (B)>, hjd::decode_kernel<S, 0, 20 | (B)>,                \
                      hjd::decode_kernel<S, 0, 24 | (B)>, hjd::decode_kernel<S, 0, 64 | (B)>,                \
                      hjd::decode_kernel<S, 0, 80 | (B)>, hjd::decode_kernel<S, 0, 256 | (B)>}
        // [4:2:0, 4:4:4, 4:4:4 d16 gather][stages]
        static const KP kStageK[3][8] = {HJD_ST(1, 0), HJD_ST(0, 0), HJD_ST(0, hjd::kVarD16)};
#undef HJD_ST
        const int col = sampling == HJD_YUV420 ? 0 : device_d16_gather(device) ? 2 : 1;   // as the product gathers
        const KP k = kStageK[col][si];
        hipLaunchKernelGGL(k, dim3(grid), dim3(hjd::kGroupThreads), 0, static_cast<hipStream_t>(stream), d_coefs,
                           d_qt_nat, reinterpret_cast<const FrameDev*>(d_frames), nframes, tasks,
                           static_cast<uint8_t*>(d_out), chunk, rem);
        HJD_HIP(hipGetLastError());
        return HJD_OK;
    }
    // [sampling index][input format][variant bits 0-1]
    const int key = (sg.index << 3) | (fmt << 2) | (variant & 3);
#define HJD_K4(S, F) hjd::decode_kernel<S, F, 0>, hjd::decode_kernel<S, F, 1>, hjd::decode_kernel<S, F, 2>, \
                     hjd::decode_kernel<S, F, 3>
    static const KP kTable[48] = {HJD_K4(0, 0), HJD_K4(0, 1), HJD_K4(1, 0), HJD_K4(1, 1),
                                 HJD_K4(2, 0), HJD_K4(2, 1), HJD_K4(3, 0), HJD_K4(3, 1),
                                 HJD_K4(4, 0), HJD_K4(4, 1), HJD_K4(5, 0), HJD_K4(5, 1)};
#undef HJD_K4
    KP k = kTable[key];
    if (sampling == HJD_YUV444 && fmt == 0 && (variant & 2) == 0 && device_d16_gather(device))
        k = (variant & 1) ? hjd::decode_kernel<0, 0, hjd::kVarPlainStores | hjd::kVarD16>
                          : hjd::decode_kernel<0, 0, hjd::kVarD16>;
    hipLaunchKernelGGL(k, dim3(grid), dim3(hjd::kGroupThreads), 0, static_cast<hipStream_t>(stream),
                       d_coefs, d_qt_nat, reinterpret_cast<const FrameDev*>(d_frames), nframes, tasks,
                       static_cast<uint8_t*>(d_out), chunk, rem);
    HJD_HIP(hipGetLastError());
    return HJD_OK;
}

extern "C" {

int hjd_abi_version(void) { return HJD_ABI_VERSION; }

const char* hjd_last_error(void) { return g_last_error.c_str(); }

int hjd_device_count(int* count)
{
    if (!count) return fail(HJD_E_INVALID, "count is NULL");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) {
        *count = 0;
        if (e == hipErrorNoDevice) return HJD_OK;
        return fail(HJD_E_HIP, "hipGetDeviceCount: %s", hipGetErrorString(e));
    }
    *count = n;
    return HJD_OK;
}

int hjd_ctx_create(int device, hjd_ctx** out)
{
    if (!out) return fail(HJD_E_INVALID, "out is NULL");
    *out = nullptr;
    int n = 0;
    int rc = hjd_device_count(&n);
    if (rc) return rc;
    if (device < 0 || device >= n) return fail(HJD_E_NO_DEVICE, "device %d not present (%d devices)", device, n);
    HJD_HIP(hipSetDevice(device));
    hjd_ctx* c = new (std::nothrow) hjd_ctx;
    if (!c) return fail(HJD_E_NOMEM, "context allocation");
    c->device = device;
    int cu = 0;
    if (hipDeviceGetAttribute(&cu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && cu > 0)
        c->num_cu = cu;
    // the d16 gather probe runs here, once per device, so that no launch (which
    // may be inside a stream capture) ever has to run it; a failed probe leaves
    // no HIP error behind and the launches use the v_perm kernels
    (void)hjd_internal::d16_probe(device);
    *out = c;
    return HJD_OK;
}

int hjd_ctx_destroy(hjd_ctx* ctx)
{
    delete ctx;
    return HJD_OK;
}

int hjd_ctx_device(const hjd_ctx* ctx) { return ctx ? ctx->device : -1; }

static int geometry(int width, int height, int sampling, int& mcu_w, int& mcu_h, int& bpm, int& tasks_mcus)
{
    if (width <= 0 || height <= 0 || width > 65535 || height > 65535)
        return fail(HJD_E_INVALID, "invalid dimensions %dx%d", width, height);
    SamplingGeom g;
    if (!sampling_geom(sampling, &g))
        return fail(HJD_E_INVALID, "unsupported sampling %d (4:4:4, 4:2:0, 4:2:2, gray, 4:1:1 or 4:4:0)",
                    sampling);
    bpm = g.bpm;
    tasks_mcus = g.mcus_per_task;
    mcu_w = (width - 1) / g.mcu_px_w + 1;   // src/decoder.cpp:189-190
    mcu_h = (height - 1) / g.mcu_px_h + 1;
    return HJD_OK;
}

int hjd_frame_blocks(int width, int height, int sampling, int64_t* nblocks)
{
    int mw, mh, bpm, tasks_mcus;
    int rc = geometry(width, height, sampling, mw, mh, bpm, tasks_mcus);
    if (rc) return rc;
    if (!nblocks) return fail(HJD_E_INVALID, "nblocks is NULL");
    *nblocks = static_cast<int64_t>(mw) * mh * bpm;
    return HJD_OK;
}

int hjd_plan_create(hjd_ctx* ctx, const hjd_frame* frames, int nframes, int input_format,
                    const int32_t* qtables, int nq, hjd_plan** out)
{
    if (!ctx || !out || (!frames && nframes > 0) || nframes < 0)
        return fail(HJD_E_INVALID, "invalid plan arguments");
    *out = nullptr;
    if (input_format != HJD_IN_Q16_ZIGZAG && input_format != HJD_IN_I32_NATURAL)
        return fail(HJD_E_INVALID, "unknown input format %d", input_format);
    if (input_format == HJD_IN_Q16_ZIGZAG && (!qtables || nq <= 0))
        return fail(HJD_E_INVALID, "quantisation tables required for HJD_IN_Q16_ZIGZAG");

    std::vector<FrameDev> fd(static_cast<size_t>(std::max(nframes, 1)));
    int64_t tasks = 0, pixels = 0, blocks = 0;
    int sampling = nframes > 0 ? frames[0].sampling : HJD_YUV420;
    const int out_format = nframes > 0 ? frames[0].out_format : HJD_OUT_BGRX;
    const int obytes = hjd_internal::out_format_bytes(out_format);
    if (!obytes) return fail(HJD_E_INVALID, "unknown output format %d", out_format);
    for (int i = 0; i < nframes; ++i) {
        const hjd_frame& f = frames[i];
        int mw, mh, bpm, tasks_mcus;
        int rc = geometry(f.width, f.height, f.sampling, mw, mh, bpm, tasks_mcus);
        if (rc) return fail(rc, "frame %d: %s", i, g_last_error.c_str());
        if (f.sampling != sampling)
            return fail(HJD_E_INVALID, "frame %d: mixed sampling in one plan (use one plan per sampling)", i);
        if (f.out_format != out_format)
            return fail(HJD_E_INVALID, "frame %d: mixed output formats in one plan (use one plan per format)", i);
        if (f.out_pitch < static_cast<int64_t>(obytes) * f.width || (f.out_pitch & 3) || (f.out_offset & 3))
            return fail(HJD_E_INVALID, "frame %d: bad output pitch/offset", i);
        FrameDev& d = fd[i];
        if (input_format == HJD_IN_Q16_ZIGZAG) {
            for (int c = 0; c < 3; ++c)
                if (f.qt_index[c] < 0 || f.qt_index[c] >= nq)
                    return fail(HJD_E_INVALID, "frame %d: qt_index[%d]=%d out of range", i, c, f.qt_index[c]);
        }
        d.coef_base = static_cast<int64_t>(f.coef_offset);
        d.out_base = static_cast<int64_t>(f.out_offset);
        d.task_begin = tasks;
        d.width = f.width;
        d.height = f.height;
        d.pitch = f.out_pitch;
        d.sampling = f.sampling;
        d.mcu_w = mw;
        d.strips = (mw + tasks_mcus - 1) / tasks_mcus;
        for (int c = 0; c < 3; ++c) d.qt[c] = input_format == HJD_IN_Q16_ZIGZAG ? f.qt_index[c] : 0;
        d.vec_ok = hjd_internal::out_vector_ok(out_format, f.out_pitch, static_cast<int64_t>(f.out_offset)) ? 1 : 0;
        tasks += static_cast<int64_t>(d.strips) * mh;
        pixels += static_cast<int64_t>(f.width) * f.height;
        blocks += static_cast<int64_t>(mw) * mh * bpm;
    }

    HJD_HIP(hipSetDevice(ctx->device));
    hjd_plan* p = new (std::nothrow) hjd_plan;
    if (!p) return fail(HJD_E_NOMEM, "plan allocation");
    p->ctx = ctx;
    p->input_format = input_format;
    p->sampling = sampling;
    p->out_format = out_format;
    p->nframes = nframes;
    p->tasks = tasks;
    p->pixels = pixels;
    p->coef_bytes = blocks * (input_format == HJD_IN_Q16_ZIGZAG ? 128 : 256);

    // qtables: file (zigzag) order -> natural order, so a lane reads its row's
    // 8 factors contiguously.
    const int nqt = input_format == HJD_IN_Q16_ZIGZAG ? nq : 1;
    std::vector<int32_t> qnat(static_cast<size_t>(nqt) * 64, 0);
    if (input_format == HJD_IN_Q16_ZIGZAG)
        for (int t = 0; t < nq; ++t)
            for (int k = 0; k < 64; ++k) qnat[t * 64 + kZigzag[k]] = qtables[t * 64 + k];

    hipError_t e = hipMalloc(&p->d_frames, fd.size() * sizeof(FrameDev));
    if (e == hipSuccess) e = hipMalloc(&p->d_qt, qnat.size() * sizeof(int32_t));
    if (e == hipSuccess) e = hipMemcpy(p->d_frames, fd.data(), fd.size() * sizeof(FrameDev), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(p->d_qt, qnat.data(), qnat.size() * sizeof(int32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess) {
        (void)hipFree(p->d_frames);
        (void)hipFree(p->d_qt);
        delete p;
        return fail(HJD_E_HIP, "plan upload: %s", hipGetErrorString(e));
    }
    *out = p;
    return HJD_OK;
}

int hjd_plan_destroy(hjd_plan* plan)
{
    if (!plan) return HJD_OK;
    (void)hipSetDevice(plan->ctx->device);
    (void)hipFree(plan->d_frames);
    (void)hipFree(plan->d_qt);
    delete plan;
    return HJD_OK;
}

int hjd_plan_set_variant(hjd_plan* plan, int variant)
{
    if (!plan) return fail(HJD_E_INVALID, "plan is NULL");
    if (variant < 0 || variant > 3) return fail(HJD_E_INVALID, "unknown kernel variant %d", variant);
    plan->variant = variant;
    return HJD_OK;
}

int hjd_plan_set_chunk(hjd_plan* plan, int tasks)
{
    if (!plan || tasks < 0 || tasks > 4096) return fail(HJD_E_INVALID, "invalid chunk arguments");
    plan->tuned_per_wave = tasks;
    // exactly `tasks` per wave: no occupancy floor (unlike the shape default)
    plan->tuned_grid = tasks ? grid_for_chunk(std::max<int64_t>(plan->tasks, 1), tasks, false) : 0;   // 0: default
    return HJD_OK;
}

int hjd_plan_set_kernel(hjd_plan* plan, int mode)
{
    if (!plan) return fail(HJD_E_INVALID, "plan is NULL");
    if (mode != HJD_KERNEL_AUTO && mode != HJD_KERNEL_PERSISTENT && mode != HJD_KERNEL_LATENCY)
        return fail(HJD_E_INVALID, "unknown kernel mode %d", mode);
    plan->kernel_mode = mode;
    return HJD_OK;
}

int64_t hjd_plan_tasks(const hjd_plan* plan) { return plan ? plan->tasks : -1; }
int64_t hjd_plan_pixels(const hjd_plan* plan) { return plan ? plan->pixels : -1; }
int64_t hjd_plan_coef_bytes(const hjd_plan* plan) { return plan ? plan->coef_bytes : -1; }

// Grid of the fused kernel: short contiguous task chunks per wave and many
// more workgroups than fit at once (measured on MI355X, profiles/
// r01_tune_grid_*.json): the hardware dispatches groups in order, so the
// resident waves always work inside a narrow window of the batch and HBM sees
// far better locality than with 4096 persistent waves spread over the whole
// batch (4:2:0 +12 %, 4:4:4 +13 % over one persistent wave per slot).  With
// the XCD-contiguous group order (hjd_kernels.hpp group_order) the best chunk
// is 2 tasks per wave at 4:2:0 (+3.9 % over 1 on 1024-frame batches) and 16 at
// the VALU-heavier samplings 4:4:4, 4:2:2 and 4:4:0 (+1.3 % over 8 at 4:4:4;
// profiles/r02_tune_tasks_per_wave.json).  The lighter, memory-bound shapes
// want one task per wave: grayscale (0.69 -> 0.80 of 8 TB/s), 4:1:1 (0.65-0.71
// -> 0.76) and both int32 (idct.h) formats (4:2:0 0.67 -> 0.76-0.78, 4:4:4
// 0.74-0.75 -> 0.765-0.77), same box (profiles/r03_tune_tasks_per_wave_ext.json).
// HJD_TASKS_PER_WAVE overrides it (tuning).
static int64_t default_per_wave(int sampling, int fmt)
{
    static const int64_t env = [] {
        const char* e = getenv("HJD_TASKS_PER_WAVE");
        return e ? static_cast<int64_t>(atoll(e)) : int64_t(0);
    }();
    if (env > 0) return env;
    if (fmt != 0 || sampling == HJD_GRAY || sampling == HJD_YUV411_H4V1) return 1;
    return sampling == HJD_YUV420 ? 2 : 16;
}

// Tasks per wave a chunk request turns into: with the occupancy floor (the
// shape default and the autotune candidates) never fewer than ~4 waves per
// SIMD (256 CUs x 4 SIMDs), since a single 4:4:4 frame at 16 tasks per wave
// would leave most of the chip idle; hjd_plan_set_chunk pins it exactly.
static int64_t effective_per_wave(int64_t tasks, int64_t per_wave, bool occupancy_floor)
{
    if (occupancy_floor) per_wave = std::min<int64_t>(per_wave, tasks / (4 * 1024));
    return std::max<int64_t>(1, per_wave);
}

// Groups for `per_wave` tasks per wave.
static int grid_for_chunk(int64_t tasks, int64_t per_wave, bool occupancy_floor)
{
    per_wave = effective_per_wave(tasks, per_wave, occupancy_floor);
    const int64_t waves = (tasks + per_wave - 1) / per_wave;
    const int64_t groups = (waves + hjd::kWavesPerGroup - 1) / hjd::kWavesPerGroup;
    return static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(groups, int64_t(1) << 24)));
}

// A default launch of this plan takes the persistent kernel (not the latency one).
static bool plan_is_persistent(const hjd_plan* p)
{
    return p->kernel_mode == HJD_KERNEL_PERSISTENT ||
           (p->kernel_mode == HJD_KERNEL_AUTO && p->tasks > latency_max_tasks());
}

static int default_grid(const hjd_ctx* ctx, int64_t work_waves)
{
    const int64_t cap = static_cast<int64_t>(ctx->num_cu) * 4;
    const int64_t need = (work_waves + hjd::kWavesPerGroup - 1) / hjd::kWavesPerGroup;
    return static_cast<int>(std::max<int64_t>(1, std::min(cap, need)));
}

int hjd_plan_launch(hjd_plan* plan, const void* d_coefs, void* d_out, void* stream, int grid_blocks)
{
    if (!plan) return fail(HJD_E_INVALID, "plan is NULL");
    if (plan->tasks == 0) return HJD_OK;
    if (!d_coefs || !d_out) return fail(HJD_E_INVALID, "NULL device buffer");
    if ((reinterpret_cast<uintptr_t>(d_coefs) | reinterpret_cast<uintptr_t>(d_out)) & 15)
        return fail(HJD_E_INVALID, "device buffers must be 16-byte aligned");
    if (grid_blocks < 0) return fail(HJD_E_INVALID, "grid_blocks < 0");
    // hjd_plan_autotune's / hjd_plan_set_chunk's chunk, for plans that take the
    // persistent kernel anyway (a small AUTO plan keeps the latency kernel)
    if (grid_blocks == 0 && plan->tuned_grid > 0 && plan_is_persistent(plan)) grid_blocks = plan->tuned_grid;
    return hjd_internal::launch_decode(plan->ctx->device, plan->ctx->num_cu, plan->sampling, plan->input_format,
                                       plan->variant, d_coefs, plan->d_qt,
                                       reinterpret_cast<const hjd_internal::FrameRecord*>(plan->d_frames),
                                       plan->nframes, plan->tasks, d_out, stream, grid_blocks, plan->out_format,
                                       plan->kernel_mode);
}

// The fused kernel's launch adapted to the device it runs on (VERDICT r3:
// the same 4:2:0 kernel ran ~10 % slower on some MI355X boxes, its memory
// side with it, while 4:4:4 did not; which per-wave chunk and store policy
// keep HBM busiest differs by box and shape: profiles/r04c_tpw_sweep.json).
// Times every candidate -- 1, 2, 4, 8 and 16 tasks per wave x nt / plain
// output stores (BGRX) -- on the plan's own buffers, `rounds` interleaved
// rounds of one warm + two timed launches each, keeps the fastest (minimum
// over rounds) for the plan's later default launches.  All candidates give
// identical pixels.  Synchronous; plans small enough for the latency kernel
// are left as they are.
//
// The choice is cached per process: device x sampling x input format x output
// format x the plan's other variant bits x task-count octave (floor(log2
// tasks)).  A later plan of the same key takes the cached shape with no
// launch (the search cost ~1 s per plan).  HJD_AUTOTUNE_CACHE=0
// disables the cache; hjd_autotune_cache_clear() empties it.
namespace {
// A cached choice applies to plans of the same kernel and batch geometry
// (frame count and task count), not just the same size octave.
struct TuneKey {
    int device, sampling, input_format, out_format, keep_variant, nframes;
    int64_t tasks;
    bool operator<(const TuneKey& o) const
    {
        return std::tie(device, sampling, input_format, out_format, keep_variant, nframes, tasks) <
               std::tie(o.device, o.sampling, o.input_format, o.out_format, o.keep_variant, o.nframes, o.tasks);
    }
};
std::mutex g_tune_mu;
std::map<TuneKey, std::pair<int, int>> g_tune;   // -> (tasks per wave, store bit)

bool tune_cache_enabled()
{
    const char* e = getenv("HJD_AUTOTUNE_CACHE");
    return !(e && e[0] == '0');
}
}  // namespace

int hjd_autotune_cache_clear(void)
{
    std::lock_guard<std::mutex> lock(g_tune_mu);
    g_tune.clear();
    return HJD_OK;
}

int hjd_plan_autotune(hjd_plan* plan, const void* d_coefs, void* d_out, void* stream, int rounds,
                      int32_t* tasks_per_wave, int32_t* variant)
{
    if (!plan || rounds < 0 || rounds > 16) return fail(HJD_E_INVALID, "invalid autotune arguments");
    if (!d_coefs || !d_out || ((reinterpret_cast<uintptr_t>(d_coefs) | reinterpret_cast<uintptr_t>(d_out)) & 15))
        return fail(HJD_E_INVALID, "NULL or unaligned device buffer");
    if (rounds == 0) rounds = 2;
    auto report = [&]() {
        if (tasks_per_wave) *tasks_per_wave = plan->tuned_per_wave;
        if (variant) *variant = plan->variant;
        return HJD_OK;
    };
    plan->autotune_launches = 0;
    plan->autotune_cached = 0;
    if (plan->tasks == 0 || !plan_is_persistent(plan)) return report();
    const int keep = plan->variant & ~1;
    const TuneKey key{plan->ctx->device, plan->sampling, plan->input_format, plan->out_format, keep, plan->nframes,
                      plan->tasks};
    if (tune_cache_enabled()) {
        std::lock_guard<std::mutex> lock(g_tune_mu);
        auto it = g_tune.find(key);
        if (it != g_tune.end()) {
            plan->tuned_per_wave = it->second.first;
            plan->tuned_grid = grid_for_chunk(plan->tasks, it->second.first);
            plan->variant = keep | it->second.second;
            plan->autotune_cached = 1;
            return report();
        }
    }
    struct Cand {
        int64_t per_wave;   // tasks per wave
        int store;          // variant bit 0
        int grid;
        float best_ms;
    };
    std::vector<Cand> cands;
    for (int64_t pw : {1, 2, 4, 8, 16}) {
        const int g = grid_for_chunk(plan->tasks, pw);
        bool dup = false;
        for (const Cand& c : cands) dup |= c.grid == g;
        if (dup) continue;
        for (int st = 0; st < (plan->out_format == HJD_OUT_BGRX ? 2 : 1); ++st) cands.push_back({pw, st, g, 1e30f});
    }
    HJD_HIP(hipSetDevice(plan->ctx->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    hipEvent_t e0, e1;
    HJD_HIP(hipEventCreate(&e0));
    if (hipEventCreate(&e1) != hipSuccess) {
        (void)hipEventDestroy(e0);
        return fail(HJD_E_HIP, "hipEventCreate");
    }
    int rc = HJD_OK;
    for (int r = 0; r < rounds && rc == HJD_OK; ++r) {
        for (Cand& c : cands) {
            const int v = keep | c.store;
            auto go = [&]() {
                plan->autotune_launches++;
                return hjd_internal::launch_decode(plan->ctx->device, plan->ctx->num_cu, plan->sampling,
                                                   plan->input_format, v, d_coefs, plan->d_qt,
                                                   reinterpret_cast<const hjd_internal::FrameRecord*>(plan->d_frames),
                                                   plan->nframes, plan->tasks, d_out, s, c.grid, plan->out_format,
                                                   HJD_KERNEL_PERSISTENT);
            };
            float ms = 0;
            if ((rc = go()) || (rc = hipEventRecord(e0, s) == hipSuccess ? HJD_OK : HJD_E_HIP) || (rc = go()) ||
                (rc = go()) || (rc = hipEventRecord(e1, s) == hipSuccess ? HJD_OK : HJD_E_HIP) ||
                (rc = hipEventSynchronize(e1) == hipSuccess ? HJD_OK : HJD_E_HIP) ||
                (rc = hipEventElapsedTime(&ms, e0, e1) == hipSuccess ? HJD_OK : HJD_E_HIP))
                break;
            c.best_ms = std::min(c.best_ms, ms / 2);
        }
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (rc) return rc == HJD_E_HIP ? fail(HJD_E_HIP, "autotune timing failed") : rc;
    const Cand* best = &cands[0];
    for (const Cand& c : cands)
        if (c.best_ms < best->best_ms) best = &c;
    plan->tuned_grid = best->grid;
    plan->tuned_per_wave = static_cast<int>(best->per_wave);
    plan->variant = keep | best->store;
    if (tune_cache_enabled()) {
        std::lock_guard<std::mutex> lock(g_tune_mu);
        g_tune[key] = {static_cast<int>(best->per_wave), best->store};
    }
    return report();
}

int hjd_plan_launch_shape(const hjd_plan* plan, hjd_launch_shape* out)
{
    if (!plan || !out) return fail(HJD_E_INVALID, "invalid arguments");
    hjd_launch_shape r;
    memset(&r, 0, sizeof(r));
    r.variant = plan->variant;
    r.autotune_launches = plan->autotune_launches;
    r.autotune_cached = plan->autotune_cached;
    if (plan->tasks > 0 && !plan_is_persistent(plan)) {
        r.kernel = HJD_KERNEL_LATENCY;
        r.grid = static_cast<int32_t>(std::min<int64_t>(plan->tasks, INT32_MAX));
        r.tasks_per_wave = 1;
        r.max_tasks_per_wave = 1;
    } else {
        r.kernel = HJD_KERNEL_PERSISTENT;
        const int fmt = plan->input_format == HJD_IN_Q16_ZIGZAG ? 0 : 1;
        const int64_t t = std::max<int64_t>(plan->tasks, 1);
        const bool pinned = plan->tuned_grid > 0;
        r.tasks_per_wave = static_cast<int32_t>(
            pinned ? effective_per_wave(t, plan->tuned_per_wave, false)
                   : effective_per_wave(t, default_per_wave(plan->sampling, fmt), true));
        r.grid = pinned ? plan->tuned_grid : grid_for_chunk(t, default_per_wave(plan->sampling, fmt));
        if ((plan->variant & hjd::kVarWgInterleave) != 0) {   // groups take quads of tasks
            const int64_t quads = (t + hjd::kWavesPerGroup - 1) / hjd::kWavesPerGroup;
            r.max_tasks_per_wave = static_cast<int32_t>((quads + r.grid - 1) / r.grid);
        } else {
            const int64_t waves = static_cast<int64_t>(r.grid) * hjd::kWavesPerGroup;
            r.max_tasks_per_wave = static_cast<int32_t>((t + waves - 1) / waves);
        }
    }
    *out = r;
    return HJD_OK;
}

int hjd_debug_plan_launch_stages(hjd_plan* plan, int stages, const void* d_coefs, void* d_out, void* stream,
                                 int grid_blocks)
{
    if (!plan) return fail(HJD_E_INVALID, "plan is NULL");
    if (stages != 4 && stages != 16 && stages != 20 && stages != 64 && stages != 80 && stages != 8 && stages != 24 &&
        stages != 256)
        return fail(HJD_E_INVALID, "unknown stage variant %d", stages);
    if (plan->input_format != HJD_IN_Q16_ZIGZAG || plan->out_format != HJD_OUT_BGRX ||
        (plan->sampling != HJD_YUV420 && plan->sampling != HJD_YUV444))
        return fail(HJD_E_INVALID, "stage variants: 4:2:0 / 4:4:4, int16 zigzag in, BGRX out");
    if (plan->tasks == 0) return HJD_OK;
    if (!d_coefs || !d_out || ((reinterpret_cast<uintptr_t>(d_coefs) | reinterpret_cast<uintptr_t>(d_out)) & 15))
        return fail(HJD_E_INVALID, "NULL or unaligned device buffer");
    return hjd_internal::launch_decode(plan->ctx->device, plan->ctx->num_cu, plan->sampling, plan->input_format,
                                       stages << kStageShift, d_coefs, plan->d_qt,
                                       reinterpret_cast<const hjd_internal::FrameRecord*>(plan->d_frames),
                                       plan->nframes, plan->tasks, d_out, stream,
                                       grid_blocks > 0 ? grid_blocks : plan->tuned_grid,
                                       plan->out_format, HJD_KERNEL_PERSISTENT);
}

int hjd_idct_blocks(hjd_ctx* ctx, const int32_t* d_in, int32_t* d_out, int64_t nblocks, void* stream)
{
    if (!ctx || nblocks < 0 || ((!d_in || !d_out) && nblocks > 0)) return fail(HJD_E_INVALID, "invalid arguments");
    if (nblocks == 0) return HJD_OK;
    HJD_HIP(hipSetDevice(ctx->device));
    const int grid = default_grid(ctx, (nblocks + 7) / 8);
    hipLaunchKernelGGL(hjd::idct_blocks_kernel, dim3(grid), dim3(hjd::kGroupThreads), 0,
                       static_cast<hipStream_t>(stream), d_in, d_out, nblocks);
    HJD_HIP(hipGetLastError());
    return HJD_OK;
}

int hjd_debug_csc(hjd_ctx* ctx, const int32_t* d_y, const int32_t* d_u, const int32_t* d_v, uint32_t* d_out,
                  int64_t n, int mode, void* stream)
{
    if (!ctx || n < 0 || (mode != 0 && mode != 1)) return fail(HJD_E_INVALID, "invalid arguments");
    if (n == 0) return HJD_OK;
    HJD_HIP(hipSetDevice(ctx->device));
    const int grid = static_cast<int>(std::min<int64_t>((n + 255) / 256, 65536));
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (mode == 0)
        hipLaunchKernelGGL(hjd::csc_kernel<0>, dim3(grid), dim3(256), 0, s, d_y, d_u, d_v, d_out, n);
    else
        hipLaunchKernelGGL(hjd::csc_kernel<1>, dim3(grid), dim3(256), 0, s, d_y, d_u, d_v, d_out, n);
    HJD_HIP(hipGetLastError());
    return HJD_OK;
}

int hjd_debug_csc_exhaustive(hjd_ctx* ctx, uint32_t* d_out, int mode, void* stream)
{
    if (!ctx || !d_out || (mode != 0 && mode != 1)) return fail(HJD_E_INVALID, "invalid arguments");
    HJD_HIP(hipSetDevice(ctx->device));
    hipStream_t s = static_cast<hipStream_t>(stream);
    if (mode == 0)
        hipLaunchKernelGGL(hjd::csc_exhaustive_kernel<0>, dim3(8192), dim3(256), 0, s, d_out);
    else
        hipLaunchKernelGGL(hjd::csc_exhaustive_kernel<1>, dim3(8192), dim3(256), 0, s, d_out);
    HJD_HIP(hipGetLastError());
    return HJD_OK;
}

}  // extern "C"
