// hjd_probe.hip -- measurement and hardware-probe kernels of libhjd.so.
//
// 1. hjd_debug_rw_mix: the box's own streaming ceiling for a read:write byte
//    mix.  The fused kernel moves 6 KiB in + 8 KiB out per 4:2:0 task and
//    6 KiB in + 4 KiB out per 4:4:4 task; this kernel moves the
//    same mixes as pure streams (16 B per lane, coalesced, nt by default,
//    oversubscribed in-order grid, XCD-contiguous order -- the fused kernel's
//    own launch shape) with no compute, so bench.py can state the fraction of
//    THIS box's achievable rate next to the fraction of the 8 TB/s spec.
// 2. The d16 gather probe: the 4:4:4 kernels gather coefficient pairs with
//    ds_read_u16_d16_hi, which is only a valid gather where that load zeroes
//    the low half of its destination (sramecc+ parts).  hjd_ctx_create runs a
//    one-wave probe per device (eagerly, outside any launch or stream capture)
//    and the launches take the kVarD16 kernels only if it completed and every
//    lane saw the low half zeroed (hjd_runtime.hip d16_gather_selected).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>

#include "hjd.h"
#include "hjd_internal.h"

namespace {

constexpr int kRwWaves = 4;   // waves per 256-thread group

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// The fused kernel's XCD-contiguous group order (hjd_kernels.hpp group_order,
// default HJD_XCD_CHUNK 0): XCD x = bid % 8 owns one contiguous eighth.
__device__ __forceinline__ uint32_t xcd_order(uint32_t bid, uint32_t ngroups)
{
    const uint32_t x = bid & 7, k = bid >> 3, q = ngroups >> 3, rem = ngroups & 7;
    return x * q + min(x, rem) + k;
}

// Each wave moves `upw` consecutive units; unit u reads R KiB at src + u*R KiB
// and writes W KiB at dst + u*W KiB (16 B per lane per KiB).  The loaded data
// feeds every store, so no load is dead.  flags bit 2 (pipelined): the next
// unit's loads are issued before this unit's stores, the fused kernel's
// one-task-ahead prefetch; otherwise each unit loads, then stores.
// Stores of unit u.  Contiguous: W KiB at dst + u*W KiB.  Image rows (flags
// bit 3): the fused kernel's store geometry -- dst is a stack of 3840-px BGRX
// images (pitch 15360 B = 30 strips of 512 B); unit u is strip u % 30 of row
// band u / 30 (2W rows), and each wave store instruction writes two 512-B row
// segments (lanes 0-31 one row, lanes 32-63 the next).
template <int R, int W>
__device__ __forceinline__ void rw_store(u32x4* __restrict__ dst, int64_t u, int lane, u32x4 acc, bool nt, bool rows)
{
    constexpr int64_t kPitch = 15360 / 16, kStrips = 30;   // in 16-B words
    u32x4* d = rows ? dst + (u / kStrips) * (2 * W) * kPitch + (u % kStrips) * 32 + (lane >> 5) * kPitch + (lane & 31)
                    : dst + u * W * 64 + lane;
#pragma unroll
    for (int k = 0; k < W; ++k) {
        u32x4 o = acc;
        o.y += static_cast<unsigned>(k);
        u32x4* q = rows ? d + 2 * k * kPitch : d + 64 * k;
        if (nt)
            __builtin_nontemporal_store(o, q);
        else
            *q = o;
    }
}

template <int R>
__device__ __forceinline__ void rw_load(const u32x4* __restrict__ src, int64_t u, int lane, u32x4 (&v)[R > 0 ? R : 1],
                                        bool nt)
{
    const u32x4* s = src + u * R * 64 + lane;
#pragma unroll
    for (int k = 0; k < R; ++k) v[k] = nt ? __builtin_nontemporal_load(s + 64 * k) : s[64 * k];
}

template <int R, int W>
__global__ __launch_bounds__(256) void rw_mix_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                     int64_t units, int upw, int flags)
{
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const uint32_t grp = (flags & 2) ? xcd_order(blockIdx.x, gridDim.x) : blockIdx.x;
    const int64_t gw = static_cast<int64_t>(grp) * kRwWaves + wave;
    const int64_t u0 = gw * upw;
    const int64_t u1 = u0 + upw < units ? u0 + upw : units;
    const bool nt = (flags & 1) != 0;
    const bool rows = (flags & 8) != 0;
    if constexpr (R > 0 && W > 0) {
        if (flags & 4) {   // pipelined
            u32x4 cur[R], nxt[R];
            if (u0 < u1) rw_load<R>(src, u0, lane, cur, nt);
            for (int64_t u = u0; u < u1; ++u) {
                if (u + 1 < u1) rw_load<R>(src, u + 1, lane, nxt, nt);
                u32x4 acc = {static_cast<unsigned>(lane), 0u, 0u, static_cast<unsigned>(u)};
#pragma unroll
                for (int k = 0; k < R; ++k) acc ^= cur[k];
                rw_store<R, W>(dst, u, lane, acc, nt, rows);
#pragma unroll
                for (int k = 0; k < R; ++k) cur[k] = nxt[k];
            }
            return;
        }
    }
    for (int64_t u = u0; u < u1; ++u) {
        u32x4 acc = {static_cast<unsigned>(lane), 0u, 0u, static_cast<unsigned>(u)};
        if constexpr (R > 0) {
            u32x4 v[R];
            rw_load<R>(src, u, lane, v, nt);
#pragma unroll
            for (int k = 0; k < R; ++k) acc ^= v[k];
        }
        if constexpr (W > 0) {
            rw_store<R, W>(dst, u, lane, acc, nt, rows);
        } else {
            // read-only mix: keep the loads alive without a store per unit (a
            // data-dependent condition the compiler cannot fold; dst >= 1 KiB)
            if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == static_cast<unsigned>(units) * 2654435761u) dst[lane] = acc;
        }
    }
}

// One wave: every lane presets its destination word's low half, loads a u16
// from LDS into the high half with ds_read_u16_d16_hi and waits for it inside
// the same asm statement, then stores the word.  Zeroing parts give
// (value << 16); half-preserving parts give (value << 16) | preset.
__global__ __launch_bounds__(64) void d16_probe_kernel(uint32_t* __restrict__ out)
{
    __shared__ unsigned short buf[64];
    const int lane = threadIdx.x;
    buf[lane] = static_cast<unsigned short>(0x1234 + 3 * lane);
    __syncthreads();
    uint32_t v = 0x5a5au + static_cast<uint32_t>(lane);
    const uint32_t addr = static_cast<uint32_t>(reinterpret_cast<size_t>(&buf[63 - lane]));
    asm volatile("ds_read_u16_d16_hi %0, %1\n\ts_waitcnt lgkmcnt(0)" : "+v"(v) : "v"(addr) : "memory");
    out[lane] = v;
}

// Clock probe (bench.py's sclk under load): one lane samples the shader-clock
// counter (s_memtime) and the 100-MHz real-time counter (s_memrealtime) every
// `interval` real-time ticks, `nsamples` times, and stores each pair with a
// vector store.  Bounded: it ends after nsamples * interval ticks.  Launched
// on a side stream beside the pixel kernel, its sample pairs give the clock
// the chip holds while that kernel runs (MI355X lowers it under load).
__global__ __launch_bounds__(64) void clock_probe_kernel(unsigned long long* __restrict__ out, int nsamples,
                                                         int interval)
{
    if (threadIdx.x != 0) return;
    unsigned long long next = __builtin_amdgcn_s_memrealtime();
    for (int i = 0; i < nsamples; ++i) {
        next += static_cast<unsigned long long>(interval);
        unsigned long long r;
        do {
            __builtin_amdgcn_s_sleep(8);
            r = __builtin_amdgcn_s_memrealtime();
        } while (r < next);
        const unsigned long long c = __builtin_amdgcn_s_memtime();
        out[2 * i] = r;
        out[2 * i + 1] = c;
    }
}

std::mutex g_probe_mu;
std::vector<int> g_probe;   // per device: -1 not run (or the run failed), 0 preserves, 1 zeroes

// A failed HIP call inside the probe must not leave its error behind for the
// caller's next hipGetLastError() (a launch would then report a failure of
// the probe as its own).
int probe_failed(int prev)
{
    (void)hipGetLastError();
    (void)hipSetDevice(prev);
    (void)hipGetLastError();
    return -1;
}

// One run of the probe on `device`: 1 zeroes, 0 preserves, -1 could not run
// (HIP error, cleared).  HJD_D16_PROBE=hipfail makes the first HIP call fail
// for real (an allocation no device can satisfy): the test of the failure path.
int run_probe(int device)
{
    int prev = 0;
    if (hipGetDevice(&prev) != hipSuccess) return probe_failed(0);
    if (hipSetDevice(device) != hipSuccess) return probe_failed(prev);
    const char* force = getenv("HJD_D16_PROBE");
    const size_t bytes = (force && strcmp(force, "hipfail") == 0) ? (size_t(1) << 60) : 64 * sizeof(uint32_t);
    uint32_t* d = nullptr;
    if (hipMalloc(&d, bytes) != hipSuccess) return probe_failed(prev);
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        (void)hipFree(d);
        return probe_failed(prev);
    }
    hipLaunchKernelGGL(d16_probe_kernel, dim3(1), dim3(64), 0, s, d);
    uint32_t h[64];
    int result = -1;
    if (hipGetLastError() == hipSuccess && hipMemcpyAsync(h, d, sizeof(h), hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess) {
        result = 1;
        for (int lane = 0; lane < 64; ++lane)
            if (h[lane] != static_cast<uint32_t>(0x1234 + 3 * (63 - lane)) << 16) result = 0;
    }
    const bool ok = hipStreamDestroy(s) == hipSuccess && hipFree(d) == hipSuccess && result >= 0;
    if (!ok) return probe_failed(prev);
    (void)hipSetDevice(prev);
    return result;
}

}  // namespace

// 1 if ds_read_u16_d16_hi zeroes the low half on `device` (every lane), 0 if it
// does not or the probe could not run.  A completed probe is cached per device;
// a failed one is not (the next call -- the next hjd_ctx_create -- tries
// again).  HJD_D16_PROBE=fail forces 0 (tests of the fallback).
int hjd_internal::d16_probe(int device)
{
    std::lock_guard<std::mutex> lock(g_probe_mu);
    if (device < 0) return 0;
    if (static_cast<size_t>(device) >= g_probe.size()) g_probe.resize(device + 1, -1);
    if (g_probe[device] >= 0) return g_probe[device];
    const char* force = getenv("HJD_D16_PROBE");
    if (force && strcmp(force, "fail") == 0) {
        g_probe[device] = 0;
        return 0;
    }
    const int r = run_probe(device);
    if (r >= 0) g_probe[device] = r;
    return r > 0 ? 1 : 0;
}

int hjd_internal::d16_probe_cached(int device)
{
    std::lock_guard<std::mutex> lock(g_probe_mu);
    if (device < 0 || static_cast<size_t>(device) >= g_probe.size()) return -1;
    return g_probe[device];
}

extern "C" {

int hjd_debug_rw_mix(hjd_ctx* ctx, const void* d_src, void* d_dst, int64_t src_bytes, int64_t dst_bytes,
                     int read_kib, int write_kib, int units_per_wave, int flags, void* stream, int64_t* units_out)
{
    if (!ctx || units_per_wave <= 0 || (flags & ~15)) return hjd_internal::set_error(HJD_E_INVALID, "invalid arguments");
    using K = void (*)(const u32x4*, u32x4*, int64_t, int, int);
    K k = nullptr;
    if (read_kib == 6 && write_kib == 8) k = rw_mix_kernel<6, 8>;
    else if (read_kib == 6 && write_kib == 4) k = rw_mix_kernel<6, 4>;
    else if (read_kib == 0 && write_kib == 8) k = rw_mix_kernel<0, 8>;
    else if (read_kib == 6 && write_kib == 0) k = rw_mix_kernel<6, 0>;
    else if (read_kib == 4 && write_kib == 4) k = rw_mix_kernel<4, 4>;
    else if (read_kib == 3 && write_kib == 4) k = rw_mix_kernel<3, 4>;
    else
        return hjd_internal::set_error(HJD_E_INVALID, "unsupported mix %d:%d KiB (6:8, 6:4, 0:8, 6:0, 4:4, 3:4)",
                                       read_kib, write_kib);
    int64_t units = INT64_MAX;
    if (read_kib > 0) units = std::min<int64_t>(units, src_bytes / (1024 * read_kib));
    if (write_kib > 0) units = std::min<int64_t>(units, dst_bytes / (1024 * write_kib));
    if (flags & 8) {   // image rows: whole bands of 30 strips
        if (write_kib == 0) return hjd_internal::set_error(HJD_E_INVALID, "image-row stores need a write mix");
        units = units / 30 * 30;
    }
    if (units <= 0 || !d_dst || dst_bytes < 1024 || (read_kib > 0 && !d_src)) return hjd_internal::set_error(HJD_E_INVALID, "buffers too small");
    if ((reinterpret_cast<uintptr_t>(d_src) | reinterpret_cast<uintptr_t>(d_dst)) & 15)
        return hjd_internal::set_error(HJD_E_INVALID, "buffers must be 16-byte aligned");
    const int64_t waves = (units + units_per_wave - 1) / units_per_wave;
    const int64_t groups = (waves + kRwWaves - 1) / kRwWaves;
    if (groups > (int64_t(1) << 30)) return hjd_internal::set_error(HJD_E_INVALID, "grid too large");
    if (hipSetDevice(hjd_ctx_device(ctx)) != hipSuccess) return hjd_internal::set_error(HJD_E_HIP, "hipSetDevice");
    hipLaunchKernelGGL(k, dim3(static_cast<uint32_t>(groups)), dim3(256), 0, static_cast<hipStream_t>(stream),
                       static_cast<const u32x4*>(d_src), static_cast<u32x4*>(d_dst), units, units_per_wave, flags);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hjd_internal::set_error(HJD_E_HIP, "rw_mix launch: %s", hipGetErrorString(e));
    if (units_out) *units_out = units;
    return HJD_OK;
}

int hjd_debug_clock_probe(hjd_ctx* ctx, uint64_t* d_out, int nsamples, int interval_ticks, void* stream)
{
    if (!ctx || !d_out || nsamples <= 0 || nsamples > 1000000 || interval_ticks < 100 || interval_ticks > 10000000)
        return hjd_internal::set_error(HJD_E_INVALID, "invalid clock probe arguments");
    if (hipSetDevice(hjd_ctx_device(ctx)) != hipSuccess) return hjd_internal::set_error(HJD_E_HIP, "hipSetDevice");
    hipLaunchKernelGGL(clock_probe_kernel, dim3(1), dim3(64), 0, static_cast<hipStream_t>(stream),
                       reinterpret_cast<unsigned long long*>(d_out), nsamples, interval_ticks);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hjd_internal::set_error(HJD_E_HIP, "clock probe launch: %s", hipGetErrorString(e));
    return HJD_OK;
}

int hjd_debug_d16_gather(int device, int* probe_zeroes, int* selected)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n)
        return hjd_internal::set_error(HJD_E_NO_DEVICE, "device %d not present", device);
    if (probe_zeroes) *probe_zeroes = hjd_internal::d16_probe(device);
    if (selected) *selected = hjd_internal::d16_gather_selected(device) ? 1 : 0;
    return HJD_OK;
}

}  // extern "C"
