// hjd_internal.h -- helpers shared by the translation units of libhjd.so.
#pragma once
#include <stdint.h>

#include <vector>

struct hjd_ctx;
struct hjd_jpeg_info;

namespace hjd_internal {

// Record the calling thread's last error (returned by hjd_last_error()) and
// return `code`.  Defined in hjd_runtime.hip.
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Per-sampling geometry shared by the parser, the plans and the kernels.  A
// pixel-kernel task is always 48 coefficient blocks (hjd::kTaskBlocks).
struct SamplingGeom {
    int index;          // kernel template index: 0 4:4:4, 1 4:2:0, 2 4:2:2, 3 gray, 4 4:1:1, 5 4:4:0
    int mcu_px_w, mcu_px_h;
    int bpm;            // blocks per MCU
    int mcus_per_task;  // 48 / bpm
};
inline bool sampling_geom(int sampling, SamplingGeom* g)
{
    switch (sampling) {
    case 0: *g = {0, 8, 8, 3, 16}; return true;    // HJD_YUV444
    case 1: *g = {1, 16, 16, 6, 8}; return true;   // HJD_YUV420
    case 3: *g = {2, 16, 8, 4, 12}; return true;   // HJD_YUV422
    case 4: *g = {3, 8, 8, 1, 48}; return true;    // HJD_GRAY
    case 5: *g = {4, 32, 8, 6, 8}; return true;    // HJD_YUV411_H4V1
    case 6: *g = {5, 8, 16, 4, 12}; return true;   // HJD_YUV440
    default: return false;
    }
}

// Device frame record of the fused kernel (layout of hjd::FrameDev).
struct FrameRecord {
    int64_t coef_base, out_base, task_begin;
    int32_t width, height, pitch, sampling, mcu_w, strips;
    int32_t qt[3];
    int32_t vec_ok;
};

// Fill a one-frame record (task_begin 0); returns the frame's task count, or
// a negative status for an unsupported geometry.  out_format: HJD_OUT_*.
int64_t make_frame_record(int width, int height, int sampling, int64_t coef_base, int64_t out_base, int pitch,
                          const int qt_index[3], FrameRecord* rec, int out_format = 0);

// Launch the fused kernel on device-resident frame records / natural-order
// qtables (no host synchronisation, safe to call from any host thread).
int launch_decode(int device, int num_cu, int sampling, int input_format, int variant, const void* d_coefs,
                  const int32_t* d_qt_nat, const FrameRecord* d_frames, int nframes, int64_t tasks, void* d_out,
                  void* stream, int grid_blocks, int out_format = 0, int kernel_mode = 0);

// Bytes per output pixel of an HJD_OUT_* format (0 if unknown).
inline int out_format_bytes(int out_format) { return out_format == 0 ? 4 : out_format == 1 ? 3 : 0; }

// Rows of this format can take the kernel's full-width vector stores.
inline bool out_vector_ok(int out_format, int64_t pitch, int64_t out_base)
{
    return out_format == 1 ? ((pitch | out_base) & 3) == 0 : ((pitch | out_base) & 15) == 0;
}

// Parsed header of one sequential scan as the GPU entropy path needs it
// (jpeg_host.cpp).  File-level fields (width .. nblocks, out_bpm, qt) describe
// the whole image; the rest the scan.
struct ScanHeader {
    int width, height, sampling, restart_interval, mcu_w, mcu_h;
    int bpm;                     // blocks per MCU of this scan (1 for a non-interleaved scan)
    int out_bpm;                 // blocks per MCU of the image (the coefficient layout)
    int64_t nblocks;             // blocks of the image (mcu_w * mcu_h * out_bpm)
    int64_t scan_blocks;         // blocks this scan codes
    size_t scan_offset;          // first byte of entropy-coded data
    int32_t qt[3][64];           // per frame component, zigzag (file) order
    int jcomp[6], jdc[6], jac[6], jslot[6];   // per bitstream block of an MCU
    bool table_defined[2][4];    // [class: 0 DC, 1 AC][id]
    uint8_t counts[2][4][16];
    uint8_t symbols[2][4][256];
    int nsym[2][4];
    // Sequential files with several scans (T.81 B.2.3; an extension, the
    // reference takes one interleaved scan): `extra_scans` > 0 on the first
    // scan's header says how many more scans the frame can hold (<= 2, one per
    // component not in the first scan); parse_scan_headers() lists them.
    int extra_scans;
    int layout;                  // 0: MCU-interleaved; 1: one component in raster block order (A.2.2)
    int comp_bw, comp_bh;        // layout 1: the component's block grid
    int comp_lh, comp_lv;        // layout 1: log2 of its sampling factors
};
int parse_scan_header(const uint8_t* data, size_t size, ScanHeader* h);
// Every scan of a sequential file (hs[0] == what parse_scan_header gives).
// Progressive files fail.
int parse_scan_headers(const uint8_t* data, size_t size, std::vector<ScanHeader>* hs);

// Host Huffman decode of two files on the calling thread (jpeg_host.cpp): as
// two hjd_jpeg_decode_coefs calls, with the symbol steps of the two files
// interleaved when both are single-scan sequential files.  rc[i] per file.
int jpeg_decode_coefs_two(const uint8_t* const data[2], const size_t size[2], ::hjd_jpeg_info* const info[2],
                          int16_t* const coefs[2], const int64_t capacity[2], int rc[2]);

// hjd_ctx accessors for the other translation units
int ctx_num_cu(const struct ::hjd_ctx* ctx);

// d16 gather (hjd_probe.hip): d16_probe() is 1 if ds_read_u16_d16_hi zeroes
// the low half of its destination on `device` (one-wave probe; a completed run
// is cached per device, a failed one returns 0 and is retried next time;
// HJD_D16_PROBE=fail forces 0).  hjd_ctx_create runs it.  d16_probe_cached()
// never runs it: the cached answer, or -1.  d16_gather_selected(): whether
// the 4:4:4 launches take the kVarD16 kernels (the cached probe passed and
// HJD_D16 is not 0); a launch never runs the probe itself, so it stays legal
// inside stream capture.
int d16_probe(int device);
int d16_probe_cached(int device);
bool d16_gather_selected(int device);

}  // namespace hjd_internal

namespace hjd_internal {

// NUMA locality of a device's host-side workers: the CPUs
// of the NUMA node the GPU's PCIe device hangs off (sysfs), or an empty set
// when unknown.  bind_current_thread() applies such a set (no-op if empty)
// and returns the previous mask so a caller can restore it.
struct CpuSet {
    std::vector<int> cpus;
};
CpuSet device_local_cpus(int device);
// Default host worker count of a stream on `device` (nthreads = 0): the
// process's CPU share (hjd_host_cpu_share) capped by the device's CPU slice
// (device_local_cpus; uncapped when the topology is unknown).
int default_worker_threads(int device);
CpuSet node_cpus(int node);   // CPUs of NUMA node `node` this process may use (empty: unknown)
std::vector<int> bind_current_thread(const CpuSet& s);
void restore_current_thread(const std::vector<int>& prev);

}  // namespace hjd_internal

#ifndef __HIP_DEVICE_COMPILE__   // host code only (the device pass parses, never emits, its callers)
#include <immintrin.h>
#endif

namespace hjd_internal {

// The scan-copy step of both host destuff routines (jpeg_host.cpp
// destuff_scan, hjd_entropy.hip destuff): copy the bytes of [s, end) before
// the first 0xFF to o (advanced) and return where that 0xFF is (or end).
// AVX2 compares, 64 bytes per test while none is an 0xFF, instead of a memchr
// + memcpy call pair per run: entropy-coded data has an 0xFF every ~200 bytes,
// so the calls' overhead dominated.  Vector steps store whole vectors (bytes
// past the 0xFF are overwritten later) only while they fit before oend; the
// rest is copied bytewise.  Returns a position that is not an 0xFF and not
// end only when the output is full (o == oend).
#ifndef __HIP_DEVICE_COMPILE__
__attribute__((target("avx2"))) inline const uint8_t* copy_until_ff_avx2(const uint8_t* s, const uint8_t* end,
                                                                          uint8_t*& o, uint8_t* oend)
{
    const __m256i ff = _mm256_set1_epi8(static_cast<char>(0xFF));
    while (end - s >= 64 && oend - o >= 64) {
        const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s));
        const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + 32));
        const uint32_t ma = static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(a, ff)));
        const uint32_t mb = static_cast<uint32_t>(_mm256_movemask_epi8(_mm256_cmpeq_epi8(b, ff)));
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(o), a);
        _mm256_storeu_si256(reinterpret_cast<__m256i*>(o + 32), b);
        if (ma | mb) {
            const uint64_t m = (static_cast<uint64_t>(mb) << 32) | ma;
            const int k = __builtin_ctzll(m);
            o += k;
            return s + k;
        }
        s += 64;
        o += 64;
    }
    return s;
}
#endif

inline const uint8_t* copy_until_ff(const uint8_t* s, const uint8_t* end, uint8_t*& o, uint8_t* oend)
{
#ifndef __HIP_DEVICE_COMPILE__
    static const bool avx2 = [] {
        __builtin_cpu_init();
        return __builtin_cpu_supports("avx2") != 0;
    }();
    if (avx2) {
        s = copy_until_ff_avx2(s, end, o, oend);
        if (s < end && *s == 0xFF) return s;
    }
#endif
    while (s < end && *s != 0xFF && o < oend) *o++ = *s++;
    return s;
}

}  // namespace hjd_internal
