// stream_pipeline.hip -- host Huffman || H2D || fused kernel (include/hjd_host.h).
//
// The reference runs parse -> Huffman -> one blocking upload -> kernel ->
// blocking read-back strictly in sequence for one image (src/parser.cpp:375-397,
// src/decoder.cpp:352-416).  Here every submitted JPEG becomes a job:
//   worker thread:  Huffman-decode into pinned slot s (job j uses s = j % nslots)
//                   together with its frame record + natural-order qtables;
//   copy stream:    one hipMemcpyAsync of the slot to device slot s;
//   compute stream: the fused kernel reads device slot s, writes the caller's
//                   BGRX buffer.
// Slot reuse is ordered by events: the host waits for job j-nslots' upload
// before refilling pinned slot s, and the upload of job j waits (on the GPU)
// for job j-nslots' kernel before overwriting device slot s.
// Every upload and kernel is bracketed by timing events (2 * nslots sets,
// harvested by the job 2 * nslots later, whose kernel wait is long over, or
// at sync; the ordering events carry no timing): hjd_stream_busy reports how long the copy
// engine and the kernels were busy, i.e. how much of the wall time the
// pipeline kept the GPU side fed (bench.py config5_stream_host).
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <thread>
#include <vector>

#include "hjd.h"
#include "hjd_host.h"
#include "hjd_internal.h"

using hjd_internal::FrameRecord;
using hjd_internal::set_error;

namespace {

constexpr size_t kHeader = 1024;   // [FrameRecord | pad][qt natural 3x64 int32][pad] then coefficients
constexpr size_t kQtOffset = 256;

constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Job {
    int64_t index;
    const uint8_t* data;
    size_t size;
    void* d_out;
    int32_t pitch;
    int out_format;   // HJD_OUT_* at submit time
};

}  // namespace

struct hjd_stream {
    hjd_ctx* ctx = nullptr;
    int device = 0, num_cu = 256;
    int64_t max_blocks = 0;
    size_t slot_bytes = 0;
    int nslots = 0;
    std::vector<uint8_t*> host;      // pinned staging
    std::vector<uint8_t*> dev;       // device slots
    std::vector<hipEvent_t> h2d_done, kernel_done;     // per slot, ordering only (no timing)
    // Timing brackets of job j in set j % (2 * nslots): harvested when job
    // j + 2 * nslots is issued, whose acquire() already waited for job j's
    // kernel (job j + nslots's copy waits on it), so harvesting never blocks.
    std::vector<hipEvent_t> t_h2d0, t_h2d1, t_k0, t_k1;
    std::vector<char> timed_pending;    // the set holds a job's unharvested timing events
    std::vector<int64_t> slot_issued;   // last job index whose GPU work was issued on the slot
    hipStream_t copy = nullptr, compute = nullptr;

    std::mutex mu;
    std::condition_variable cv_jobs, cv_slots, cv_idle;
    std::deque<Job> queue;
    int64_t submitted = 0, finished = 0;
    bool stop = false;
    std::vector<std::thread> workers;

    std::atomic<int64_t> images{0}, pixels{0}, decode_ns{0}, h2d_bytes{0}, launches{0};
    std::atomic<int64_t> h2d_busy_ns{0}, kernel_busy_ns{0};
    std::atomic<int> out_format{HJD_OUT_BGRX};   // for subsequent submits
    int first_error = HJD_OK;
    std::string first_error_msg;

    void record_error(int rc, const char* msg)
    {
        std::lock_guard<std::mutex> g(mu);
        if (first_error == HJD_OK) {
            first_error = rc;
            first_error_msg = msg;
        }
    }

    int acquire(const Job& job);
    int issue(const Job& job, int rc, const hjd_jpeg_info& info);
    void worker();
    void harvest(int t);
};

// Add timing set t's job's copy and kernel durations to the busy totals.  The
// caller owns the set (the job 2 * nslots later, or sync with every job
// finished); the kernel it times has finished by then.
void hjd_stream::harvest(int t)
{
    if (!timed_pending[t]) return;
    timed_pending[t] = 0;
    float copy_ms = 0, kernel_ms = 0;
    if (hipEventSynchronize(t_k1[t]) != hipSuccess || hipEventElapsedTime(&copy_ms, t_h2d0[t], t_h2d1[t]) != hipSuccess ||
        hipEventElapsedTime(&kernel_ms, t_k0[t], t_k1[t]) != hipSuccess) {
        (void)hipGetLastError();
        return;
    }
    h2d_busy_ns += static_cast<int64_t>(copy_ms * 1e6);
    kernel_busy_ns += static_cast<int64_t>(kernel_ms * 1e6);
}

int hjd_stream::acquire(const Job& job)
{
    const int s = static_cast<int>(job.index % nslots);
    {   // wait until the previous job on this slot has issued its GPU work
        std::unique_lock<std::mutex> lk(mu);
        cv_slots.wait(lk, [&] { return slot_issued[s] == job.index - nslots || stop; });
    }
    if (hipSetDevice(device) != hipSuccess) return set_error(HJD_E_HIP, "hipSetDevice");
    if (job.index >= nslots && hipEventSynchronize(h2d_done[s]) != hipSuccess)   // pinned slot free
        return set_error(HJD_E_HIP, "hipEventSynchronize(h2d)");
    return HJD_OK;
}

int hjd_stream::issue(const Job& job, int rc, const hjd_jpeg_info& info)
{
    const int s = static_cast<int>(job.index % nslots);
    uint8_t* h = host[s];
    if (rc == HJD_OK && job.pitch < hjd_internal::out_format_bytes(job.out_format) * info.width)
        rc = set_error(HJD_E_INVALID, "output pitch too small");

    const size_t coef_bytes = rc == HJD_OK ? static_cast<size_t>(info.nblocks) * 128 : 0;
    int64_t tasks = 0;
    if (rc == HJD_OK) {
        FrameRecord rec;
        const int qti[3] = {0, 1, 2};
        tasks = hjd_internal::make_frame_record(info.width, info.height, info.sampling, 0,
                                                0, job.pitch, qti, &rec, job.out_format);
        if (tasks < 0) rc = static_cast<int>(tasks);
        memcpy(h, &rec, sizeof(rec));
        int32_t* qn = reinterpret_cast<int32_t*>(h + kQtOffset);
        for (int c = 0; c < 3; ++c)
            for (int k = 0; k < 64; ++k) qn[c * 64 + kZigzag[k]] = info.qt[c][k];
    }

    const int t = static_cast<int>(job.index % (2 * nslots));
    harvest(t);   // the job issued 2 * nslots ago (finished: see t_h2d0)
    // Issue the GPU work (also on failure, with nothing to do, so the slot's
    // event chain stays intact for the next job).
    const bool work = rc == HJD_OK && tasks > 0;
    hipError_t e = hipStreamWaitEvent(copy, kernel_done[s], 0);
    if (e == hipSuccess && work) e = hipEventRecord(t_h2d0[t], copy);
    if (e == hipSuccess && rc == HJD_OK)
        e = hipMemcpyAsync(dev[s], h, kHeader + coef_bytes, hipMemcpyHostToDevice, copy);
    if (e == hipSuccess && work) e = hipEventRecord(t_h2d1[t], copy);
    if (e == hipSuccess) e = hipEventRecord(h2d_done[s], copy);
    if (e == hipSuccess) e = hipStreamWaitEvent(compute, h2d_done[s], 0);
    if (e == hipSuccess && work) e = hipEventRecord(t_k0[t], compute);
    int lrc = HJD_OK;
    if (e == hipSuccess && work) {
        lrc = hjd_internal::launch_decode(device, num_cu, info.sampling, HJD_IN_Q16_ZIGZAG, 0, dev[s] + kHeader,
                                          reinterpret_cast<const int32_t*>(dev[s] + kQtOffset),
                                          reinterpret_cast<const FrameRecord*>(dev[s]), 1, tasks, job.d_out,
                                          compute, 0, job.out_format);
        launches++;
    }
    if (e == hipSuccess && work) e = hipEventRecord(t_k1[t], compute);
    if (e == hipSuccess) e = hipEventRecord(kernel_done[s], compute);
    timed_pending[t] = e == hipSuccess && work && lrc == HJD_OK;
    {   // always marked issued, so the slot's next job never waits on a failed one
        std::lock_guard<std::mutex> g(mu);
        slot_issued[s] = job.index;
    }
    cv_slots.notify_all();
    if (e != hipSuccess) return set_error(HJD_E_HIP, "stream issue: %s", hipGetErrorString(e));
    if (rc != HJD_OK) return rc;
    if (lrc != HJD_OK) return lrc;
    images++;
    pixels += static_cast<int64_t>(info.width) * info.height;
    h2d_bytes += static_cast<int64_t>(kHeader + coef_bytes);
    return HJD_OK;
}

// A worker takes the next two jobs when two are queued and decodes them on
// its thread with their Huffman steps interleaved (jpeg_decode_coefs_two,
// +10 % per thread), then issues them in order; HJD_STREAM_PAIR=0 takes one at
// a time.  Consecutive jobs use different slots (nslots >= 2), and a pair only
// waits for jobs older than itself, so the oldest pair in flight can always
// proceed.
void hjd_stream::worker()
{
    static const bool pair = [] {
        const char* e = getenv("HJD_STREAM_PAIR");
        return !(e && e[0] == '0');
    }();
    for (;;) {
        Job jobs[2];
        int n = 0;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_jobs.wait(lk, [&] { return stop || !queue.empty(); });
            if (queue.empty()) return;
            jobs[n++] = queue.front();
            queue.pop_front();
            if (pair && !queue.empty()) {
                jobs[n++] = queue.front();
                queue.pop_front();
            }
        }
        int rc[2] = {HJD_OK, HJD_OK};
        hjd_jpeg_info info[2];
        for (int i = 0; i < n; ++i) rc[i] = acquire(jobs[i]);
        int16_t* coefs[2];
        for (int i = 0; i < n; ++i) coefs[i] = reinterpret_cast<int16_t*>(host[jobs[i].index % nslots] + kHeader);
        const auto t0 = std::chrono::steady_clock::now();
        if (n == 2 && rc[0] == HJD_OK && rc[1] == HJD_OK) {
            const uint8_t* d[2] = {jobs[0].data, jobs[1].data};
            const size_t sz[2] = {jobs[0].size, jobs[1].size};
            hjd_jpeg_info* ip[2] = {&info[0], &info[1]};
            const int64_t cap[2] = {max_blocks, max_blocks};
            hjd_internal::jpeg_decode_coefs_two(d, sz, ip, coefs, cap, rc);
        } else {
            for (int i = 0; i < n; ++i)
                if (rc[i] == HJD_OK)
                    rc[i] = hjd_jpeg_decode_coefs(jobs[i].data, jobs[i].size, &info[i], coefs[i], max_blocks);
        }
        decode_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        // In a pair whose files both failed, the thread's last error is the
        // second file's: decode the first alone again (errors are rare) so the
        // stream records the first failing job's own message.
        if (n == 2 && rc[0] != HJD_OK && rc[1] != HJD_OK && rc[0] != HJD_E_HIP)
            (void)hjd_jpeg_decode_coefs(jobs[0].data, jobs[0].size, &info[0], coefs[0], max_blocks);
        for (int i = 0; i < n; ++i) {
            rc[i] = issue(jobs[i], rc[i], info[i]);
            if (rc[i] != HJD_OK) record_error(rc[i], hjd_last_error());
        }
        {
            std::lock_guard<std::mutex> g(mu);
            finished += n;
        }
        cv_idle.notify_all();
    }
}

extern "C" {

int hjd_stream_create(hjd_ctx* ctx, int64_t max_blocks, int nslots, int nthreads, hjd_stream** out)
{
    if (!ctx || !out || max_blocks <= 0 || nslots < 2) return set_error(HJD_E_INVALID, "invalid stream arguments");
    *out = nullptr;
    if (nthreads <= 0) nthreads = hjd_internal::default_worker_threads(hjd_ctx_device(ctx));
    hjd_stream* st = new (std::nothrow) hjd_stream;
    if (!st) return set_error(HJD_E_NOMEM, "stream allocation");
    st->ctx = ctx;
    st->device = hjd_ctx_device(ctx);
    st->num_cu = hjd_internal::ctx_num_cu(ctx);
    st->max_blocks = max_blocks;
    st->slot_bytes = kHeader + static_cast<size_t>(max_blocks) * 128;
    st->nslots = nslots;
    auto bail = [&](const char* what, hipError_t e) {
        hjd_stream_destroy(st);
        return set_error(HJD_E_HIP, "%s: %s", what, hipGetErrorString(e));
    };
    hipError_t e = hipSetDevice(st->device);
    if (e != hipSuccess) return bail("hipSetDevice", e);
    if ((e = hipStreamCreateWithFlags(&st->copy, hipStreamNonBlocking)) != hipSuccess) return bail("stream", e);
    if ((e = hipStreamCreateWithFlags(&st->compute, hipStreamNonBlocking)) != hipSuccess) return bail("stream", e);
    st->host.assign(nslots, nullptr);
    st->dev.assign(nslots, nullptr);
    st->h2d_done.assign(nslots, nullptr);
    st->kernel_done.assign(nslots, nullptr);
    for (auto* v : {&st->t_h2d0, &st->t_h2d1, &st->t_k0, &st->t_k1}) v->assign(2 * nslots, nullptr);
    st->timed_pending.assign(2 * nslots, 0);
    st->slot_issued.assign(nslots, 0);
    for (int s = 0; s < nslots; ++s) {
        st->slot_issued[s] = s - nslots;
        if ((e = hipHostMalloc(reinterpret_cast<void**>(&st->host[s]), st->slot_bytes, hipHostMallocDefault)) !=
            hipSuccess)
            return bail("hipHostMalloc", e);
        if ((e = hipMalloc(reinterpret_cast<void**>(&st->dev[s]), st->slot_bytes)) != hipSuccess)
            return bail("hipMalloc", e);
        if ((e = hipEventCreateWithFlags(&st->h2d_done[s], hipEventDisableTiming)) != hipSuccess) return bail("event", e);
        if ((e = hipEventCreateWithFlags(&st->kernel_done[s], hipEventDisableTiming)) != hipSuccess)
            return bail("event", e);
    }
    for (int t = 0; t < 2 * nslots; ++t)
        for (auto* v : {&st->t_h2d0, &st->t_h2d1, &st->t_k0, &st->t_k1})
            if ((e = hipEventCreate(&(*v)[t])) != hipSuccess) return bail("event", e);
    // NUMA-local workers; HJD_NUMA=0 disables
    const char* numa_env = getenv("HJD_NUMA");
    const hjd_internal::CpuSet local = (numa_env && numa_env[0] == '0') ? hjd_internal::CpuSet{}
                                                                       : hjd_internal::device_local_cpus(st->device);
    for (int t = 0; t < nthreads; ++t)
        st->workers.emplace_back([st, local] {
            hjd_internal::bind_current_thread(local);
            st->worker();
        });
    *out = st;
    return HJD_OK;
}

int hjd_stream_destroy(hjd_stream* st)
{
    if (!st) return HJD_OK;
    {
        std::lock_guard<std::mutex> g(st->mu);
        st->stop = true;
    }
    st->cv_jobs.notify_all();
    st->cv_slots.notify_all();
    for (auto& t : st->workers) t.join();
    (void)hipSetDevice(st->device);
    if (st->compute) (void)hipStreamSynchronize(st->compute);
    if (st->copy) (void)hipStreamSynchronize(st->copy);
    for (size_t s = 0; s < st->host.size(); ++s) {
        if (st->host[s]) (void)hipHostFree(st->host[s]);
        if (st->dev[s]) (void)hipFree(st->dev[s]);
        if (st->h2d_done[s]) (void)hipEventDestroy(st->h2d_done[s]);
        if (st->kernel_done[s]) (void)hipEventDestroy(st->kernel_done[s]);
    }
    for (auto* v : {&st->t_h2d0, &st->t_h2d1, &st->t_k0, &st->t_k1})
        for (hipEvent_t ev : *v)
            if (ev) (void)hipEventDestroy(ev);
    if (st->copy) (void)hipStreamDestroy(st->copy);
    if (st->compute) (void)hipStreamDestroy(st->compute);
    delete st;
    return HJD_OK;
}

int hjd_stream_submit(hjd_stream* st, const uint8_t* data, size_t size, void* d_out, int32_t out_pitch)
{
    const int fmt = st ? st->out_format.load() : HJD_OUT_BGRX;
    const uintptr_t amask = fmt == HJD_OUT_BGR24 ? 3 : 15;
    if (!st || !data || !d_out || out_pitch <= 0 || (out_pitch & 3) || (reinterpret_cast<uintptr_t>(d_out) & amask))
        return set_error(HJD_E_INVALID, "invalid submit arguments (d_out must be 16-byte (BGR24: 4-byte) aligned)");
    {
        std::lock_guard<std::mutex> g(st->mu);
        st->queue.push_back(Job{st->submitted++, data, size, d_out, out_pitch, fmt});
    }
    st->cv_jobs.notify_one();
    return HJD_OK;
}

int hjd_stream_set_output_format(hjd_stream* st, int out_format)
{
    if (!st) return set_error(HJD_E_INVALID, "stream is NULL");
    if (!hjd_internal::out_format_bytes(out_format)) return set_error(HJD_E_INVALID, "unknown output format %d", out_format);
    st->out_format = out_format;   // each job keeps the format it was submitted with
    return HJD_OK;
}

int hjd_stream_sync(hjd_stream* st, int64_t stats[5])
{
    if (!st) return set_error(HJD_E_INVALID, "stream is NULL");
    {
        std::unique_lock<std::mutex> lk(st->mu);
        st->cv_idle.wait(lk, [&] { return st->finished == st->submitted; });
    }
    hipError_t e = hipSetDevice(st->device);
    if (e == hipSuccess) e = hipStreamSynchronize(st->compute);
    if (e == hipSuccess) e = hipStreamSynchronize(st->copy);
    if (e == hipSuccess)
        for (int t = 0; t < 2 * st->nslots; ++t) st->harvest(t);   // every job is finished
    if (stats) {
        stats[0] = st->images;
        stats[1] = st->pixels;
        stats[2] = st->decode_ns;
        stats[3] = st->h2d_bytes;
        stats[4] = st->launches;
    }
    if (e != hipSuccess) return set_error(HJD_E_HIP, "stream sync: %s", hipGetErrorString(e));
    std::lock_guard<std::mutex> g(st->mu);
    if (st->first_error != HJD_OK) {
        const int rc = st->first_error;
        st->first_error = HJD_OK;
        return set_error(rc, "%s", st->first_error_msg.c_str());
    }
    return HJD_OK;
}

int hjd_stream_busy(hjd_stream* st, int64_t* h2d_busy_ns, int64_t* kernel_busy_ns)
{
    if (!st) return set_error(HJD_E_INVALID, "stream is NULL");
    if (h2d_busy_ns) *h2d_busy_ns = st->h2d_busy_ns;
    if (kernel_busy_ns) *kernel_busy_ns = st->kernel_busy_ns;
    return HJD_OK;
}

}  // extern "C"
