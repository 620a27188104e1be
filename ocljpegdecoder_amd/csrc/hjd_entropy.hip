// hjd_entropy.hip -- GPU entropy decoding of baseline JPEG scans (include/hjd_host.h,
// SURVEY.md s8(f) rank 3).
//
// Host side (per JPEG, at memcpy speed): parse the header, build the device
// Huffman tables, copy the entropy-coded segment into pinned memory while
// removing byte stuffing (FF00 -> FF) and RST markers, recording where each
// restart interval ends.  Device side (one batch of frames per launch chain):
//   ent_sync_kernel   a group stages its bit window in LDS; each thread decodes
//                     its S-bit subsequence from a guessed entry, then the group
//                     iterates entry(k+1) = run(entry(k)) until nothing changes.
//                     Groups own 248 subsequences and also decode the 8 before
//                     them ("warm-up"), shared with the previous group;
//   ent_link_kernel   one thread per group: the chains of consecutive groups are
//                     joined if some warm-up entry equals the predecessor's entry
//                     for the same subsequence (a pure comparison, no decoding);
//   ent_fallback_kernel  frames with an unjoined boundary are redone sequentially
//                     (not seen on real data at the default S; correct anyway);
//   ent_write_kernel  ordered segmented scan of the statistics (block index, DC
//                     predictors) and a final run per subsequence that writes
//                     int16 zigzag blocks straight to HBM in MCU-major order;
// then the fused pixel kernel (hjd_kernels.hpp) turns the blocks into BGRX.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <vector>

#include "hjd.h"
#include "hjd_entropy.hpp"
#include "hjd_host.h"
#include "hjd_internal.h"

using hjd_internal::FrameRecord;
using hjd_internal::set_error;
using namespace hjd::ent;

#define HJD_HIP(expr)                                                                          \
    do {                                                                                       \
        hipError_t e_ = (expr);                                                                \
        if (e_ != hipSuccess) return set_error(HJD_E_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

namespace {

constexpr int kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

constexpr size_t kDataPad = 64;      // readable bytes after each frame's bit string (16-B chunks read ahead)
constexpr size_t kAlign = 256;

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---------------------------------------------------------------------------
// Host preparation
// ---------------------------------------------------------------------------

// Canonical Huffman code (T.81 C.2 / F.2.2.3) -> first-level LUT of unit
// entries + MAXCODE.  dc: the table's class (T.81 B.2.4.2 Tc = 0).
int build_lut(HuffLut& t, const uint8_t counts[16], const uint8_t* syms, int nsym, bool dc)
{
    memset(&t, 0, sizeof(t));
    int code = 0, k = 0;
    for (int len = 1; len <= 16; ++len) {
        const int n = counts[len - 1];
        const int first = code;
        for (int i = 0; i < n; ++i, ++k, ++code) {
            if (k >= nsym || code >= (1 << len)) return -1;
            t.vals[k] = syms[k];
            if (len <= kLutBits) {
                const int shift = kLutBits - len;
                for (int r = 0; r < (1 << shift); ++r)
                    t.lut[(code << shift) | r] = static_cast<uint16_t>(unit_entry(len, syms[k], dc));
            }
        }
        t.maxcode[len] = n ? code - 1 : -1;
        t.delta[len] = (k - n) - first;   // valptr - mincode
        code <<= 1;
    }
    t.maxcode[0] = -1;
    return 0;
}

// A host destuff that hands finished output to the GPU while it runs (a
// latency decoder's lone image): fire(h, done) once `done` >= next output
// bytes are final; fire sets the next threshold.
struct DestuffHook {
    size_t next;
    void (*fire)(DestuffHook* h, size_t done);
    void* ctx;
};

// Copy an entropy-coded segment without byte stuffing and RST markers.  Ends
// at the first marker that is not RSTn (normally EOI) or at the end of the
// buffer.  seg_end receives the destuffed BIT offset where each restart
// interval ends (the last one = total length).
int destuff(const uint8_t* p, const uint8_t* end, uint8_t* out, size_t cap, std::vector<uint32_t>& seg_end,
            size_t& out_len, DestuffHook* hook = nullptr)
{
    uint8_t* q = out;
    uint8_t* const qend = out + cap;
    int nrst = 0;
    seg_end.clear();
    while (p < end) {
        p = hjd_internal::copy_until_ff(p, end, q, qend);
        if (hook && static_cast<size_t>(q - out) >= hook->next) hook->fire(hook, static_cast<size_t>(q - out));
        if (p == end) break;
        if (*p != 0xFF) return set_error(HJD_E_INVALID, "scan larger than the staging capacity");
        if (p + 1 >= end) break;                       // truncated at FF
        const uint8_t b = p[1];
        if (b == 0x00) {                               // stuffed FF
            if (q >= qend) return set_error(HJD_E_INVALID, "scan larger than the staging capacity");
            *q++ = 0xFF;
            p += 2;
        } else if (b == 0xFF) {                        // fill byte before a marker
            p += 1;
        } else if (b >= 0xD0 && b <= 0xD7) {           // RSTn (src/decoder.cpp:288-307)
            if (b != 0xD0 + (nrst & 7))
                return set_error(HJD_E_INVALID, "expected RST%d, found RST%d", nrst & 7, b - 0xD0);
            seg_end.push_back(static_cast<uint32_t>((q - out) * 8));
            ++nrst;
            p += 2;
        } else {
            break;                                     // EOI (or another marker): end of scan
        }
    }
    seg_end.push_back(static_cast<uint32_t>((q - out) * 8));
    out_len = static_cast<size_t>(q - out);
    return HJD_OK;
}

// Pixel-kernel launch class of a sampling (parse_scan_header admits only known ones).
inline int sampling_class(int sampling)
{
    hjd_internal::SamplingGeom g;
    return hjd_internal::sampling_geom(sampling, &g) ? g.index : 0;
}

// Host-side result of preparing one JPEG: its (first) scan, which is the
// whole image for the reference's single interleaved scan, plus `more` for
// the further scans of a sequential file with several (an extension; each
// becomes an entropy frame of its own writing into the same coefficients).
constexpr int kMaxScans = 3;   // sequential: one scan per component at most (T.81 B.2.3)
struct Prepared {
    int rc = HJD_OK;
    int width = 0, height = 0, sampling = 0, bpm = 0;
    int64_t nblocks = 0;       // blocks this scan codes
    int64_t out_blocks = 0;    // blocks of the image
    uint32_t layout = kLayoutMcu, geo = 0, mcu_w = 0;   // EntFrame fields (block_dest)
    std::vector<Prepared> more;
    uint32_t data_bits = 0;
    size_t data_off = 0;       // in the batch data area
    int ntab = 0;
    int restart_mcus = 0;      // DRI (0: none)
    HuffLut tabs[kMaxTables];
    uint16_t jinfo[6] = {0, 0, 0, 0, 0, 0};
    std::vector<uint32_t> seg_end;
    int32_t qt[3][64];         // zigzag
    void* d_out = nullptr;
    int32_t pitch = 0;
    // device destuff: the raw scan goes to the device (data_bits is then the
    // raw upper bound until destuff_scan_kernel writes the real length)
    int destuff = 0;           // kDestuffHost / kDestuffFromCaller / kDestuffFromStaging
    const uint8_t* raw_src = nullptr;   // caller's pinned bytes (kDestuffFromCaller)
    uint32_t raw_len = 0;
    uint64_t raw_off = 0;      // raw-area offset of the first scan byte (RawCursor::place)

    // end of the data area this file uses (all scans, with their pads)
    size_t data_end() const
    {
        size_t e = data_off + data_bits / 8 + kDataPad;
        for (const Prepared& q : more) e = std::max(e, q.data_off + q.data_bits / 8 + kDataPad);
        return e;
    }
};

// Data-area bytes a JPEG of `size` bytes may need: its destuffed scans are
// shorter than the file, but each scan is padded and aligned.
inline size_t data_need(size_t size) { return align_up(size + kDataPad, 16) + (kMaxScans - 1) * (kDataPad + 16); }

constexpr int kDestuffHost = 0;          // memchr/memcpy destuff into pinned staging (destuff() above)
constexpr int kDestuffFromCaller = 1;    // raw bytes DMA'd from the caller's pinned buffer, destuffed on the GPU
constexpr int kDestuffFromStaging = 2;   // raw bytes memcpy'd into pinned staging, destuffed on the GPU

// The scan-level fields of q from its header: geometry, and the tables the
// scan references, deduplicated into slots.
int scan_fields(const hjd_internal::ScanHeader& h, Prepared& q)
{
    q.bpm = h.bpm;
    q.nblocks = h.scan_blocks;
    q.restart_mcus = h.restart_interval;
    q.layout = h.layout ? kLayoutRaster : kLayoutMcu;
    q.geo = geo_make(static_cast<uint32_t>(h.out_bpm), static_cast<uint32_t>(h.comp_lh),
                     static_cast<uint32_t>(h.comp_lv), static_cast<uint32_t>(h.comp_bw));
    q.mcu_w = static_cast<uint32_t>(h.mcu_w);
    int slot_of[2][4];
    for (auto& a : slot_of)
        for (int& v : a) v = -1;
    q.ntab = 0;
    for (int j = 0; j < h.bpm; ++j) {
        const int ids[2] = {h.jdc[j], h.jac[j]};
        int slot[2];
        for (int cls = 0; cls < 2; ++cls) {
            int& s = slot_of[cls][ids[cls]];
            if (s < 0) {
                if (q.ntab >= kMaxTables) return set_error(HJD_E_INVALID, "too many Huffman tables");
                s = q.ntab++;
                if (build_lut(q.tabs[s], h.counts[cls][ids[cls]], h.symbols[cls][ids[cls]], h.nsym[cls][ids[cls]],
                              cls == 0))
                    return set_error(HJD_E_INVALID, "invalid Huffman table");
            }
            slot[cls] = s;
        }
        q.jinfo[j] = static_cast<uint16_t>(jinfo_make(slot[0], slot[1], h.jcomp[j], h.jslot[j]));
    }
    return HJD_OK;
}

// Restart intervals a scan must hold: DRI counts the scan's MCUs, which are
// single blocks in a non-interleaved scan.
inline int64_t scan_segments(const hjd_internal::ScanHeader& h)
{
    const int64_t units = h.layout ? h.scan_blocks : static_cast<int64_t>(h.mcu_w) * h.mcu_h;
    return h.restart_interval > 0 ? (units + h.restart_interval - 1) / h.restart_interval : 1;
}

// Host destuff of one scan into dst (cap bytes, the pad included).
int destuff_scan(const hjd_internal::ScanHeader& h, const uint8_t* data, size_t size, uint8_t* dst, size_t cap,
                 Prepared& q, DestuffHook* hook = nullptr)
{
    if (h.scan_offset > size) return set_error(HJD_E_INVALID, "scan offset past the end of the file");
    if (cap <= kDataPad) return set_error(HJD_E_INVALID, "scan bytes exceed the batch capacity");
    size_t len = 0;
    q.raw_len = static_cast<uint32_t>(std::min<size_t>(size - h.scan_offset, 0xFFFFFFFFu));   // bytes the host reads
    // a large scan: the first ~60 % of the output goes to the GPU while the host destuffs the rest
    if (hook) hook->next = size - h.scan_offset >= (256u << 10) ? (size - h.scan_offset) * 3 / 5 : SIZE_MAX;
    int rc = destuff(data + h.scan_offset, data + size, dst, cap - kDataPad, q.seg_end, len, hook);
    if (rc) return rc;
    if (len == 0) return set_error(HJD_E_INVALID, "empty scan");
    if (len >= (1u << 28)) return set_error(HJD_E_INVALID, "scan too large for one frame (>= 256 MiB)");
    const int64_t want = scan_segments(h);
    if (static_cast<int64_t>(q.seg_end.size()) != want)
        return set_error(HJD_E_INVALID, "%zu restart intervals in the scan, %lld expected", q.seg_end.size(),
                         static_cast<long long>(want));
    if (h.nblocks >= (1ll << 31)) return set_error(HJD_E_INVALID, "frame too large");
    memset(dst + len, 0xFF, kDataPad);
    q.data_bits = static_cast<uint32_t>(len * 8);
    return HJD_OK;
}

// A sequential file with several scans: every scan destuffed on the host, one
// after the other from dst (cap bytes); quantisation tables as of each
// component's scan.
int prepare_multiscan(const uint8_t* data, size_t size, uint8_t* dst, size_t cap, Prepared& pf)
{
    std::vector<hjd_internal::ScanHeader> hs;
    int rc = hjd_internal::parse_scan_headers(data, size, &hs);
    if (rc) return rc;
    if (hs.empty() || hs.size() > static_cast<size_t>(kMaxScans)) return set_error(HJD_E_INVALID, "bad scan count");
    pf.more.resize(hs.size() - 1);
    size_t off = 0;
    for (size_t k = 0; k < hs.size(); ++k) {
        Prepared& q = k == 0 ? pf : pf.more[k - 1];
        rc = scan_fields(hs[k], q);
        if (rc) return rc;
        if (off >= cap) return set_error(HJD_E_INVALID, "scan bytes exceed the batch capacity");
        q.data_off = pf.data_off + off;
        rc = destuff_scan(hs[k], data, size, dst + off, cap - off, q);
        if (rc) return rc;
        for (int j = 0; j < hs[k].bpm; ++j) {
            const int c = hs[k].jcomp[j];
            memcpy(pf.qt[c], hs[k].qt[c], sizeof(pf.qt[c]));
        }
        off = align_up(off + q.data_bits / 8 + kDataPad, 16);
    }
    return HJD_OK;
}

int prepare(const uint8_t* data, size_t size, uint8_t* dst, size_t cap, Prepared& pf, int mode = kDestuffHost,
            uint64_t raw_off = 0, DestuffHook* hook = nullptr)
{
    hjd_internal::ScanHeader h;
    int rc = hjd_internal::parse_scan_header(data, size, &h);
    if (rc) return rc;
    pf.width = h.width;
    pf.height = h.height;
    pf.sampling = h.sampling;
    pf.out_blocks = h.nblocks;
    memcpy(pf.qt, h.qt, sizeof(pf.qt));
    if (h.extra_scans > 0) {   // several scans: plan_raw keeps them on the host destuff path
        if (mode != kDestuffHost) return set_error(HJD_E_INVALID, "multi-scan JPEG: host destuff only");
        return prepare_multiscan(data, size, dst, cap + kDataPad, pf);
    }
    rc = scan_fields(h, pf);
    if (rc) return rc;
    if (h.scan_offset > size) return set_error(HJD_E_INVALID, "scan offset past the end of the file");
    if (mode != kDestuffHost) {
        // the header is all the host reads; the GPU finds stuffing, markers and the scan's end
        const size_t raw = size - h.scan_offset;
        if (raw == 0) return set_error(HJD_E_INVALID, "empty scan");
        if (raw >= (1u << 28)) return set_error(HJD_E_INVALID, "scan too large for one frame (>= 256 MiB)");
        if (raw > cap) return set_error(HJD_E_INVALID, "scan larger than the staging capacity");
        if (h.nblocks >= (1ll << 31)) return set_error(HJD_E_INVALID, "frame too large");
        const int64_t nmcu = static_cast<int64_t>(h.mcu_w) * h.mcu_h;
        const int64_t want = h.restart_interval > 0 ? (nmcu + h.restart_interval - 1) / h.restart_interval : 1;
        if (want > raw / 2 + 1) return set_error(HJD_E_INVALID, "%lld restart intervals cannot fit %zu scan bytes",
                                                 static_cast<long long>(want), raw);
        pf.seg_end.assign(static_cast<size_t>(want), 0u);   // filled on the device
        pf.destuff = mode;
        pf.raw_len = static_cast<uint32_t>(raw);
        pf.raw_src = data + h.scan_offset;
        pf.raw_off = raw_off;
        if (mode == kDestuffFromStaging) memcpy(dst, pf.raw_src, raw);
        pf.data_bits = static_cast<uint32_t>(raw * 8);      // upper bound (groups are laid out for it)
        return HJD_OK;
    }
    return destuff_scan(h, data, size, dst, cap + kDataPad, pf, hook);
}

// Device destuff ("Destuff on the GPU").  A frame whose scan
// bytes reach the device raw (straight from the caller's pinned buffer, or
// copied into pinned staging) is destuffed by three kernels over 16-KiB tiles:
// count -> per-frame scan -> write.  Its destuffed bit string lands where a
// host-destuffed frame's would, at data_off of the data area, so the entropy
// kernels are unchanged; the host only parses the header.
constexpr uint32_t kTileBytes = 16384;
constexpr int kTileThreads = 256;
constexpr uint32_t kNoEnd = 0xFFFFFFFFu;

// The raw bytes of a frame sit at any byte offset of the raw area (so that
// frames adjacent in the caller's memory stay adjacent there and move in one
// DMA); the kernels address them from the 16-B aligned `raw_off - begin` in
// "region" coordinates [0, begin + raw_len) and ignore the first `begin` bytes.
struct RawFrame {          // one per frame of a batch (32 B)
    uint64_t raw_off;      // raw area offset of the first scan byte
    uint32_t raw_len;      // scan bytes from the end of the SOS header to the end of the file
    uint32_t begin;        // raw_off & 15
    uint32_t tile_base;    // first tile of the frame
    uint32_t ntiles;       // 0: destuffed on the host
    uint32_t end;          // region offset where the scan ends (destuff_scan_kernel)
    uint32_t pad;
};
static_assert(sizeof(RawFrame) == 32, "RawFrame layout");

__host__ __device__ __forceinline__ uint32_t raw_region_len(uint32_t begin, uint32_t raw_len) { return begin + raw_len; }

// Places raw scans in a batch's raw area.  A caller-pinned scan that follows
// the previous one in the caller's memory within kMirrorGap bytes (a JPEG
// header, typically) is placed at the same distance, so the run moves with one
// DMA; anything else goes after the area in use, at the source's alignment mod 16.
//
// Capacity contract: a batch whose files total F bytes fits a raw area of
// F + kSlack bytes per frame, whatever lies between the files.  Mirroring
// consumes the gap between two scans (the next file's header, plus whatever
// the caller left between the files), so it is taken only while the area in
// use stays within the bytes of the files placed so far plus kSlack each
// (`allow`); otherwise, or when the mirrored offset would not fit, the scan
// is placed compactly (<= 30 bytes of alignment) and starts a new DMA run.
// By induction the area in use never exceeds F + 48 bytes per frame, and the
// 32-byte read-ahead fits in the kDataPad + 16 bytes data_cap() adds per frame.
struct RawCursor {
    static constexpr uint64_t kMirrorGap = 64 * 1024;
    static constexpr uint64_t kSlack = 48;
    static constexpr uint64_t kReadAhead = 32;   // destuff kernels' 16-B loads straddling the end
    const uint8_t* last_src = nullptr;
    uint64_t last_off = 0;
    uint64_t end = 0;
    uint64_t allow = 0;      // sum of (file bytes + kSlack) over the frames placed
    // n = scan bytes at src; file = bytes of the whole file; reserve = area
    // that must stay free after this scan (for frames still to come).
    bool place(const uint8_t* src, size_t n, size_t file, bool mirror, size_t cap, uint64_t& off,
               uint64_t reserve = 0)
    {
        const uint64_t allow_next = allow + file + kSlack;
        uint64_t o = ~0ull;
        if (mirror && last_src && src > last_src && last_off + static_cast<uint64_t>(src - last_src) >= end &&
            last_off + static_cast<uint64_t>(src - last_src) - end <= kMirrorGap) {
            o = last_off + static_cast<uint64_t>(src - last_src);
            if (o + n > allow_next || o + n + kReadAhead + reserve > cap) o = ~0ull;
        }
        if (o == ~0ull) {
            o = (end + 15) / 16 * 16 + (reinterpret_cast<uintptr_t>(src) & 15);
            if (o + n + kReadAhead + reserve > cap) return false;
        }
        off = o;
        end = o + n;
        allow = allow_next;
        last_src = mirror ? src : nullptr;
        last_off = o;
        return true;
    }
};

// ---------------------------------------------------------------------------
// Batch layout.  The header (frames | tables | segment ends | group->frame map |
// pixel-kernel records | natural-order qtables) is laid out compactly per batch
// at offset 0; the destuffed scans live at the fixed offset `data`.  Pinned
// staging and the device blob use the same layout, so one copy moves each part.
// ---------------------------------------------------------------------------
struct Caps {
    int max_frames;
    int64_t max_scan_bytes, max_blocks;
    int sub_bits;
    int64_t max_subs, max_wgs, max_segs, max_tiles;
    size_t hdr_cap, data;
};

Caps make_caps(int max_frames, int64_t max_scan_bytes, int64_t max_blocks, int sub_bits)
{
    Caps c;
    c.max_frames = max_frames;
    c.max_scan_bytes = max_scan_bytes;
    c.max_blocks = max_blocks;
    c.sub_bits = sub_bits;
    // entropy frames: one per scan, kMaxScans per JPEG at most
    const int64_t ef = static_cast<int64_t>(max_frames) * kMaxScans;
    c.max_subs = (max_scan_bytes * 8 + sub_bits - 1) / sub_bits + ef;
    c.max_wgs = (c.max_subs + kOwn - 1) / kOwn + ef;
    // restart segments: one per restart interval; a non-interleaved scan (or a
    // gray file) with Ri = 1 has one per block, so blocks + one per entropy frame
    c.max_segs = max_blocks + ef;
    c.max_tiles = max_scan_bytes / kTileBytes + max_frames;
    const size_t per_frame = (sizeof(EntFrame) + sizeof(HuffLut) * kMaxTables + 8) * kMaxScans + sizeof(FrameRecord) +
                             192 * 4 + sizeof(RawFrame) + 4;
    c.hdr_cap = align_up(per_frame * max_frames + 4 * static_cast<size_t>(c.max_segs + c.max_wgs + c.max_tiles) +
                             10 * kAlign, kAlign);
    c.data = c.hdr_cap;
    return c;
}

struct HdrOffsets {
    size_t frames, tabs, seg, wg, recs, qt, rawf, tilef, status, used;
};

// Device-side view of a batch (kernel argument).
struct EntBatchDev {
    const EntFrame* frames;
    const HuffLut* tabs;
    const uint32_t* seg_end;
    const uint32_t* wg_frame;
    const uint8_t* data;
    uint64_t* entries;
    SubStats* stats;
    uint64_t* mids;       // [sub] verified state at the first unit boundary >= k*S + S/2
    SubStats* stats1;     // [sub] statistics of the first half (entry -> mid)
    uint64_t* wentries;   // [group][kWarm] warm-up entries
    uint32_t* linked;     // [group] 1 if joined to the previous group's chain
    SubStats* agg;
    SubStats* agg2;       // [group] null, or the rest of agg: a group's statistics in the next chain chunk
    uint32_t* status;     // [nframes], ent_write_kernel's finished-workgroup count, [nframes] chain chunk counts
    uint32_t* host_status;   // null, or pinned host words the last write workgroup copies status to
    int16_t* coefs;
    uint32_t nframes, nwg, sub_bits, ntab_max;   // ntab_max: tables of the largest frame (dynamic LDS)
    uint32_t ntab_total;                         // tables of the batch
    uint8_t* steps_g;                            // [table][1 << kStepBits] AC step entries (ent_steps_kernel)
    uint32_t nsub_total;                         // subsequences of the batch
    // device destuff (ntiles == 0: every frame of the batch was destuffed on the host)
    const uint8_t* raw;          // raw scan bytes, frame f at frames[f].data_off
    RawFrame* rawf;              // [nframes]
    const uint32_t* tile_frame;  // [ntiles] frame of each tile
    uint32_t* tiles;             // [3][ntiles] scratch: emitted bytes, markers, end (then offsets)
    uint32_t ntiles;
    // speculative sync (latency decoders; null otherwise): [sub][kMaxBpm] records
    struct SpecRec* spec;        // [sub][kMaxBpm]
    struct CandRec* cand;        // [sub][kSlots]
    uint8_t* cmap;               // [sub][kSlotRow]
    uint8_t* cslot;              // [sub] the verified chain's slot (ent_chain_lb_kernel / ent_chain_kernel)
    uint32_t spec_lead;          // lead-in of the spec runs (bits)
    uint32_t* chainfn;           // [frame][chain_chunks][kLbWords] look-back words of the chunks (ent_chain_lb_kernel)
    uint32_t* chain_broken;      // non-null: the look-back chain kernel runs (its words are allocated)
    uint32_t chain_chunks;       // chunks of the frame with the most subsequences (grid width)
    uint32_t chain_epoch;        // 1 .. 2^24 - 1, new per launch: tags the look-back words (no clearing)
};


// `blocks`: the frame's block_info() records (fill_blocks), LDS on the device.
__host__ __device__ __forceinline__ RunCtx make_ctx(const EntBatchDev& b, const EntFrame& F, const HuffLut* tabs,
                                                    const BlockInfo* blocks, const uint8_t* steps = nullptr)
{
    RunCtx c;
    c.data = b.data + F.data_off;
    c.seg_end = b.seg_end + F.seg_base;
    c.tabs = tabs;
    c.blocks = blocks;
    c.nseg = F.nseg;
    c.data_bits = F.data_bits;
    c.bpm = F.bpm;
    c.seg_blocks = F.seg_blocks;
    c.steps = steps;
    c.layout = F.layout;
    c.geo = F.geo;
    c.mcu_w = F.mcu_w;
    return c;
}

// The frame's AC step tables (step_entry) from its LUTs: [table][1 << kStepBits].
__host__ __device__ __forceinline__ void fill_steps(uint8_t* steps, const HuffLut* tabs, int ntab, int tid,
                                                    int nthreads)
{
    for (int i = tid; i < (ntab << kStepBits); i += nthreads)
        steps[i] = step_entry(tabs[i >> kStepBits], static_cast<uint32_t>(i) & ((1u << kStepBits) - 1));
}

// A frame's step tables from the batch's (ent_steps_kernel) into LDS.
__device__ __forceinline__ void copy_steps(uint8_t* steps, const EntBatchDev& b, const EntFrame& F, int tid,
                                           int nthreads)
{
    const uint4* src = reinterpret_cast<const uint4*>(b.steps_g + (static_cast<size_t>(F.tab_base) << kStepBits));
    uint4* dst = reinterpret_cast<uint4*>(steps);
    for (int i = tid; i < (F.ntab << kStepBits) / 16; i += nthreads) dst[i] = src[i];
}

// Host side of the block records (the kernels fill their LDS copy per thread).
inline void fill_blocks(BlockInfo (&t)[kMaxBpm], const EntFrame& F)
{
    for (int j = 0; j < kMaxBpm; ++j) t[j] = block_info(F.jinfo[j]);
}

__host__ __device__ __forceinline__ uint64_t guess_entry(const RunCtx& c, uint32_t start)
{
    return pack_state(start, 0, 0, find_segment(c.seg_end, c.nseg, start));
}

__host__ __device__ __forceinline__ uint32_t frame_groups(uint32_t nsub) { return (nsub + kOwn - 1) / kOwn; }

// Subsequence handled by thread t of frame group gl (may be < 0 or >= nsub).
__host__ __device__ __forceinline__ int64_t group_sub(uint32_t gl, int t)
{
    return static_cast<int64_t>(gl) * kOwn - kWarm + t;
}

// Speculative sync (latency mode, DESIGN.md s10 "Single-image latency").
// The round-based sync guesses one entry per subsequence, (k*S, j = 0,
// z = 0): bits and z fall into step with the true decode within a few hundred
// bits, but the block-in-MCU index j only by chance, so a lone frame's chains
// take ~7 serial rounds of S-bit re-runs to verify (measured by the emulation:
// 4-10 rounds per group on an FHD q90 frame at S = 1024).  Here:
//   ent_spec_kernel   runs every subsequence k from all P = bpm guesses
//                     (k*S - W, j, 0), a lead-in of W bits before its start:
//                     the state at its middle (checkpoint), its exit and the
//                     second half's statistics.  One of the P guesses meets
//                     the true decode within 512 bits for 89 % of starts and
//                     within 1024 for 98 % (one guess: 25 % and 54 %;
//                     hjd_debug_entropy_syncstats with HJD_SYNC_PHASES);
//   ent_cand_kernel   runs k from each of its predecessor's P spec exits
//                     (subsequence 0: from the frame start), stopping at the
//                     middle when the run meets one of k's checkpoints; the
//                     exit's index among k's spec exits is k+1's entry slot
//                     (cmap).  An exit that is none of them opens an overflow
//                     slot of k+1 (two levels), so the maps are total on real
//                     data;
//   ent_chain_kernel  one workgroup per frame composes the slot maps (a scan
//                     over threads, each owning a range of subsequences) from
//                     the frame start: every subsequence's verified entry,
//                     statistics and mid-state follow without serial rounds,
//                     and the group records (agg, wentries, linked) the link,
//                     fallback and write kernels read.
// The chain is exact by construction (every record comes from a real run of
// its subsequence from the entry it names, starting at the frame start); a
// chain that leaves all slots (none seen) falls back to the sequential repair.
// The write kernel decodes a verified subsequence as four quarters, each from
// the state at its first unit boundary >= k*S + q*S/4 (q = 0: the entry):
// the runs below stop there on the way and keep those states.
__host__ __device__ __forceinline__ uint32_t quarter_stop(uint32_t k, uint32_t S, uint32_t q)
{
    return k * S + (q * S) / 4;
}
struct SpecRec {          // spec run of subsequence k from guess (k*S - W, j, 0)
    uint64_t cp;          // state at the first unit boundary >= k*S + S/2
    uint64_t x;           // exit
    SubStats s2;          // statistics cp -> x
    SubStats s3;          // statistics cp -> q3
    uint64_t q3, pad;     // state at the third quarter (as cp at the middle)
};
static_assert(sizeof(SpecRec) == 64, "SpecRec layout");
struct CandRec {          // subsequence k run from the entry of one of its slots
    SubStats s1, s;       // [0] [1] statistics entry -> mid and entry -> exit
    uint64_t e, mid;      // [2] entry, mid-state
    uint64_t y, q1;       // [3] exit, first-quarter state
    SubStats sq1;         // [4] statistics entry -> q1
    SubStats sq3;         // [5] statistics mid -> q3
    uint64_t q3, pad0;    // [6] third-quarter state
    uint64_t pad1, pad2;  // [7]
};
static_assert(sizeof(CandRec) == 128, "CandRec layout");
constexpr uint32_t kNoCand = 0xFF;                   // no slot
constexpr int kOvfLevels = 2;                        // overflow slots: P per level
constexpr int kSlots = (1 + kOvfLevels) * kMaxBpm;   // candidate and overflow slots per subsequence
constexpr int kRepairSlot = kSlots;                  // written by ent_chain_kernel's repair
constexpr int kChainSlots = kSlots + 1;
constexpr int kCandRow = kChainSlots;                // CandRec row stride
constexpr int kSlotRow = 20;                         // cmap row stride (bytes, >= kChainSlots)
static_assert(kSlotRow >= kChainSlots, "cmap row");

// The spec run of subsequence k from guess j, with a lead-in of `lead` bits.
__host__ __device__ __forceinline__ SpecRec spec_run(const RunCtx& c, uint32_t k, uint32_t j, uint32_t S, uint32_t lead)
{
    const uint32_t start = k * S > lead ? k * S - lead : 0u;
    const uint64_t g = guess_entry(c, start);
    SpecRec r;
    // one run through the middle (cp) and the third quarter (q3) to the exit
    const uint32_t mpos[2] = {quarter_stop(k, S, 2), quarter_stop(k, S, 3)};
    uint64_t ms[2];
    SubStats mst[2], s4 = stats_identity();
    r.x = run<false, 2>(c, pack_state(st_pos(g), j, 0, st_seg(g)), (k + 1) * S, s4, nullptr, mpos, ms, mst);
    r.cp = ms[0];
    r.q3 = ms[1];
    r.s3 = mst[1];
    r.s2 = stats_combine(r.s3, s4);
    r.pad = 0;
    return r;
}

// Subsequence k from entry e: to the middle; if that state is one of k's
// spec checkpoints, the rest is that spec run's, else decode on.  sk: k's P
// spec records.  Returns the index of the exit among k's spec exits, or kNoCand.
__host__ __device__ __forceinline__ uint32_t cand_run(const RunCtx& c, uint32_t k, uint64_t e, uint32_t S,
                                                      const SpecRec* sk, uint32_t P, CandRec& out)
{
    out.e = e;
    out.pad0 = out.pad1 = out.pad2 = 0;
    const uint32_t m1 = quarter_stop(k, S, 1), m3 = quarter_stop(k, S, 3);
    SubStats s12 = stats_identity();
    out.mid = run<false, 1>(c, e, quarter_stop(k, S, 2), s12, nullptr, &m1, &out.q1, &out.sq1);
    out.s1 = stats_combine(out.sq1, s12);
    uint32_t jm = kNoCand;
    for (uint32_t j = 0; j < P; ++j)
        if (jm == kNoCand && same_state(out.mid, sk[j].cp)) jm = j;
    if (jm != kNoCand) {
        out.y = sk[jm].x;
        out.q3 = sk[jm].q3;
        out.sq3 = sk[jm].s3;
        out.s = stats_combine(out.s1, sk[jm].s2);
    } else {
        SubStats s4 = stats_identity();
        out.y = run<false, 1>(c, out.mid, (k + 1) * S, s4, nullptr, &m3, &out.q3, &out.sq3);
        out.s = stats_combine(out.s1, stats_combine(out.sq3, s4));
    }
    uint32_t idx = kNoCand;
    for (uint32_t j = 0; j < P; ++j)
        if (idx == kNoCand && same_state(out.y, sk[j].x)) idx = j;
    return idx;
}

// Candidate c < P of subsequence k (entry: spec exit c of k-1, or the frame
// start), and its overflow continuation: while the exit is none of the
// successor's spec exits, the successor is run from it in overflow slot
// (level + 1) * P + c, up to kOvfLevels levels.  Each slot has exactly one writer.
__host__ __device__ __forceinline__ void cand_chain(const RunCtx& c, const EntBatchDev& b, const EntFrame& F,
                                                    uint32_t k, uint32_t cidx)
{
    const uint32_t P = F.bpm, S = b.sub_bits;
    uint64_t e = k == 0 ? guess_entry(c, 0)
                        : b.spec[(static_cast<uint64_t>(F.sub_base) + k - 1) * kMaxBpm + cidx].x;
    uint32_t slot = cidx;
    for (int level = 0;; ++level) {
        const uint64_t row = static_cast<uint64_t>(F.sub_base) + k;
        CandRec r;
        const uint32_t nx = cand_run(c, k, e, S, b.spec + row * kMaxBpm, P, r);
        b.cand[row * kCandRow + slot] = r;
        if (nx != kNoCand || level == kOvfLevels || k + 1 >= F.nsub) {
            b.cmap[row * kSlotRow + slot] = static_cast<uint8_t>(nx);
            return;
        }
        const uint32_t next = static_cast<uint32_t>(level + 1) * P + cidx;
        b.cmap[row * kSlotRow + slot] = static_cast<uint8_t>(next);
        e = r.y;
        slot = next;
        ++k;
    }
}

// The chain leaves every slot at subsequence brk (its predecessor, entered at
// slot sp, exits at a state none of brk's slots holds): run brk on from that
// exit in the repair slot, and its successors until the exit is a spec exit
// again, linking the predecessor's map to the repair slot.
__host__ __device__ __forceinline__ void chain_repair(const RunCtx& c, const EntBatchDev& b, const EntFrame& F,
                                                      uint32_t brk, uint32_t sp)
{
    uint8_t* cm = b.cmap + static_cast<uint64_t>(F.sub_base) * kSlotRow;
    uint64_t e = b.cand[(static_cast<uint64_t>(F.sub_base) + brk - 1) * kCandRow + sp].y;
    cm[static_cast<uint64_t>(brk - 1) * kSlotRow + sp] = static_cast<uint8_t>(kRepairSlot);
    for (uint32_t k = brk;; ++k) {
        const uint64_t row = static_cast<uint64_t>(F.sub_base) + k;
        CandRec r;
        const uint32_t nx = cand_run(c, k, e, b.sub_bits, b.spec + row * kMaxBpm, F.bpm, r);
        b.cand[row * kCandRow + kRepairSlot] = r;
        if (nx != kNoCand || k + 1 >= F.nsub) {
            cm[static_cast<uint64_t>(k) * kSlotRow + kRepairSlot] = static_cast<uint8_t>(nx);
            return;
        }
        cm[static_cast<uint64_t>(k) * kSlotRow + kRepairSlot] = static_cast<uint8_t>(kRepairSlot);
        e = r.y;
    }
}

// The verified chain's record of subsequence k: the speculative sync leaves it
// in the chain's slot of k (cslot), the round-based sync in the sync arrays.
// 16-B vector reads (a SubStats copy goes through scratch on the device).
__host__ __device__ __forceinline__ SubStats stats_of(const u32x4& v)
{
    SubStats r;
    memcpy(&r, &v, sizeof(r));
    return r;
}
__host__ __device__ __forceinline__ const u32x4* sub_rec(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    const uint64_t row = static_cast<uint64_t>(F.sub_base) + k;
    return reinterpret_cast<const u32x4*>(b.cand + row * kCandRow + b.cslot[row]);
}
__host__ __device__ __forceinline__ SubStats sub_stats(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    return b.spec ? stats_of(sub_rec(b, F, k)[1]) : b.stats[F.sub_base + k];
}
__host__ __device__ __forceinline__ SubStats sub_stats1(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    return b.spec ? stats_of(sub_rec(b, F, k)[0]) : b.stats1[F.sub_base + k];
}
__host__ __device__ __forceinline__ uint64_t sub_entry(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    if (!b.spec) return b.entries[F.sub_base + k];
    const u32x4 v = sub_rec(b, F, k)[2];
    return static_cast<uint64_t>(v.x) | static_cast<uint64_t>(v.y) << 32;
}
__host__ __device__ __forceinline__ uint64_t sub_mid(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    if (!b.spec) return b.mids[F.sub_base + k];
    const u32x4 v = sub_rec(b, F, k)[2];
    return static_cast<uint64_t>(v.z) | static_cast<uint64_t>(v.w) << 32;
}
// Speculative sync only: the quarter states and statistics (CandRec).
__host__ __device__ __forceinline__ uint64_t sub_q1(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    const u32x4 v = sub_rec(b, F, k)[3];
    return static_cast<uint64_t>(v.z) | static_cast<uint64_t>(v.w) << 32;
}
__host__ __device__ __forceinline__ uint64_t sub_q3(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    const u32x4 v = sub_rec(b, F, k)[6];
    return static_cast<uint64_t>(v.x) | static_cast<uint64_t>(v.y) << 32;
}
__host__ __device__ __forceinline__ SubStats sub_sq1(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    return stats_of(sub_rec(b, F, k)[4]);
}
__host__ __device__ __forceinline__ SubStats sub_sq3(const EntBatchDev& b, const EntFrame& F, uint32_t k)
{
    return stats_of(sub_rec(b, F, k)[5]);
}
// Piece p of the write kernel's split of subsequence k (pieces: 2 halves, or
// 4 quarters under the speculative sync): its entry state, its stop, and the
// statistics from k's entry to that state.
__host__ __device__ __forceinline__ uint32_t write_pieces(const EntBatchDev& b) { return b.spec ? 4u : 2u; }
__host__ __device__ __forceinline__ uint64_t piece_entry(const EntBatchDev& b, const EntFrame& F, uint32_t k,
                                                        uint32_t p, SubStats& pre)
{
    pre = stats_identity();
    if (p == 0) return sub_entry(b, F, k);
    if (!b.spec) {
        pre = sub_stats1(b, F, k);
        return sub_mid(b, F, k);
    }
    if (p == 1) {
        pre = sub_sq1(b, F, k);
        return sub_q1(b, F, k);
    }
    pre = sub_stats1(b, F, k);
    if (p == 2) return sub_mid(b, F, k);
    pre = stats_combine(pre, sub_sq3(b, F, k));
    return sub_q3(b, F, k);
}
__host__ __device__ __forceinline__ uint32_t piece_stop(const EntBatchDev& b, uint32_t k, uint32_t p)
{
    return quarter_stop(k, b.sub_bits, (p + 1) * (4 / write_pieces(b)));
}

// ---------------------------------------------------------------------------
// Kernels (gfx950)
// ---------------------------------------------------------------------------

// The frame's Huffman tables and block records into LDS (caller syncs).  The
// jinfo entries are read from the global frame record (a per-thread index into
// a register copy would put the record in scratch).
__device__ __forceinline__ void load_tables(HuffLut* lds, BlockInfo* blocks, const HuffLut* g, const EntFrame& F,
                                            const EntFrame* Fg, int tid, int nthreads)
{
    const u32x4* src = reinterpret_cast<const u32x4*>(g);
    u32x4* dst = reinterpret_cast<u32x4*>(lds);
    const int n = F.ntab * static_cast<int>(sizeof(HuffLut) / 16);
    for (int i = tid; i < n; i += nthreads) dst[i] = src[i];
    if (tid < kMaxBpm) blocks[tid] = block_info(Fg->jinfo[tid]);
}

__device__ __forceinline__ SubStats shfl_down_stats(const SubStats& s, int d)
{
    SubStats r;
    r.nblk = static_cast<uint32_t>(__shfl_down(static_cast<int>(s.nblk), d));
    r.flags = static_cast<uint32_t>(__shfl_down(static_cast<int>(s.flags), d));
    r.dc[0] = __shfl_down(s.dc[0], d);
    r.dc[1] = __shfl_down(s.dc[1], d);
    r.dc[2] = __shfl_down(s.dc[2], d);
    return r;
}

__device__ __forceinline__ SubStats shfl_up_stats(const SubStats& s, int d)
{
    SubStats r;
    r.nblk = static_cast<uint32_t>(__shfl_up(static_cast<int>(s.nblk), d));
    r.flags = static_cast<uint32_t>(__shfl_up(static_cast<int>(s.flags), d));
    r.dc[0] = __shfl_up(s.dc[0], d);
    r.dc[1] = __shfl_up(s.dc[1], d);
    r.dc[2] = __shfl_up(s.dc[2], d);
    return r;
}

// Ordered inclusive scan of one value per thread over the workgroup: each wave
// scans its 64 lanes by shuffles, then the waves' totals are combined through
// LDS (two barriers instead of two per step).  On return buf[t] holds thread
// t's inclusive result and the workgroup is synchronised.
template <int N = kGroupSubs>
__device__ __forceinline__ SubStats block_scan_inclusive(SubStats v, SubStats* buf, int tid)
{
    static_assert(N % 64 == 0 && N / 64 <= 16, "whole waves");
    const int lane = tid & 63, wv = tid >> 6;
    for (int d = 1; d < 64; d <<= 1) {
        const SubStats o = shfl_up_stats(v, d);
        if (lane >= d) v = stats_combine(o, v);
    }
    __shared__ SubStats wsum[N / 64];
    if (lane == 63) wsum[wv] = v;
    __syncthreads();
    SubStats pre = stats_identity();
    for (int w = 0; w < wv; ++w) pre = stats_combine(pre, wsum[w]);
    v = stats_combine(pre, v);
    buf[tid] = v;
    __syncthreads();
    return v;
}

// Ordered reduction over one wave's lanes (lane order = subsequence order);
// the result is valid in lane 0.
__device__ __forceinline__ SubStats wave_reduce_ordered(SubStats v, int lane)
{
    for (int d = 1; d < 64; d <<= 1) {
        const SubStats o = shfl_down_stats(v, d);
        if ((lane & (2 * d - 1)) == 0) v = stats_combine(v, o);
    }
    return v;
}


// LDS layout of the sync kernel after the group's tables (dynamic shared memory).
struct SyncLds {
    uint64_t x[kGroupSubs];      // current exit of each subsequence
    uint64_t used[kGroupSubs];   // entry each subsequence was last run from
    SubStats st[kGroupSubs];     // statistics of that run
    uint16_t list[2][kGroupSubs];
    int32_t nlist[2];
    SubStats wsum[kGroupSubs / 64];
};

__host__ __device__ constexpr size_t sync_lds_bytes(uint32_t ntab)
{
    return (sizeof(HuffLut) + (1u << kStepBits)) * ntab + sizeof(SyncLds);
}

__global__ __launch_bounds__(kGroupSubs) void ent_sync_kernel(EntBatchDev b)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    HuffLut* tabs = reinterpret_cast<HuffLut*>(smem);
    uint8_t* steps = smem + sizeof(HuffLut) * b.ntab_max;
    SyncLds& L = *reinterpret_cast<SyncLds*>(smem + (sizeof(HuffLut) + (1u << kStepBits)) * b.ntab_max);
    const int tid = threadIdx.x;
    const uint32_t w = blockIdx.x;
    const uint32_t f = b.wg_frame[w];
    const EntFrame F = b.frames[f];
    const uint32_t gl = w - F.wg_base;
    const uint32_t S = b.sub_bits;
    // groups laid out for a device-destuffed frame's upper bound (raw bytes) past its real end
    if (gl >= frame_groups(F.nsub)) return;
    __shared__ BlockInfo blocks[kMaxBpm];
    const RunCtx c = make_ctx(b, F, tabs, blocks, steps);
    load_tables(tabs, blocks, b.tabs + F.tab_base, F, b.frames + f, tid, kGroupSubs);
    copy_steps(steps, b, F, tid, kGroupSubs);
    if (tid < 2) L.nlist[tid] = 0;
    __syncthreads();
    const int64_t k0 = group_sub(gl, 0);
    const int64_t k = k0 + tid;
    const bool valid = k >= 0 && k < static_cast<int64_t>(F.nsub);
    const uint32_t ku = static_cast<uint32_t>(k);
    // phase 1: every subsequence from its guessed entry, in two runs split at
    // its middle (the checkpoint), keeping the state there and the statistics
    // of the second half
    const uint32_t mid = ku * S + S / 2;
    uint64_t used = valid ? guess_entry(c, ku * S) : 0;
    SubStats st = stats_identity(), suf = stats_identity();
    uint64_t cp = used, x = used;
    // the write kernel decodes each subsequence as two halves, from the entry and
    // from the mid-state: every run that produces a subsequence's final entry
    // records its mid-state and first-half statistics (the last such run wins)
    const bool rec = valid && tid >= kWarm;
    if (valid) {
        cp = run<false>(c, used, mid, st, nullptr);
        if (rec) {
            b.mids[F.sub_base + ku] = cp;
            b.stats1[F.sub_base + ku] = st;
        }
        x = run<false>(c, cp, (ku + 1) * S, suf, nullptr);
        st = stats_combine(st, suf);
    }
    L.x[tid] = x;
    __syncthreads();
    // round 0, step A: every subsequence from its predecessor's exit, first to
    // the checkpoint only (all lanes busy).  A run that arrives in phase 1's
    // checkpoint state continues exactly as phase 1 did (a run is a function of
    // its state), so its exit and second-half statistics are known; the
    // others are "pending" and go on in step B.  Measured (syncstats): at
    // 4:2:0 53% of guessed runs are in step by mid-subsequence, at 4:4:4 94%,
    // so round 0 decodes 0.74 / 0.53 of the bits it decoded in full.
    bool pending = false;
    uint64_t resume = 0;
    if (valid && tid > 0 && k > 0) {
        const uint64_t e = L.x[tid - 1];
        if (!same_state(e, used)) {
            SubStats s2 = stats_identity();
            resume = run<false>(c, e, mid, s2, nullptr);
            if (rec) {
                b.mids[F.sub_base + ku] = resume;
                b.stats1[F.sub_base + ku] = s2;
            }
            used = e;
            if (same_state(resume, cp)) {
                st = stats_combine(s2, suf);
            } else {
                pending = true;
                st = s2;
            }
        }
    }
    L.used[tid] = used;
    L.st[tid] = st;
    __syncthreads();   // everyone has read L.x (old) before it is overwritten
    if (pending) {     // park the resume state where the exit goes
        L.x[tid] = resume;
        L.list[1][atomicAdd(&L.nlist[1], 1)] = static_cast<uint16_t>(tid);
    }
    __syncthreads();
    // step B: the pending second halves, compacted onto the first lanes
    if (tid < L.nlist[1]) {
        const int item = L.list[1][tid];
        const uint32_t kk = static_cast<uint32_t>(k0 + item);
        SubStats s2 = stats_identity();
        const uint64_t x2 = run<false>(c, L.x[item], (kk + 1) * S, s2, nullptr);
        L.st[item] = stats_combine(L.st[item], s2);
        L.x[item] = x2;
    }
    __syncthreads();
    // a changed exit changes the successor's entry
    if (pending && !same_state(L.x[tid], x) && tid + 1 < kGroupSubs && k + 1 < static_cast<int64_t>(F.nsub))
        L.list[0][atomicAdd(&L.nlist[0], 1)] = static_cast<uint16_t>(tid + 1);
    __syncthreads();
    // later rounds: only the subsequences whose entry changed, compacted onto the
    // first lanes, so idle waves do not replay a full decode
    for (int r = 0;; r ^= 1) {
        const int n = L.nlist[r];
        if (n == 0) break;
        uint64_t x2 = 0, e = 0;
        SubStats s2 = stats_identity();
        int item = -1;
        if (tid < n) {
            item = L.list[r][tid];
            e = L.x[item - 1];
            const uint32_t kk = static_cast<uint32_t>(k0 + item);
            if (!same_state(e, L.used[item])) {
                const uint64_t m2 = run<false>(c, e, kk * S + S / 2, s2, nullptr);
                if (item >= kWarm) {
                    b.mids[F.sub_base + kk] = m2;
                    b.stats1[F.sub_base + kk] = s2;
                }
                SubStats s3 = stats_identity();
                x2 = run<false>(c, m2, (kk + 1) * S, s3, nullptr);
                s2 = stats_combine(s2, s3);
            } else {
                item = -1;
            }
        }
        if (tid == 0) L.nlist[r ^ 1] = 0;
        __syncthreads();   // all reads of L.x done; the next list is empty
        if (item >= 0) {
            L.used[item] = e;
            L.st[item] = s2;
            if (!same_state(x2, L.x[item])) {
                L.x[item] = x2;
                if (item + 1 < kGroupSubs && k0 + item + 1 < static_cast<int64_t>(F.nsub))
                    L.list[r ^ 1][atomicAdd(&L.nlist[r ^ 1], 1)] = static_cast<uint16_t>(item + 1);
            }
        }
        __syncthreads();
    }
    const bool own = valid && tid >= kWarm;
    used = L.used[tid];
    st = L.st[tid];
    if (own) {
        b.entries[F.sub_base + ku] = used;
        b.stats[F.sub_base + ku] = st;
    } else if (tid < kWarm) {
        b.wentries[static_cast<uint64_t>(w) * kWarm + tid] = used;   // 0 for invalid (frame start group)
    }
    // statistics of the owned range: ordered reduce per wave, then across waves
    const SubStats ws = wave_reduce_ordered(own ? st : stats_identity(), tid & 63);
    if ((tid & 63) == 0) L.wsum[tid >> 6] = ws;
    __syncthreads();
    if (tid == 0) {
        SubStats a = L.wsum[0];
        for (int i = 1; i < kGroupSubs / 64; ++i) a = stats_combine(a, L.wsum[i]);
        b.agg[w] = a;
    }
}

// The AC step tables of every Huffman table of the batch, once per batch (the
// sync / spec / cand kernels copy their frame's from here instead of each
// workgroup deriving them from the LUTs).  Grid (tables, kStepGroups): one
// entry per thread, so the serial chain is one entry's few LUT lookups.
constexpr int kStepsThreads = 256;
constexpr int kStepGroups = (1 << kStepBits) / kStepsThreads;
static_assert(kStepGroups * kStepsThreads == (1 << kStepBits), "step groups");
__global__ __launch_bounds__(kStepsThreads) void ent_steps_kernel(EntBatchDev b)
{
    __shared__ HuffLut t;
    const uint32_t ti = blockIdx.x;
    const int tid = threadIdx.x;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(b.tabs + ti);
    uint32_t* dst = reinterpret_cast<uint32_t*>(&t);
    for (int i = tid; i < static_cast<int>(sizeof(t.lut) / 4); i += kStepsThreads) dst[i] = src[i];   // the LUT is all step_entry reads
    __syncthreads();
    const uint32_t e = blockIdx.y * kStepsThreads + static_cast<uint32_t>(tid);
    b.steps_g[(static_cast<size_t>(ti) << kStepBits) + e] = step_entry(t, e);
}

// ---- speculative sync (latency decoders) ------------------------------------
// Grid (groups, kMaxBpm): block (w, j) runs guess j of group w's owned
// subsequences (the warm-up ones belong to the previous group).
__global__ __launch_bounds__(kGroupSubs) void ent_spec_kernel(EntBatchDev b)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    HuffLut* tabs = reinterpret_cast<HuffLut*>(smem);
    uint8_t* steps = smem + sizeof(HuffLut) * b.ntab_max;
    __shared__ BlockInfo blocks[kMaxBpm];
    const int tid = threadIdx.x;
    const uint32_t w = blockIdx.x, j = blockIdx.y;
    const uint32_t f = b.wg_frame[w];
    const EntFrame F = b.frames[f];
    const uint32_t gl = w - F.wg_base;
    if (gl >= frame_groups(F.nsub) || j >= F.bpm) return;
    load_tables(tabs, blocks, b.tabs + F.tab_base, F, b.frames + f, tid, kGroupSubs);
    copy_steps(steps, b, F, tid, kGroupSubs);
    __syncthreads();
    const int64_t k = group_sub(gl, tid);
    if (tid < kWarm || k >= static_cast<int64_t>(F.nsub)) return;
    const RunCtx c = make_ctx(b, F, tabs, blocks, steps);
    const uint64_t row = static_cast<uint64_t>(F.sub_base) + static_cast<uint64_t>(k);
    if (j == 0) {   // the subsequence's slot map starts empty (ent_cand_kernel fills what exists)
        uint32_t* m = reinterpret_cast<uint32_t*>(b.cmap + row * kSlotRow);
#pragma unroll
        for (int i = 0; i < kSlotRow / 4; ++i) m[i] = 0xFFFFFFFFu;
    }
    b.spec[row * kMaxBpm + j] = spec_run(c, static_cast<uint32_t>(k), j, b.sub_bits, b.spec_lead);
}

// Grid (groups, kMaxBpm): block (w, i) runs candidate i of group w's owned
// subsequences, with its overflow continuation (cand_chain).
__global__ __launch_bounds__(kGroupSubs) void ent_cand_kernel(EntBatchDev b)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    HuffLut* tabs = reinterpret_cast<HuffLut*>(smem);
    uint8_t* steps = smem + sizeof(HuffLut) * b.ntab_max;
    __shared__ BlockInfo blocks[kMaxBpm];
    const int tid = threadIdx.x;
    const uint32_t w = blockIdx.x, i = blockIdx.y;
    const uint32_t f = b.wg_frame[w];
    const EntFrame F = b.frames[f];
    const uint32_t gl = w - F.wg_base;
    if (gl >= frame_groups(F.nsub) || i >= F.bpm) return;
    load_tables(tabs, blocks, b.tabs + F.tab_base, F, b.frames + f, tid, kGroupSubs);
    copy_steps(steps, b, F, tid, kGroupSubs);
    __syncthreads();
    const int64_t k = group_sub(gl, tid);
    if (tid < kWarm || k >= static_cast<int64_t>(F.nsub)) return;
    const RunCtx c = make_ctx(b, F, tabs, blocks, steps);
    cand_chain(c, b, F, static_cast<uint32_t>(k), i);
}

// One workgroup per frame walks the chain from the frame start (slot 0 of
// subsequence 0) through chunks of kChainChunk subsequences: the chunk's slot
// maps are loaded into LDS (coalesced), thread t composes its kChainRows
// consecutive rows into one function, the group scans those functions, and the
// chunk's entering slot under the prefix is thread t's entering slot.  Where
// the chain leaves every slot (an exit that is none of the successor's
// candidates even after the overflow levels; rare), thread 0 re-runs it from
// the known exit in the repair slot of the following subsequences until it
// lands in a slot again, and the chunk is scanned anew.  The output is the
// chain's slot of every subsequence (cslot): the write kernel reads each
// subsequence's entry, statistics and mid-state from that slot's record.  Last,
// one wave per group reduces the group's statistics (agg).
// Maps and functions are rows of kSlotRow bytes handled as 5 dwords; a lookup
// selects its byte in registers (LDS byte reads cost ~5x more here).
constexpr int kChainThreads = 512;
constexpr int kChainRows = 2;                                  // rows per thread and chunk
constexpr int kChainChunk = kChainThreads * kChainRows;        // 1024 subsequences
constexpr int kRowWords = kSlotRow / 4;
constexpr int kLbWords = 8;   // look-back words per chunk (ent_chain_lb_kernel)

struct ChainLds {
    uint32_t rows[kChainChunk][kRowWords];      // the chunk's slot maps
    uint32_t fn[2][kChainThreads][kRowWords];   // scan of the threads' functions (double buffer)
    unsigned long long brk;                     // first break: subsequence << 8 | its predecessor's slot
    uint32_t carry;                             // slot entering the chunk
    uint32_t tables_loaded;
    HuffLut tabs[kMaxTables];                   // the frame's tables (repairs only)
    uint8_t steps[kMaxTables << kStepBits];
    BlockInfo blocks[kMaxBpm];
};

struct SlotRow {
    uint32_t w[kRowWords];
};

__device__ __forceinline__ uint32_t row_get(const SlotRow& r, uint32_t a)   // a < kChainSlots
{
    const uint32_t x = a < 8 ? (a < 4 ? r.w[0] : r.w[1]) : a < 16 ? (a < 12 ? r.w[2] : r.w[3]) : r.w[4];
    return (x >> ((a & 3) * 8)) & 0xFFu;
}

__device__ __forceinline__ SlotRow row_load(const uint32_t* p)
{
    SlotRow r;
#pragma unroll
    for (int i = 0; i < kRowWords; ++i) r.w[i] = p[i];
    return r;
}

// f then g: (g . f)(s) = g(f(s)), kNoCand absorbing; bytes past kChainSlots stay kNoCand
// (slot_compose, hjd_entropy.hpp: byte permutes, no per-slot selects)
static_assert(kRowWords == 5 && kNoCand == 0xFF, "slot_compose's row format");
__device__ __forceinline__ SlotRow row_compose(const SlotRow& f, const SlotRow& g)
{
    SlotRow r;
    slot_compose(f.w, g.w, r.w);
    return r;
}

__device__ __forceinline__ SlotRow slot_ident()
{
    SlotRow ident;
#pragma unroll
    for (int i = 0; i < kRowWords; ++i) ident.w[i] = 0xFFFFFFFFu;
#pragma unroll
    for (int s = 0; s < kChainSlots; ++s)
        ident.w[s >> 2] = (ident.w[s >> 2] & ~(0xFFu << ((s & 3) * 8))) | (static_cast<uint32_t>(s) << ((s & 3) * 8));
    return ident;
}

// Rows c0 .. c0 + cn of a frame's slot maps (cm) into rows[]: 4-byte words,
// coalesced, all of a thread's loads in flight at once; rows past cn: none.
__device__ __forceinline__ void chunk_load(uint32_t (*rows)[kRowWords], const uint8_t* cm, uint32_t c0, uint32_t cn,
                                           int tid)
{
    constexpr int kWords = kChainChunk * kRowWords / kChainThreads;   // 10
    const uint32_t* src = reinterpret_cast<const uint32_t*>(cm + static_cast<uint64_t>(c0) * kSlotRow);
    uint32_t* dst = &rows[0][0];
    const uint32_t nw = cn * kRowWords;
    uint32_t t[kWords];
#pragma unroll
    for (int i = 0; i < kWords; ++i) {
        const uint32_t j = static_cast<uint32_t>(tid + i * kChainThreads);
        t[i] = j < nw ? src[j] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int i = 0; i < kWords; ++i) dst[tid + i * kChainThreads] = t[i];
}

// Thread t composes its kChainRows rows of the loaded chunk; the group scans
// the functions (inclusive: fn[cur][t] = thread 0's rows then ... then t's).
// Call after the rows are visible (barrier); returns cur.
__device__ __forceinline__ int chunk_scan(uint32_t (*rows)[kRowWords], uint32_t (*fn)[kChainThreads][kRowWords],
                                          uint32_t cn, int tid)
{
    const uint32_t r0 = static_cast<uint32_t>(tid) * kChainRows;
    SlotRow v = slot_ident();
#pragma unroll 1
    for (uint32_t r = r0; r < r0 + kChainRows && r < cn; ++r) v = row_compose(v, row_load(rows[r]));
#pragma unroll
    for (int i = 0; i < kRowWords; ++i) fn[0][tid][i] = v.w[i];
    __syncthreads();
    int cur = 0;
#pragma unroll 1
    for (int d = 1; d < kChainThreads; d <<= 1) {
        const SlotRow mine = row_load(fn[cur][tid]);
        const SlotRow o = tid >= d ? row_compose(row_load(fn[cur][tid - d]), mine) : mine;
#pragma unroll
        for (int i = 0; i < kRowWords; ++i) fn[cur ^ 1][tid][i] = o.w[i];
        cur ^= 1;
        __syncthreads();
    }
    return cur;
}

// This thread's rows' chain slots (entering at `slot`) into cslot; returns the
// slot after its last row.
__device__ __forceinline__ uint32_t chunk_write_slots(const uint32_t (*rows)[kRowWords], uint8_t* cslot, uint32_t base,
                                                      uint32_t cn, int tid, uint32_t slot)
{
    const uint32_t r0 = static_cast<uint32_t>(tid) * kChainRows;
    uint32_t s = slot;
    uint32_t packed[(kChainRows + 3) / 4] = {};
#pragma unroll
    for (int i = 0; i < kChainRows; ++i) {
        packed[i >> 2] |= (s & 0xFFu) << ((i & 3) * 8);
        if (r0 + i < cn) s = row_get(row_load(rows[r0 + i]), s);
    }
    uint8_t* out = cslot + base + r0;
    if (kChainRows % 4 == 0 && r0 + kChainRows <= cn && ((base + r0) & 3) == 0) {
#pragma unroll
        for (int i = 0; i < kChainRows / 4; ++i) reinterpret_cast<uint32_t*>(out)[i] = packed[i];
    } else {
        for (uint32_t i = 0; i < kChainRows && r0 + i < cn; ++i) out[i] = static_cast<uint8_t>(packed[i >> 2] >> ((i & 3) * 8));
    }
    return s;
}

// Group g of frame F: the ordered reduction of its owned subsequences' chain
// statistics (one wave; lane = its lane) into agg, and the group marked linked.
__device__ __forceinline__ void group_agg(const EntBatchDev& b, const EntFrame& F, uint32_t g, int lane)
{
    const uint32_t w = F.wg_base + g;
    const uint32_t end = (g + 1) * kOwn < F.nsub ? (g + 1) * kOwn : F.nsub;
    SubStats q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // 4 x 64 >= kOwn; the four loads in flight together
        const uint32_t k = g * kOwn + static_cast<uint32_t>(lane) * 4 + i;
        q[i] = k < end ? sub_stats(b, F, k) : stats_identity();
    }
    SubStats a = stats_identity();
#pragma unroll
    for (int i = 0; i < 4; ++i) a = stats_combine(a, q[i]);
    a = wave_reduce_ordered(a, lane);
    if (lane == 0) {
        b.agg[w] = a;
        b.linked[w] = 1u;
    }
}

// Chunk [c0, c0 + cn) of frame F entered at slot `carry`, by one workgroup,
// repairing every break on the way (tid 0 runs the repair; the chunk's maps
// are reloaded after each, and a repair may run on into the next chunk's
// rows): writes the chunk's cslot and returns the slot after its last row.
__device__ __forceinline__ uint32_t walk_chunk(const EntBatchDev& b, uint32_t f, const EntFrame& F, ChainLds& L,
                                               uint32_t c0, uint32_t cn, uint32_t carry, int tid)
{
    const uint32_t n = F.nsub;
    uint8_t* cm = b.cmap + static_cast<uint64_t>(F.sub_base) * kSlotRow;
    const uint32_t r0 = static_cast<uint32_t>(tid) * kChainRows;   // this thread's rows within the chunk
    uint32_t slot;
    for (;;) {
        __syncthreads();
        chunk_load(L.rows, cm, c0, cn, tid);
        if (tid == 0) L.brk = ~0ull;
        __syncthreads();
        const int cur = chunk_scan(L.rows, L.fn, cn, tid);
        slot = tid == 0 ? carry : (carry == kNoCand ? kNoCand : row_get(row_load(L.fn[cur][tid - 1]), carry));
        // the first subsequence without a slot: the row whose map sends the
        // chain's slot to none (subsequence 0's slots all exist)
        uint32_t s = slot;
        for (uint32_t r = r0; r < r0 + kChainRows && r < cn && s != kNoCand; ++r) {
            const uint32_t nx = row_get(row_load(L.rows[r]), s);
            if (nx == kNoCand && c0 + r + 1 < n) {
                atomicMin(&L.brk, (static_cast<unsigned long long>(c0 + r + 1) << 8) | s);
                break;
            }
            s = nx;
        }
        __syncthreads();
        const unsigned long long brk = L.brk;
        if (brk == ~0ull) break;
        if (!L.tables_loaded) {   // the frame's tables, for the repair runs (rare)
            load_tables(L.tabs, L.blocks, b.tabs + F.tab_base, F, b.frames + f, tid, kChainThreads);
            __syncthreads();
            fill_steps(L.steps, L.tabs, F.ntab, tid, kChainThreads);
            __syncthreads();
            if (tid == 0) L.tables_loaded = 1;
        }
        if (tid == 0) {   // (the status bit tells the host a repair ran: hjd_gdec_sync)
            chain_repair(make_ctx(b, F, L.tabs, L.blocks, L.steps), b, F, static_cast<uint32_t>(brk >> 8),
                         static_cast<uint32_t>(brk & 0xFF));
            atomicOr(&b.status[f], kStatusFallback);
        }
    }
    // the chain's slot of each of this thread's rows
    const uint32_t s = chunk_write_slots(L.rows, b.cslot, F.sub_base + c0, cn, tid, slot);
    __syncthreads();
    if (r0 < cn && (r0 + kChainRows >= cn)) L.carry = s;   // the thread holding the chunk's last row
    __syncthreads();
    return L.carry;
}

// The serial walk of frame f by one workgroup (decoders without look-back words).
__device__ __forceinline__ void chain_walk(const EntBatchDev& b, uint32_t f, ChainLds& L, int tid)
{
    const EntFrame F = b.frames[f];
    const uint32_t n = F.nsub;
    if (tid == 0) L.tables_loaded = 0;
    uint32_t carry = 0;
    for (uint32_t c0 = 0; c0 < n; c0 += kChainChunk)
        carry = walk_chunk(b, f, F, L, c0, n - c0 < static_cast<uint32_t>(kChainChunk) ? n - c0 : kChainChunk, carry, tid);
    const int wv = tid >> 6, lane = tid & 63;
    for (uint32_t g = wv; g < frame_groups(F.nsub); g += kChainThreads / 64) {
        group_agg(b, F, g, lane);
        if (b.agg2 && lane == 0) b.agg2[F.wg_base + g] = stats_identity();
    }
}

// Every frame walked serially (decoders without look-back words).
__global__ __launch_bounds__(kChainThreads) void ent_chain_kernel(EntBatchDev b)
{
    __shared__ ChainLds L;
    chain_walk(b, blockIdx.x, L, threadIdx.x);
}

// ---- the chain, chunks in parallel (the case without repairs) -----------------
// ent_chain_kernel's walk takes its chunks one after another (a lone FHD
// frame has 16 of 1024 subsequences; 1024 measured best for the look-back
// kernel: 17.3 us per FHD frame against 20.0 at 2048 and 19.8 at 512).  Where no repair is needed the chunks are
// independent given their entering slot, so one kernel over (chunk, frame)
// runs them side by side with a decoupled look-back: every chunk composes its
// maps into one function (the scan) and publishes it, then thread 0 finds the
// slot entering the chunk from the nearest published exit before it and the
// published maps in between (look-back words tagged with the launch's epoch,
// so nothing is cleared between launches), publishes its own exit, and the
// chunk writes its rows' slots.  A chunk whose predecessor has published
// nothing yet was dispatched after it (lower blockIdx.x first), so the wait
// ends.  Each chunk then reduces the chain statistics of the groups it holds:
// a group's part in its first chunk into agg, its part in the next into agg2
// (so no chunk waits for another's slots).  A chunk whose path leaves every
// slot repairs it itself (walk_chunk) before it publishes its exit; the maps
// send the chunks after it to none, and those wait for that exit instead.
// Breaks in different chunks are repaired side by side (the walk of a whole
// frame by one workgroup after any break cost ~50 us per break on a q90 4:4:4
// FHD frame).
struct ChainParLds {
    uint32_t rows[kChainChunk][kRowWords];
    uint32_t fn[2][kChainThreads][kRowWords];
    uint8_t slots[kChainChunk];   // the chain's slot of each row
    uint32_t carry, broken, published;
};
union ChainLbLds {
    ChainParLds p;
    ChainLds w;   // the walk, after the chunk's own work
};

// Ordered reduction (one wave) of the chain statistics of subsequences
// [lo, hi) of frame F (hi - lo <= 256), slots from LDS (row k at slots[k - c0]).
__device__ __forceinline__ SubStats range_stats(const EntBatchDev& b, const EntFrame& F, uint32_t lo, uint32_t hi,
                                                const uint8_t* slots, uint32_t c0, int lane)
{
    SubStats q[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {   // the four loads in flight together
        const uint32_t k = lo + static_cast<uint32_t>(lane) * 4 + i;
        if (k < hi) {
            const uint64_t row = static_cast<uint64_t>(F.sub_base) + k;
            q[i] = stats_of(reinterpret_cast<const u32x4*>(b.cand + row * kCandRow + slots[k - c0])[1]);
        } else {
            q[i] = stats_identity();
        }
    }
    SubStats a = stats_identity();
#pragma unroll
    for (int i = 0; i < 4; ++i) a = stats_combine(a, q[i]);
    return wave_reduce_ordered(a, lane);
}

__global__ __launch_bounds__(kChainThreads) void ent_chain_lb_kernel(EntBatchDev b)
{
    __shared__ ChainLbLds U;
    ChainParLds& L = U.p;
    const int tid = threadIdx.x;
    const uint32_t c = blockIdx.x, f = blockIdx.y;
    const EntFrame F = b.frames[f];
    const uint32_t n = F.nsub, c0 = c * kChainChunk;
    if (c0 >= n) return;   // (uniform: past this frame's chunks, not counted)
    const uint32_t cn = n - c0 < static_cast<uint32_t>(kChainChunk) ? n - c0 : kChainChunk;
    if (tid == 0) L.broken = 0;
    chunk_load(L.rows, b.cmap + static_cast<uint64_t>(F.sub_base) * kSlotRow, c0, cn, tid);
    __syncthreads();
    const int cur = chunk_scan(L.rows, L.fn, cn, tid);
    // look-back (a word row per chunk: [0] epoch << 8 | exit slot, [1] epoch
    // once [2..6], the chunk's composed map, are written).  The map is published
    // first; the entry slot is then found by walking back to the nearest
    // published exit (chunk 0's entry is slot 0) and applying the maps of the
    // chunks in between, so no chunk waits for its predecessor's exit.
    uint32_t* const lb = b.chainfn + static_cast<uint64_t>(f) * b.chain_chunks * kLbWords;
    if (tid == 0) {   // (one thread writes the map and releases it)
        for (int i = 0; i < kRowWords; ++i) lb[c * kLbWords + 2 + i] = L.fn[cur][kChainThreads - 1][i];
        __hip_atomic_store(lb + c * kLbWords + 1, b.chain_epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (tid < 64 && c <= 64) {   // wave 0: lane i < c reads chunk i's words, all in flight together
        const uint32_t i = static_cast<uint32_t>(tid);
        uint32_t ex = 0, m[kRowWords] = {};
        bool ready = i >= c;
        while (!ready) {
            ex = __hip_atomic_load(lb + i * kLbWords, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            ready = (ex >> 8) == b.chain_epoch ||
                    __hip_atomic_load(lb + i * kLbWords + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == b.chain_epoch;
            if (!ready) __builtin_amdgcn_s_sleep(1);
        }
        const bool has_exit = i < c && (ex >> 8) == b.chain_epoch;
        if (i < c && !has_exit)
            for (int k = 0; k < kRowWords; ++k) m[k] = lb[i * kLbWords + 2 + k];
        // from the last chunk before c with a published exit (else chunk 0,
        // entered at slot 0) through the maps of the chunks after it
        const uint64_t ballot = __ballot(has_exit);
        const int last = ballot ? 63 - __builtin_clzll(ballot) : -1;
        uint32_t sl = last >= 0 ? static_cast<uint32_t>(__shfl(static_cast<int>(ex & 0xFFu), last)) : 0u;
        for (int j = last + 1; j < static_cast<int>(c); ++j) {   // (uniform bounds: the whole wave shuffles)
            SlotRow r;
#pragma unroll
            for (int k = 0; k < kRowWords; ++k) r.w[k] = static_cast<uint32_t>(__shfl(static_cast<int>(m[k]), j));
            if (sl != kNoCand) sl = row_get(r, sl);
        }
        if (tid == 0) L.carry = sl;
    } else if (tid == 0 && c > 64) {   // a long frame: thread 0 walks back
        uint32_t j = c, carry = 0;   // carry: the slot entering chunk j
        while (j > 0) {
            const uint32_t v = __hip_atomic_load(lb + (j - 1) * kLbWords, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if ((v >> 8) == b.chain_epoch) {
                carry = v & 0xFFu;
                break;
            }
            if (__hip_atomic_load(lb + (j - 1) * kLbWords + 1, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) ==
                b.chain_epoch)
                --j;   // its map is there: look further back
            else
                __builtin_amdgcn_s_sleep(1);
        }
        for (; j < c; ++j)   // forward through the maps of chunks j .. c-1
            if (carry != kNoCand) carry = row_get(row_load(lb + j * kLbWords + 2), carry);
        L.carry = carry;
    }
    // The maps send the chain to none where a chunk before this one breaks:
    // that chunk repairs itself and then publishes its exit, so wait for the
    // exit of chunk c - 1 (published exits are never none, but a frame's last
    // chunk's).  This chunk publishes its exit now unless its own path breaks.
    if (tid == 0) {
        uint32_t sl = L.carry;
        while (sl == kNoCand) {
            const uint32_t v = __hip_atomic_load(lb + (c - 1) * kLbWords, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
            if ((v >> 8) == b.chain_epoch)
                sl = v & 0xFFu;
            else
                __builtin_amdgcn_s_sleep(1);
        }
        const uint32_t exit = row_get(row_load(L.fn[cur][kChainThreads - 1]), sl);
        L.published = exit != kNoCand || c0 + cn >= n;
        if (L.published)
            __hip_atomic_store(lb + c * kLbWords, (b.chain_epoch << 8) | exit, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        L.carry = sl;
    }
    __syncthreads();
    const uint32_t carry = L.carry;
    const bool published = L.published;
    const uint32_t slot = tid == 0 ? carry : (carry == kNoCand ? kNoCand : row_get(row_load(L.fn[cur][tid - 1]), carry));
    // a row whose map sends the chain's slot to none, before the frame's last
    // subsequence: this chunk repairs it below (walk_chunk)
    const uint32_t r0 = static_cast<uint32_t>(tid) * kChainRows;
    uint32_t s = slot;
    for (uint32_t r = r0; r < r0 + kChainRows && r < cn; ++r) {
        L.slots[r] = static_cast<uint8_t>(s);
        if (s == kNoCand) continue;
        const uint32_t nx = row_get(row_load(L.rows[r]), s);
        if (nx == kNoCand && c0 + r + 1 < n) L.broken = 1;
        s = nx;
    }
    chunk_write_slots(L.rows, b.cslot, F.sub_base + c0, cn, tid, slot);
    __syncthreads();
    const bool broken = L.broken;
    const uint8_t* slots = L.slots;
    if (broken) {   // the walk's LDS overlays this kernel's: after the barrier above
        if (tid == 0) U.w.tables_loaded = 0;
        const uint32_t exit = walk_chunk(b, f, F, U.w, c0, cn, carry, tid);
        if (tid == 0 && !published)
            __hip_atomic_store(lb + c * kLbWords, (b.chain_epoch << 8) | exit, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        slots = b.cslot + F.sub_base + c0;   // (written by walk_chunk; its last barrier orders them)
    }
    // group statistics: each group part in this chunk, one wave per part
    const int wv = tid >> 6, lane = tid & 63;
    const uint32_t g0 = c0 / kOwn, g1 = (c0 + cn - 1) / kOwn;
    for (uint32_t g = g0 + static_cast<uint32_t>(wv); g <= g1; g += kChainThreads / 64) {
        const uint32_t glo = g * kOwn, ghi = (g + 1) * kOwn < n ? (g + 1) * kOwn : n;
        const uint32_t lo = glo > c0 ? glo : c0, hi = ghi < c0 + cn ? ghi : c0 + cn;
        const SubStats a = range_stats(b, F, lo, hi, slots, c0, lane);
        if (lane == 0) {
            const uint32_t w = F.wg_base + g;
            if (glo >= c0) {   // the group starts here
                b.agg[w] = a;
                b.linked[w] = 1u;
                if (ghi <= c0 + cn) b.agg2[w] = stats_identity();
            } else {
                b.agg2[w] = a;
            }
        }
    }
}

__global__ __launch_bounds__(256) void ent_link_kernel(EntBatchDev b)
{
    const uint32_t w = blockIdx.x * 256 + threadIdx.x;
    if (w >= b.nwg) return;
    const uint32_t f = b.wg_frame[w];
    const EntFrame F = b.frames[f];
    const uint32_t gl = w - F.wg_base;
    if (gl == 0 || gl >= frame_groups(F.nsub)) {   // first group, or past a device-destuffed frame's end
        b.linked[w] = 1;
        return;
    }
    bool joined = false;
    for (int t = 0; t < kWarm && !joined; ++t) {
        const uint64_t k = static_cast<uint64_t>(group_sub(gl, t));
        joined = same_state(b.wentries[static_cast<uint64_t>(w) * kWarm + t], b.entries[F.sub_base + k]);
    }
    b.linked[w] = joined ? 1u : 0u;
    if (!joined) atomicOr(&b.status[f], kStatusFallback);
}

// Repair of unjoined group boundaries, in order, one lane per flagged frame:
// from the predecessor's last (verified) subsequence, re-decode forward until
// the true chain meets the recorded chain again, rewriting entries/statistics
// on the way; then recompute the aggregates of the groups touched.  Chains are
// deterministic, so once two agree at a boundary they agree from there on.
__host__ __device__ __forceinline__ void repair_frame(const EntBatchDev& b, uint32_t f, const HuffLut* tabs,
                                                     const BlockInfo* blocks)
{
    const EntFrame& F = b.frames[f];
    const RunCtx c = make_ctx(b, F, tabs, blocks);
    const uint32_t ng = frame_groups(F.nsub);
    uint32_t done = 0;          // subsequences < done are verified
    uint32_t g_lo = ng, g_hi = 0;
    for (uint32_t gl = 1; gl < ng; ++gl) {
        const uint32_t first = gl * kOwn;
        if (first < done || b.linked[F.wg_base + gl]) continue;
        uint32_t k = first - 1;
        uint64_t cur = b.entries[F.sub_base + k];
        for (;;) {
            SubStats st = stats_identity(), st2 = stats_identity();
            const uint64_t m = run<false>(c, cur, k * b.sub_bits + b.sub_bits / 2, st, nullptr);
            if (k >= first) {
                b.mids[F.sub_base + k] = m;
                b.stats1[F.sub_base + k] = st;
            }
            const uint64_t x = run<false>(c, m, (k + 1) * b.sub_bits, st2, nullptr);
            st = stats_combine(st, st2);
            if (k >= first) {
                b.entries[F.sub_base + k] = cur;
                b.stats[F.sub_base + k] = st;
                const uint32_t g = k / kOwn;
                g_lo = g < g_lo ? g : g_lo;
                g_hi = g > g_hi ? g : g_hi;
            }
            ++k;
            if (k >= F.nsub || same_state(x, b.entries[F.sub_base + k])) break;
            cur = x;
        }
        done = k;
    }
    for (uint32_t g = g_lo; g <= g_hi && g < ng; ++g) {
        SubStats a = stats_identity();
        const uint32_t end = (g + 1) * kOwn < F.nsub ? (g + 1) * kOwn : F.nsub;
        for (uint32_t i = g * kOwn; i < end; ++i) a = stats_combine(a, b.stats[F.sub_base + i]);
        b.agg[F.wg_base + g] = a;
    }
}

__global__ __launch_bounds__(64) void ent_fallback_kernel(EntBatchDev b)
{
    __shared__ HuffLut tabs[kMaxTables];
    __shared__ BlockInfo blocks[kMaxBpm];
    const int lane = threadIdx.x;
    const uint32_t f = blockIdx.x;
    if (!(b.status[f] & kStatusFallback)) return;
    const EntFrame F = b.frames[f];
    load_tables(tabs, blocks, b.tabs + F.tab_base, F, b.frames + f, lane, 64);
    __syncthreads();
    if (lane == 0) repair_frame(b, f, tabs, blocks);
}

// Several threads per subsequence (write_pieces: halves, or quarters under the
// speculative sync, which records the quarter states): in workgroup (w, p)
// thread t decodes piece p of group subsequence t (from the state recorded at
// the piece's start to the next piece's), so each serial chain is S/2 or S/4
// bits long while the sync kernel keeps its S (the sync kernel
// is fastest at S = 4096, writing at 2048).  A run that starts inside a block
// skips to the next DC unit and a run finishes the block it started past its
// stop, so the pieces write disjoint blocks; a piece's block index and DC
// predictors are the subsequence's prefix combined with the statistics up to
// the piece's start.  The pieces are separate 256-thread workgroups: more CUs
// for a lone frame's few groups, one wave per SIMD.
constexpr int kWriteThreads = kGroupSubs;

// The write kernel's end: with b.host_status set, the last workgroup to
// finish copies the frames' status words into pinned host memory, so no
// status copy follows the kernels (the host reads them after the stream's
// completion event).  Every workgroup counts itself once; the status words
// were all final (agent-scope release) before its count.
__device__ __forceinline__ void write_done(const EntBatchDev& b, int tid)
{
    if (!b.host_status) return;
    __syncthreads();
    if (tid != 0) return;
    const uint32_t nwg = gridDim.x * gridDim.y;
    if (__hip_atomic_fetch_add(b.status + b.nframes, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) != nwg - 1) return;
    for (uint32_t f = 0; f < b.nframes; ++f)
        b.host_status[f] = __hip_atomic_load(b.status + f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
    __threadfence_system();
}

__global__ __launch_bounds__(kWriteThreads) void ent_write_kernel(EntBatchDev b)
{
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    int16_t* stage = reinterpret_cast<int16_t*>(smem);                                  // [256][kStageStride]
    HuffLut* tabs = reinterpret_cast<HuffLut*>(smem + sizeof(int16_t) * kWriteThreads * kStageStride);
    SubStats* buf = reinterpret_cast<SubStats*>(stage);   // scan scratch before any block is staged
    static_assert(sizeof(SubStats) * kWriteThreads <= sizeof(int16_t) * kWriteThreads * kStageStride, "scratch");
    const int tid = threadIdx.x;
    const int t = tid;
    const uint32_t piece = blockIdx.y;
    const uint32_t w = blockIdx.x;
    const uint32_t f = b.wg_frame[w];
    const EntFrame F = b.frames[f];
    const uint32_t gl = w - F.wg_base;
    __shared__ BlockInfo blocks[kMaxBpm];
    if (gl < frame_groups(F.nsub) && piece < write_pieces(b)) {   // (uniform in the workgroup)
        load_tables(tabs, blocks, b.tabs + F.tab_base, F, b.frames + f, tid, kWriteThreads);
        // block index / DC predictors at this group's start: all previous groups of the frame
        SubStats pre = stats_identity();
        for (uint32_t base = 0; base < gl; base += kWriteThreads) {
            SubStats v = stats_identity();
            if (base + tid < gl) {
                v = b.agg[F.wg_base + base + tid];
                if (b.agg2) v = stats_combine(v, b.agg2[F.wg_base + base + tid]);
            }
            block_scan_inclusive<kWriteThreads>(v, buf, tid);
            const SubStats total = buf[kWriteThreads - 1];
            __syncthreads();
            pre = stats_combine(pre, total);
        }
        const int64_t k = group_sub(gl, t);
        const bool own = t >= kWarm && k < static_cast<int64_t>(F.nsub);
        const uint32_t ku = static_cast<uint32_t>(k);
        // subsequence prefixes
        const SubStats mine = own ? sub_stats(b, F, ku) : stats_identity();
        block_scan_inclusive<kWriteThreads>(mine, buf, tid);
        SubStats excl = stats_combine(pre, t > 0 ? buf[t - 1] : stats_identity());
        __syncthreads();   // scratch reads done before blocks are staged
        if (own) {
            SubStats lead;
            const uint64_t entry = piece_entry(b, F, ku, piece, lead);
            excl = stats_combine(excl, lead);
            const uint32_t stop = piece_stop(b, ku, piece);
            const RunCtx c = make_ctx(b, F, tabs, blocks);
            RunOut o;
            o.coefs = b.coefs + F.coef_off * 64;
            o.stage = stage + tid * kStageStride;
            o.blk = excl.nblk;
            o.nblocks = F.nblocks;
            o.nout = F.nout;
            o.pred[0] = excl.dc[0];
            o.pred[1] = excl.dc[1];
            o.pred[2] = excl.dc[2];
            SubStats st = stats_identity();
            run<true>(c, entry, stop, st, &o);
            uint32_t bad = (st.flags & kError) ? kStatusCorrupt : 0;
            if (piece + 1 == write_pieces(b) && ku == F.nsub - 1 && excl.nblk + st.nblk != F.nblocks) bad |= kStatusCount;
            if (bad) __hip_atomic_fetch_or(&b.status[f], bad, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    write_done(b, tid);
}

// ---------------------------------------------------------------------------
// Device destuff kernels.  The byte rules restate destuff() above (and T.81
// B.1.1.5 / F.1.2.3): every 0xFF is the first byte of a pair, so the fate of
// byte i depends only on (r[i-1], r[i], r[i+1]):
//   r[i] = FF: next 00 -> emit FF (stuffing); next FF -> drop (fill byte);
//              next D0..D7 -> drop, restart marker; no next byte or any other
//              next -> the scan ends here (EOI or another marker);
//   r[i] != FF after an FF: drop (the 00 of a stuffed pair, or RSTn's code);
//   otherwise emit r[i].
// ---------------------------------------------------------------------------

// Work split: a 256-thread group takes a 16-KiB tile in 4 passes; in pass p
// thread t takes the 16 bytes at p*4096 + 16t (one coalesced dwordx4 per lane).
// A lane classifies its 16 bytes with word-parallel tests: a 16-bit mask of
// 0xFF bytes, then a loop over those bytes only (0-1 per lane at q90: a 0xFF
// is ~1 byte in 256), giving a drop mask, a marker mask and the scan's end.
constexpr int kPasses = static_cast<int>(kTileBytes / (16 * kTileThreads));   // 4

struct Lane16 {
    uint64_t lo, hi;          // the 16 bytes, little-endian (byte 0 = first in the stream)
    uint32_t drop;            // bytes removed (stuffing 00, fill FF, RSTn pairs, everything from the end on)
    uint32_t marks;           // bit k: an RSTn pair starts at byte k
    uint32_t end;             // frame offset of the scan's end if it lies in these bytes, else kNoEnd
};

__device__ __forceinline__ uint32_t ff_mask4(uint32_t w)
{
    const uint32_t t = ~w;   // FF bytes -> 00; exact zero-byte test
    const uint32_t z = ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t | 0x7F7F7F7Fu);
    return ((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u);
}

__device__ __forceinline__ uint32_t byte_at(const Lane16& v, uint32_t k)
{
    return static_cast<uint32_t>((k < 8 ? v.lo >> (8 * k) : v.hi >> (8 * (k - 8))) & 0xFFu);
}

// Classify the 16 region bytes at s (16-B aligned): bytes before `begin` (not
// the scan's) and at or past `lim` (the region's length, or the known scan
// end) are dropped.  Nothing at or past `lim` is loaded: a lane whose 16 bytes
// start there (most of a frame's last tile) issues no load, and a lane that
// straddles it reads at most 15 bytes past the region, inside the 32-byte
// read-ahead every raw placement reserves (RawCursor::place).
__device__ __forceinline__ Lane16 classify16(const uint8_t* r, uint32_t s, uint32_t begin, uint32_t len, uint32_t lim)
{
    Lane16 v;
    v.marks = 0;
    v.end = kNoEnd;
    if (s >= lim) {
        v.lo = v.hi = 0;
        v.drop = 0xFFFFu;
        return v;
    }
    const u32x4 q = *reinterpret_cast<const u32x4*>(r + s);
    v.lo = static_cast<uint64_t>(q.x) | (static_cast<uint64_t>(q.y) << 32);
    v.hi = static_cast<uint64_t>(q.z) | (static_cast<uint64_t>(q.w) << 32);
    uint32_t drop = 0;
    if (lim - s < 16) drop = 0xFFFFu & ~((1u << (lim - s)) - 1u);
    uint32_t ff = ff_mask4(q.x) | (ff_mask4(q.y) << 4) | (ff_mask4(q.z) << 8) | (ff_mask4(q.w) << 12);
    if (s < begin) {                                // only in a frame's first 16 bytes (begin < 16)
        const uint32_t pre = (1u << (begin - s)) - 1u;
        drop |= pre;
        ff &= ~pre;
    }
    const uint32_t prev = s > begin ? r[s - 1] : 0u;
    if (prev == 0xFFu && !(ff & 1u)) drop |= 1u;   // second byte of a pair begun in the previous 16
    if (ff) {
        const uint32_t next16 = s + 16 < len ? r[s + 16] : 0u;
        while (ff) {
            const uint32_t k = __builtin_ctz(ff);
            ff &= ff - 1u;
            if (s + k >= lim) break;
            const bool has_next = s + k + 1 < len;
            const uint32_t nb = k < 15 ? byte_at(v, k + 1) : next16;
            const uint32_t pair = k < 15 ? 3u << k : 1u << k;   // this FF and its second byte, if in these 16
            if (has_next && nb == 0x00u) {
                drop |= (pair & ~(1u << k));                     // FF kept, 00 dropped
            } else if (has_next && nb == 0xFFu) {
                drop |= 1u << k;                                 // fill byte; the next FF leads a pair
            } else if (has_next && nb >= 0xD0u && nb <= 0xD7u) {
                drop |= pair;
                v.marks |= 1u << k;
            } else {                                             // EOI, another marker, or FF at the very end
                v.end = s + k;
                drop |= 0xFFFFu & ~((1u << k) - 1u);
                break;
            }
        }
    }
    v.drop = drop;
    return v;
}

// Pack the kept bytes of v to its low end (lowest first); returns their count.
__device__ __forceinline__ uint32_t compact16(Lane16& v)
{
    const uint32_t keep = ~v.drop & 0xFFFFu;
    const uint32_t n = __builtin_popcount(keep);
    if (n == 16) return n;
    // drops below the highest kept byte need a shift; process them from the top down
    uint32_t holes = v.drop & ((keep ? (2u << (31 - __builtin_clz(keep))) : 1u) - 1u);
    while (holes) {
        const uint32_t k = 31 - __builtin_clz(holes);
        holes &= ~(1u << k);
        if (k >= 8) {
            const uint32_t j = k - 8;
            const uint64_t low = j ? (~0ull >> (64 - 8 * j)) : 0ull;
            v.hi = (v.hi & low) | ((v.hi >> 8) & ~low);
        } else {
            const uint64_t low = k ? (~0ull >> (64 - 8 * k)) : 0ull;
            v.lo = (v.lo & low) | ((v.lo >> 8) & ~low) | (v.hi << 56);
            v.hi >>= 8;
        }
    }
    return n;
}

// Block-wide exclusive scan of two counters (256 threads); returns the totals.
__device__ __forceinline__ void block_scan2(uint32_t& a, uint32_t& b2, uint32_t& tot_a, uint32_t& tot_b, uint32_t* sa,
                                            uint32_t* sb)
{
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    uint32_t xa = a, xb = b2;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t ya = __shfl_up(xa, d), yb = __shfl_up(xb, d);
        if (lane >= d) { xa += ya; xb += yb; }
    }
    if (lane == 63) { sa[wv] = xa; sb[wv] = xb; }
    __syncthreads();
    uint32_t ba = 0, bb = 0;
    for (int i = 0; i < wv; ++i) { ba += sa[i]; bb += sb[i]; }
    tot_a = sa[0] + sa[1] + sa[2] + sa[3];
    tot_b = sb[0] + sb[1] + sb[2] + sb[3];
    a = ba + xa - a;     // exclusive
    b2 = bb + xb - b2;
    __syncthreads();
}

__device__ __forceinline__ uint32_t lane_offset(uint32_t t, int p)
{
    return static_cast<uint32_t>(p) * (16u * kTileThreads) + 16u * t;
}

__global__ __launch_bounds__(kTileThreads) void destuff_count_kernel(EntBatchDev b)
{
    __shared__ uint32_t s_end, sa[4], sb[4];
    const uint32_t t = blockIdx.x;
    const uint32_t f = b.tile_frame[t];
    const RawFrame R = b.rawf[f];
    const uint8_t* r = b.raw + (R.raw_off - R.begin);
    const uint32_t L = raw_region_len(R.begin, R.raw_len);
    const uint32_t s0 = (t - R.tile_base) * kTileBytes;
    if (threadIdx.x == 0) s_end = kNoEnd;
    __syncthreads();
    uint32_t ne[kPasses], nm[kPasses], end = kNoEnd;
#pragma unroll
    for (int p = 0; p < kPasses; ++p) {
        const uint32_t s = s0 + lane_offset(threadIdx.x, p);
        const Lane16 v = classify16(r, s, R.begin, L, L);
        ne[p] = __builtin_popcount(~v.drop & 0xFFFFu);
        nm[p] = __builtin_popcount(v.marks);
        end = min(end, v.end);
    }
    if (end != kNoEnd) atomicMin(&s_end, end);
    __syncthreads();
    const uint32_t tile_end = s_end;
    uint32_t te = 0, tm = 0;
#pragma unroll
    for (int p = 0; p < kPasses; ++p)          // what lies past the scan's end does not count
        if (s0 + lane_offset(threadIdx.x, p) <= tile_end) { te += ne[p]; tm += nm[p]; }
    uint32_t x = te, y = tm;
    block_scan2(x, y, te, tm, sa, sb);
    if (threadIdx.x == 0) {
        b.tiles[t] = te;
        b.tiles[b.ntiles + t] = tm;
        b.tiles[2 * b.ntiles + t] = tile_end;
    }
}

// One group per frame: tile offsets (exclusive scans), the frame's length,
// subsequence count, segment table tail and read-ahead pad; malformed scans
// are flagged kStatusCorrupt (what destuff()/prepare() reject on the host).
__global__ __launch_bounds__(kTileThreads) void destuff_scan_kernel(EntBatchDev b)
{
    __shared__ uint32_t sa[4], sb[4], s_stop;
    const uint32_t f = blockIdx.x;
    RawFrame& R = b.rawf[f];
    if (R.ntiles == 0) return;
    EntFrame& F = const_cast<EntFrame*>(b.frames)[f];
    const int tid = threadIdx.x;
    uint32_t carry_e = 0, carry_m = 0, end = kNoEnd;
    for (uint32_t c0 = 0; c0 < R.ntiles; c0 += kTileThreads) {
        const uint32_t j = c0 + tid;
        const uint32_t t = R.tile_base + j;
        uint32_t e = 0, m = 0, te = kNoEnd;
        if (j < R.ntiles) {
            e = b.tiles[t];
            m = b.tiles[b.ntiles + t];
            te = b.tiles[2 * b.ntiles + t];
        }
        if (tid == 0) s_stop = kNoEnd;
        __syncthreads();
        if (te != kNoEnd) atomicMin(&s_stop, j);     // first tile of the chunk holding the scan's end
        __syncthreads();
        const uint32_t stop = s_stop;
        if (j > stop) e = m = 0;
        uint32_t xe = e, xm = m, tot_e, tot_m;
        block_scan2(xe, xm, tot_e, tot_m, sa, sb);
        if (j < R.ntiles) {
            b.tiles[t] = carry_e + xe;               // byte offset of the tile's output
            b.tiles[b.ntiles + t] = carry_m + xm;    // index of its first marker
        }
        carry_e += tot_e;
        carry_m += tot_m;
        if (stop != kNoEnd) {
            if (tid == 0) s_stop = b.tiles[2 * b.ntiles + R.tile_base + stop];
            __syncthreads();
            end = s_stop;
            break;
        }
    }
    const uint32_t total = carry_e, markers = carry_m;
    const uint32_t bits = total * 8;
    uint32_t* seg = const_cast<uint32_t*>(b.seg_end) + F.seg_base;
    for (uint32_t k = min(markers, F.nseg - 1) + tid; k < F.nseg; k += kTileThreads) seg[k] = bits;
    uint8_t* out = const_cast<uint8_t*>(b.data) + F.data_off + total;
    if (tid < static_cast<int>(kDataPad)) out[tid] = 0xFF;
    if (tid == 0) {
        R.end = end == kNoEnd ? raw_region_len(R.begin, R.raw_len) : end;
        F.data_bits = bits;
        F.nsub = (bits + b.sub_bits - 1) / b.sub_bits;
        if (total == 0 || total >= (1u << 28) || markers != F.nseg - 1) atomicOr(&b.status[f], kStatusCorrupt);
    }
}

__global__ __launch_bounds__(kTileThreads) void destuff_write_kernel(EntBatchDev b)
{
    __shared__ uint32_t sa[4], sb[4];
    __shared__ uint32_t stage[kTileBytes / 4 + 8];      // output bytes of the tile, word-aligned to the output
    const uint32_t t = blockIdx.x;
    const uint32_t f = b.tile_frame[t];
    const RawFrame R = b.rawf[f];
    const EntFrame F = b.frames[f];
    const uint8_t* r = b.raw + (R.raw_off - R.begin);
    const uint32_t L = raw_region_len(R.begin, R.raw_len);
    const uint32_t s0 = (t - R.tile_base) * kTileBytes;
    const uint32_t tile_out = b.tiles[t];
    uint32_t mark_base = b.tiles[b.ntiles + t];
    const uint32_t base = tile_out & ~3u;              // stage word 0 <-> output byte `base`
    const uint32_t lo = tile_out - base;
    for (uint32_t i = threadIdx.x; i < kTileBytes / 4 + 8; i += kTileThreads) stage[i] = 0u;
    __syncthreads();
    uint32_t* seg = const_cast<uint32_t*>(b.seg_end) + F.seg_base;
    uint32_t out_pos = lo;                             // stage byte of this pass's first output
#pragma unroll
    for (int p = 0; p < kPasses; ++p) {
        const uint32_t s = s0 + lane_offset(threadIdx.x, p);
        Lane16 v = classify16(r, s, R.begin, L, R.end);
        const uint32_t marks = v.marks;                // classify16 stops at the scan's end
        const uint32_t kept_mask = ~v.drop & 0xFFFFu;
        uint32_t n = __builtin_popcount(kept_mask), nm = __builtin_popcount(marks), pe, pm;
        uint32_t xe = n, xm = nm;
        block_scan2(xe, xm, pe, pm, sa, sb);
        // restart markers: ordinal and the destuffed bit offset where the interval ends
        uint32_t mm = marks, ord = mark_base + xm;
        while (mm) {
            const uint32_t k = __builtin_ctz(mm);
            mm &= mm - 1u;
            const uint32_t code = (k < 15 ? byte_at(v, k + 1) : r[s + 16]) - 0xD0u;
            if (code != (ord & 7u)) atomicOr(b.status + f, kStatusCorrupt);   // RSTn out of order
            if (ord + 1 < F.nseg)
                seg[ord] = (tile_out + (out_pos - lo) + xe + __builtin_popcount(kept_mask & ((1u << k) - 1u))) * 8;
            ++ord;
        }
        if (n) {   // the kept bytes, packed, OR-ed into the staged words they cover
            compact16(v);
            const uint32_t o = out_pos + xe;
            const uint32_t sh = 8 * (o & 3u);
            uint32_t w[5];
            const uint32_t x0 = static_cast<uint32_t>(v.lo), x1 = static_cast<uint32_t>(v.lo >> 32);
            const uint32_t x2 = static_cast<uint32_t>(v.hi), x3 = static_cast<uint32_t>(v.hi >> 32);
            // mask off bytes past n before shifting (their content is stale)
            uint32_t m0 = n >= 4 ? ~0u : (1u << (8 * n)) - 1u;
            uint32_t m1 = n >= 8 ? ~0u : n <= 4 ? 0u : (1u << (8 * (n - 4))) - 1u;
            uint32_t m2 = n >= 12 ? ~0u : n <= 8 ? 0u : (1u << (8 * (n - 8))) - 1u;
            uint32_t m3 = n >= 16 ? ~0u : n <= 12 ? 0u : (1u << (8 * (n - 12))) - 1u;
            const uint32_t y0 = x0 & m0, y1 = x1 & m1, y2 = x2 & m2, y3 = x3 & m3;
            if (sh) {
                w[0] = y0 << sh;
                w[1] = (y1 << sh) | (y0 >> (32 - sh));
                w[2] = (y2 << sh) | (y1 >> (32 - sh));
                w[3] = (y3 << sh) | (y2 >> (32 - sh));
                w[4] = y3 >> (32 - sh);
            } else {
                w[0] = y0; w[1] = y1; w[2] = y2; w[3] = y3; w[4] = 0u;
            }
            const uint32_t wbase = o >> 2, nw = (8 * n + sh + 31) / 32;
#pragma unroll
            for (int i = 0; i < 5; ++i)
                if (static_cast<uint32_t>(i) < nw) atomicOr(&stage[wbase + i], w[i]);
        }
        out_pos += pe;
        mark_base += pm;
    }
    __syncthreads();
    // coalesced word stores; the partial words at the tile's two ends by bytes
    uint8_t* out = const_cast<uint8_t*>(b.data) + F.data_off;
    const uint32_t nbytes = out_pos;                   // = lo + the tile's output bytes
    const uint32_t nwords = (nbytes + 3) / 4;
    const uint8_t* sb8 = reinterpret_cast<const uint8_t*>(stage);
    for (uint32_t i = threadIdx.x; i < nwords; i += kTileThreads) {
        const uint32_t b0 = 4 * i, b1 = min(b0 + 4, nbytes);
        if (b0 >= lo && b1 == b0 + 4) {
            *reinterpret_cast<uint32_t*>(out + base + b0) = stage[i];
        } else {
            for (uint32_t k = max(b0, lo); k < b1; ++k) out[base + k] = sb8[k];
        }
    }
}

// ---------------------------------------------------------------------------
// Host emulation of the four kernels (test hook; same state machine and the
// same group geometry, without the LDS window)
// ---------------------------------------------------------------------------
// Host emulation of ent_spec_kernel, ent_cand_kernel and ent_chain_kernel.
void emulate_spec_sync(const EntBatchDev& b)
{
    const uint32_t S = b.sub_bits;
    for (int pass = 0; pass < 2; ++pass) {   // 0: spec runs, 1: candidate chains
        for (uint32_t w = 0; w < b.nwg; ++w) {
            const EntFrame& F = b.frames[b.wg_frame[w]];
            const uint32_t gl = w - F.wg_base;
            if (gl >= frame_groups(F.nsub)) continue;
            BlockInfo blocks[kMaxBpm];
            fill_blocks(blocks, F);
            std::vector<uint8_t> steps(static_cast<size_t>(F.ntab) << kStepBits);
            fill_steps(steps.data(), b.tabs + F.tab_base, F.ntab, 0, 1);
            const RunCtx c = make_ctx(b, F, b.tabs + F.tab_base, blocks, steps.data());
            for (int t = kWarm; t < kGroupSubs; ++t) {
                const int64_t k = group_sub(gl, t);
                if (k >= static_cast<int64_t>(F.nsub)) break;
                for (uint32_t j = 0; j < F.bpm; ++j) {
                    if (pass == 0)
                        b.spec[(static_cast<uint64_t>(F.sub_base) + static_cast<uint64_t>(k)) * kMaxBpm + j] =
                            spec_run(c, static_cast<uint32_t>(k), j, S, b.spec_lead);
                    else
                        cand_chain(c, b, F, static_cast<uint32_t>(k), j);
                }
            }
        }
    }
    for (uint32_t f = 0; f < b.nframes; ++f) {   // the chain kernel's walk, in order, with its repairs
        const EntFrame& F = b.frames[f];
        const uint32_t n = F.nsub;
        BlockInfo blocks[kMaxBpm];
        fill_blocks(blocks, F);
        std::vector<uint8_t> steps(static_cast<size_t>(F.ntab) << kStepBits);
        fill_steps(steps.data(), b.tabs + F.tab_base, F.ntab, 0, 1);
        const RunCtx c = make_ctx(b, F, b.tabs + F.tab_base, blocks, steps.data());
        uint32_t slot = 0, prev = 0;
        int nrepair = 0;
        for (uint32_t k = 0; k < n; ++k) {
            const uint64_t row = static_cast<uint64_t>(F.sub_base) + k;
            if (slot == kNoCand) {
                chain_repair(c, b, F, k, prev);
                slot = kRepairSlot;
                ++nrepair;
            }
            const CandRec& r = b.cand[row * kCandRow + slot];
            b.cslot[row] = static_cast<uint8_t>(slot);
            b.entries[row] = r.e;
            b.stats[row] = r.s;
            b.mids[row] = r.mid;
            b.stats1[row] = r.s1;
            prev = slot;
            slot = b.cmap[row * kSlotRow + slot];
        }
        if (nrepair) b.status[f] |= kStatusFallback;
        if (getenv("HJD_EMU_ROUNDS")) {
            int novf[kOvfLevels + 2] = {};
            for (uint32_t k = 0; k < n; ++k)
                for (uint32_t q = 0; q < F.bpm; ++q) {
                    const uint32_t v = b.cmap[(static_cast<uint64_t>(F.sub_base) + k) * kSlotRow + q];
                    novf[v == kNoCand ? kOvfLevels + 1 : v >= static_cast<uint32_t>(kSlots) ? 0 : v / F.bpm]++;
                }
            fprintf(stderr, "chain: nsub %u repairs %d; level-0 candidates -> spec %d, overflow %d, none %d\n", n,
                    nrepair, novf[0], novf[1], novf[kOvfLevels + 1]);
            int chain_lvl[kOvfLevels + 2] = {};   // the verified chain's slots by level (last: repair)
            for (uint32_t k = 0; k < n; ++k) {
                const uint32_t sl = b.cslot[F.sub_base + k];
                ++chain_lvl[sl >= static_cast<uint32_t>(kSlots) ? kOvfLevels + 1 : sl / F.bpm];
            }
            fprintf(stderr, "chain: slots by level %d / %d / %d, repair %d\n", chain_lvl[0], chain_lvl[1], chain_lvl[2],
                    chain_lvl[3]);
            // ent_cand_kernel's serial bits per thread (k, c) and per wave (64 lanes of one c)
            std::vector<uint32_t> cost, wmax;
            uint32_t nlev[kOvfLevels + 1] = {}, nmiss = 0;
            for (uint32_t g = 0; g < frame_groups(n); ++g)
                for (uint32_t c0 = 0; c0 < F.bpm; ++c0)
                    for (int wv = 0; wv < kGroupSubs / 64; ++wv) {
                        uint32_t wm = 0;
                        for (int l = 0; l < 64; ++l) {
                            const int t = wv * 64 + l;
                            const int64_t k0 = group_sub(g, t);
                            if (t < kWarm || k0 >= static_cast<int64_t>(n)) continue;
                            uint32_t kk = static_cast<uint32_t>(k0), slot = c0, bits = 0;
                            for (int level = 0;; ++level) {
                                const uint64_t row = static_cast<uint64_t>(F.sub_base) + kk;
                                const CandRec& r = b.cand[row * kCandRow + slot];
                                bits += st_pos(r.mid) - st_pos(r.e);
                                bool hit = false;
                                for (uint32_t j = 0; j < F.bpm; ++j) hit |= same_state(r.mid, b.spec[row * kMaxBpm + j].cp);
                                if (!hit) {
                                    bits += st_pos(r.y) - st_pos(r.mid);
                                    ++nmiss;
                                }
                                const uint32_t nx = b.cmap[row * kSlotRow + slot];
                                if (nx == kNoCand || nx < F.bpm || level == kOvfLevels || kk + 1 >= n) {
                                    ++nlev[level];
                                    break;
                                }
                                slot = nx;
                                ++kk;
                            }
                            cost.push_back(bits);
                            wm = std::max(wm, bits);
                        }
                        if (wm) wmax.push_back(wm);
                    }
            auto pct = [](std::vector<uint32_t> v, double q) {
                std::sort(v.begin(), v.end());
                return v.empty() ? 0u : v[static_cast<size_t>(q * (v.size() - 1))];
            };
            fprintf(stderr, "cand threads %zu: levels %u/%u/%u, mid misses %u; bits p50 %u p90 %u p99 %u max %u; "
                    "wave max p50 %u p90 %u max %u\n", cost.size(), nlev[0], nlev[1], nlev[2], nmiss, pct(cost, 0.5),
                    pct(cost, 0.9), pct(cost, 0.99), pct(cost, 1.0), pct(wmax, 0.5), pct(wmax, 0.9), pct(wmax, 1.0));
        }
        for (uint32_t g = 0; g < frame_groups(n); ++g) {
            const uint32_t w = F.wg_base + g;
            SubStats a = stats_identity();
            const uint32_t end = (g + 1) * kOwn < n ? (g + 1) * kOwn : n;
            for (uint32_t k = g * kOwn; k < end; ++k) a = stats_combine(a, b.stats[F.sub_base + k]);
            b.agg[w] = a;
            for (int t = 0; t < kWarm; ++t) {
                const int64_t k = group_sub(g, t);
                b.wentries[static_cast<uint64_t>(w) * kWarm + t] = k >= 0 ? b.entries[F.sub_base + k] : 0;
            }
            b.linked[w] = 1u;
        }
    }
}

void emulate(const EntBatchDev& b)
{
    const uint32_t S = b.sub_bits;
    // sync: per group, phase 1 then the rounds (or the speculative sync)
    if (b.spec) emulate_spec_sync(b);
    for (uint32_t w = 0; w < (b.spec ? 0u : b.nwg); ++w) {
        const EntFrame& F = b.frames[b.wg_frame[w]];
        BlockInfo blocks[kMaxBpm];
        fill_blocks(blocks, F);
        std::vector<uint8_t> steps(static_cast<size_t>(F.ntab) << kStepBits);
        fill_steps(steps.data(), b.tabs + F.tab_base, F.ntab, 0, 1);
        const RunCtx c = make_ctx(b, F, b.tabs + F.tab_base, blocks, steps.data());
        const uint32_t gl = w - F.wg_base;
        std::vector<uint64_t> used(kGroupSubs, 0), x(kGroupSubs, 0), xs0(kGroupSubs, 0), xs1(kGroupSubs, 0);
        std::vector<SubStats> st(kGroupSubs, stats_identity()), suf(kGroupSubs, stats_identity());
        std::vector<uint64_t> cp(kGroupSubs, 0);
        auto valid = [&](int t) { const int64_t k = group_sub(gl, t); return k >= 0 && k < int64_t(F.nsub); };
        auto record = [&](int t, uint64_t m, const SubStats& s1) {   // as the device: owned subsequences
            if (t < kWarm) return;
            const uint32_t k = static_cast<uint32_t>(group_sub(gl, t));
            b.mids[F.sub_base + k] = m;
            b.stats1[F.sub_base + k] = s1;
        };
        for (int t = 0; t < kGroupSubs; ++t) {   // phase 1, split at the checkpoint
            if (!valid(t)) continue;
            const uint32_t k = static_cast<uint32_t>(group_sub(gl, t));
            used[t] = guess_entry(c, k * S);
            cp[t] = run<false>(c, used[t], k * S + S / 2, st[t], nullptr);
            record(t, cp[t], st[t]);
            x[t] = run<false>(c, cp[t], (k + 1) * S, suf[t], nullptr);
            st[t] = stats_combine(st[t], suf[t]);
            xs0[t] = x[t];
        }
        std::vector<uint64_t>* cur = &xs0;
        std::vector<uint64_t>* nxt = &xs1;
        for (int round = 0;; ++round) {
            bool changed = false;
            for (int t = 0; t < kGroupSubs; ++t) {
                const int64_t k = group_sub(gl, t);
                if (valid(t) && t > 0 && k > 0 && !same_state((*cur)[t - 1], used[t])) {
                    const uint32_t ku = static_cast<uint32_t>(k);
                    SubStats s2 = stats_identity();
                    uint64_t x2;
                    if (round == 0) {   // round 0: to the checkpoint, on if phase 1 is not joined there
                        const uint64_t r = run<false>(c, (*cur)[t - 1], ku * S + S / 2, s2, nullptr);
                        record(t, r, s2);
                        if (same_state(r, cp[t])) {
                            x2 = x[t];
                            s2 = stats_combine(s2, suf[t]);
                        } else {
                            SubStats s3 = stats_identity();
                            x2 = run<false>(c, r, (ku + 1) * S, s3, nullptr);
                            s2 = stats_combine(s2, s3);
                        }
                    } else {
                        const uint64_t m2 = run<false>(c, (*cur)[t - 1], ku * S + S / 2, s2, nullptr);
                        record(t, m2, s2);
                        SubStats s3 = stats_identity();
                        x2 = run<false>(c, m2, (ku + 1) * S, s3, nullptr);
                        s2 = stats_combine(s2, s3);
                    }
                    changed |= !same_state(x2, x[t]);
                    used[t] = (*cur)[t - 1];
                    st[t] = s2;
                    x[t] = x2;
                }
                (*nxt)[t] = x[t];
            }
            std::swap(cur, nxt);
            if (!changed) {
                if (getenv("HJD_EMU_ROUNDS")) fprintf(stderr, "group %u: %d rounds\n", gl, round + 1);
                break;
            }
        }
        SubStats a = stats_identity();
        for (int t = 0; t < kGroupSubs; ++t) {
            const bool own = valid(t) && t >= kWarm;
            const uint32_t k = static_cast<uint32_t>(group_sub(gl, t));
            if (own) {
                b.entries[F.sub_base + k] = used[t];
                b.stats[F.sub_base + k] = st[t];
                a = stats_combine(a, st[t]);
            } else if (t < kWarm) {
                b.wentries[static_cast<uint64_t>(w) * kWarm + t] = used[t];
            }
        }
        b.agg[w] = a;
    }
    // link (the speculative sync's chain kernel writes the group records itself)
    for (uint32_t w = 0; w < (b.spec ? 0u : b.nwg); ++w) {
        const uint32_t f = b.wg_frame[w];
        const EntFrame& F = b.frames[f];
        const uint32_t gl = w - F.wg_base;
        bool joined = gl == 0;
        for (int t = 0; t < kWarm && !joined; ++t)
            joined = same_state(b.wentries[static_cast<uint64_t>(w) * kWarm + t],
                                b.entries[F.sub_base + static_cast<uint64_t>(group_sub(gl, t))]);
        b.linked[w] = joined ? 1u : 0u;
        if (!joined) b.status[f] |= kStatusFallback;
    }
    // repair
    for (uint32_t f = 0; f < b.nframes; ++f) {
        if (!(b.status[f] & kStatusFallback)) continue;
        BlockInfo blocks[kMaxBpm];
        fill_blocks(blocks, b.frames[f]);
        repair_frame(b, f, b.tabs + b.frames[f].tab_base, blocks);
    }
    // write (group order = subsequence order)
    alignas(16) int16_t stage[kStageStride];
    for (uint32_t f = 0; f < b.nframes; ++f) {
        const EntFrame& F = b.frames[f];
        BlockInfo blocks[kMaxBpm];
        fill_blocks(blocks, F);
        const RunCtx c = make_ctx(b, F, b.tabs + F.tab_base, blocks);
        SubStats pre = stats_identity();
        for (uint32_t i = 0; i < F.nsub; ++i) {
            for (uint32_t piece = 0; piece < write_pieces(b); ++piece) {   // as ent_write_kernel
                SubStats lead;
                const uint64_t entry = piece_entry(b, F, i, piece, lead);
                const SubStats p = stats_combine(pre, lead);
                RunOut o;
                o.coefs = b.coefs + F.coef_off * 64;
                o.stage = stage;
                o.blk = p.nblk;
                o.nblocks = F.nblocks;
                o.nout = F.nout;
                o.pred[0] = p.dc[0];
                o.pred[1] = p.dc[1];
                o.pred[2] = p.dc[2];
                SubStats s = stats_identity();
                run<true>(c, entry, piece_stop(b, i, piece), s, &o);
                if (s.flags & kError) b.status[f] |= kStatusCorrupt;
                if (piece + 1 == write_pieces(b) && i == F.nsub - 1 && p.nblk + s.nblk != F.nblocks)
                    b.status[f] |= kStatusCount;
            }
            pre = stats_combine(pre, sub_stats(b, F, i));
        }
    }
}

}  // namespace

// Lead-in of the speculative sync's spec runs (HJD_SPEC_LEAD overrides; tuning).
// A chain breaks where none of a subsequence's spec runs has met the true
// decode by its checkpoint; a longer lead-in makes that rarer and costs every
// spec run its length.  Measured FHD single images (ms at W = 512 / 1536,
// profiles/r06zx_spec_lead.json): bench q90 4:2:0 0.40 / 0.46 (no break),
// another q90 4:2:0 at the same 164 bits per block 0.61 / 0.46 (2 breaks),
// q90 4:4:4 0.96 / 0.47 (9 breaks), q93 4:2:0 1.10 / 0.75 (19 / 3 breaks;
// none at 2048, host emulation).  Bits per block do not tell these apart, so
// the decoder goes by its own history: a batch whose chain needed a repair
// moves the next batches one step up the ladder, and kLeadBatches clean
// batches move them one step down (a camera's frames look alike).  A repair
// right after a step down doubles the clean run the next step down waits for
// (up to kLeadBatchesMax), so a stream that needs the long lead-in pays a
// repaired frame ever more rarely.
constexpr uint32_t kLeadLadder[] = {512, 1536, 2560};
constexpr uint32_t kLeadSteps = sizeof(kLeadLadder) / sizeof(kLeadLadder[0]), kLeadBatches = 32,
                   kLeadBatchesMax = 4096;
uint32_t spec_lead_bits(uint32_t step)
{
    const char* e = getenv("HJD_SPEC_LEAD");   // read per batch (~100 ns): tests switch it in-process
    return e ? static_cast<uint32_t>(atoi(e)) : kLeadLadder[step < kLeadSteps ? step : kLeadSteps - 1];
}

// ---------------------------------------------------------------------------
// Batch object
// ---------------------------------------------------------------------------
namespace {
void gdec_early_pull(DestuffHook* h, size_t done);
}

struct hjd_gdec {
    hjd_ctx* ctx = nullptr;
    int device = 0, num_cu = 256;
    bool gpu = true;
    Caps caps{};
    HdrOffsets H{};
    uint8_t* h_stage = nullptr;         // pinned (gpu) or malloc (emulation): header + data
    uint8_t* d_blob = nullptr;
    uint64_t* d_entries = nullptr;
    SubStats* d_stats = nullptr;
    uint64_t* d_mids = nullptr;
    SubStats* d_stats1 = nullptr;
    uint64_t* d_wentries = nullptr;
    uint32_t* d_linked = nullptr;
    SubStats* d_agg = nullptr;
    uint32_t* h_status = nullptr;       // pinned; the device's status words are in the batch header (H.status)
    int16_t* d_coefs = nullptr;
    uint8_t* d_raw = nullptr;           // raw scan bytes of device-destuffed frames (same offsets as the data area)
    uint32_t* d_tiles = nullptr;        // destuff scratch [3][max_tiles]
    bool spec = false;                  // speculative sync (latency decoders: ent_spec/cand/sync_spec kernels)
    SpecRec* d_spec = nullptr;          // [max_subs][kMaxBpm]
    CandRec* d_cand = nullptr;
    uint8_t* d_cmap = nullptr;
    uint8_t* d_cslot = nullptr;
    uint32_t* d_chainfn = nullptr;
    uint32_t* d_chain_broken = nullptr;
    SubStats* d_agg2 = nullptr;         // [group] (ent_chain_lb_kernel)
    uint32_t chain_epoch = 0;           // the last launch's look-back tag
    int64_t chain_fn_rows = 0;      // capacity of d_chainfn in chunk functions
    uint8_t* d_steps = nullptr;         // [table][1 << kStepBits] (ent_steps_kernel)
    std::vector<uint8_t> steps_tabs;    // the tables d_steps was last derived from (host copy, batch order)
    double host_us[3] = {0, 0, 0};      // host time per phase (wait for staging, stage, issue): HJD_GDEC_HOST_TIMES
    int64_t host_calls = 0;
    hipEvent_t staged = nullptr, done = nullptr;
    int64_t last_h2d = 0;               // bytes the last issue moved host -> device
    int64_t last_host_scan_bytes = 0;   // scan bytes the host CPU read + wrote for the staged frames
    bool pending = false;
    bool staged_by_done = false;        // the last issue pulled its staging: `done` also means staged
    uint32_t batch_sub_bits = 0;        // S of the batch being assembled (0: caps.sub_bits)
    bool batch_spec = false;            // the pending batch took the speculative sync
    uint32_t lead_step = 0;             // spec_lead_bits' ladder step for the next batch
    uint32_t lead_left = 0;             // clean batches before it steps down
    uint32_t lead_hold = kLeadBatches;  // the clean run a step down waits for
    bool lead_stepped_down = false;     // the batch in flight runs one step lower than the last
    hipStream_t early_stream = nullptr; // this call's stream when its lone image may be pulled early
    bool early = false;                 // early pull enabled for this call
    size_t prepulled = 0;               // data-area bytes of frame 0 already pulled (gdec_early_pull)
    std::vector<Prepared> frames;
    size_t data_used = 0;
    int nframes_issued = 0;
    int first_error = HJD_OK;

    // host-side work arrays for emulation
    std::vector<uint64_t> e_entries, e_wentries, e_mids;
    std::vector<uint32_t> e_linked;
    std::vector<SubStats> e_stats, e_agg, e_stats1;
    std::vector<uint32_t> e_status;
    std::vector<SpecRec> e_spec;
    std::vector<CandRec> e_cand;
    std::vector<uint8_t> e_cmap, e_cslot;

    uint8_t* data_area() { return h_stage + caps.data; }
    // data_need() of every frame: the scan bytes, plus pad and alignment per scan
    size_t data_cap() const { return static_cast<size_t>(caps.max_scan_bytes) +
                                     (kDataPad + 16) * kMaxScans * static_cast<size_t>(caps.max_frames); }
    std::vector<int> scan_file;         // file of each entropy frame past the first n (a file's further scans)

    int wait_staging();
    int stage_frames(const uint8_t* const* datas, const size_t* sizes, int n);
    // Parse + destuff one JPEG into frames[i] / the data area at data_off
    // (thread-safe for distinct i and disjoint data ranges).
    int prepare_frame(int i, const uint8_t* data, size_t size, size_t data_off, size_t cap, int mode,
                      uint64_t raw_off);
    // Destuff mode of a JPEG and, for the device modes, its place in the raw
    // area.  fits = false when the raw scan does not fit the raw area, or
    // data_room (free bytes of the data area) minus `reserve` (bytes kept for
    // the frames still to come); with host_fallback, HJD_DESTUFF=auto then
    // picks the host path instead (fits stays true).
    int plan_raw(const uint8_t* data, size_t size, RawCursor& cur, int& mode, uint64_t& raw_off, bool& fits,
                 size_t data_room, uint64_t reserve, bool host_fallback);
    // Lays out and fills the header for the staged frames (pixel records too
    // when d_outs is given); returns the device view (pointers into `blob`).
    int assemble(uint8_t* blob, int16_t* coefs, int64_t* block_offsets, void* const* d_outs, const int32_t* pitches,
                 EntBatchDev& d);
    // pixel-kernel launch groups, one per sampling (hjd_internal::SamplingGeom::index)
    static constexpr int kClasses = 6;
    static constexpr int kClassSampling[kClasses] = {HJD_YUV444, HJD_YUV420,      HJD_YUV422,
                                                     HJD_GRAY,   HJD_YUV411_H4V1, HJD_YUV440};
    int nrec[kClasses] = {};
    int64_t tasks[kClasses] = {};
    uint8_t* out_base[kClasses] = {};
    int out_format = HJD_OUT_BGRX;      // pixel output format (hjd_gdec_set_output_format)
};

int hjd_gdec::wait_staging()
{
    if (gpu && pending) {
        HJD_HIP(hipSetDevice(device));
        HJD_HIP(hipEventSynchronize(staged_by_done ? done : staged));
    }
    return HJD_OK;
}

namespace {

// HJD_DESTUFF: "host" (always destuff on the host), "device" (always on the
// GPU; unpinned bytes are memcpy'd raw into staging), default "auto": on the
// GPU when the caller's bytes are pinned host memory (hipHostMalloc'd or
// hipHostRegister'ed, e.g. hjd_host_register), so the host CPU never touches
// the scan, on the host otherwise.
int destuff_policy()
{
    const char* e = getenv("HJD_DESTUFF");   // read per frame (~100 ns): tests switch it in-process
    if (e && !strcmp(e, "host")) return 0;
    if (e && !strcmp(e, "device")) return 2;
    return 1;
}

bool pinned_host(const void* p, size_t n)
{
    if (!p || !n) return false;
    for (const void* q : {p, static_cast<const void*>(static_cast<const uint8_t*>(p) + n - 1)}) {
        hipPointerAttribute_t a;
        if (hipPointerGetAttributes(&a, q) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (a.type != hipMemoryTypeHost) return false;
    }
    return true;
}

}  // namespace

int hjd_gdec::plan_raw(const uint8_t* data, size_t size, RawCursor& cur, int& mode, uint64_t& raw_off, bool& fits,
                       size_t data_room, uint64_t reserve, bool host_fallback)
{
    mode = kDestuffHost;
    raw_off = 0;
    fits = true;
    const int pol = gpu ? destuff_policy() : 0;
    if (pol == 0 || !data) return HJD_OK;
    const bool pinned = pinned_host(data, size);
    if (pol == 2) mode = pinned ? kDestuffFromCaller : kDestuffFromStaging;
    else if (pinned) mode = kDestuffFromCaller;
    if (mode == kDestuffHost) return HJD_OK;
    hjd_internal::ScanHeader h;
    const int rc = hjd_internal::parse_scan_header(data, size, &h);
    if (rc) return rc;
    if (h.scan_offset >= size) return set_error(HJD_E_INVALID, "empty scan");
    if (h.extra_scans > 0) {   // several scans: destuffed (and their ends found) on the host
        mode = kDestuffHost;
        return HJD_OK;
    }
    const size_t raw = size - h.scan_offset;
    // the device path needs the raw scan (stuffing, markers and the bytes
    // after EOI included) in both the raw and the data area; the host path
    // only the destuffed bytes in the data area
    fits = align_up(raw + kDataPad, 16) + reserve <= data_room &&
           cur.place(data + h.scan_offset, raw, size, mode == kDestuffFromCaller, data_cap(), raw_off, reserve);
    if (!fits && host_fallback && pol == 1) {   // auto: destuff this one on the host instead
        mode = kDestuffHost;
        raw_off = 0;
        fits = true;
    }
    return HJD_OK;
}

int hjd_gdec::prepare_frame(int i, const uint8_t* data, size_t size, size_t data_off, size_t cap, int mode,
                            uint64_t raw_off)
{
    Prepared& p = frames[static_cast<size_t>(i)];
    p = Prepared();
    p.data_off = data_off;
    if (!data) return p.rc = set_error(HJD_E_INVALID, "frame %d: NULL data", i);
    if (cap <= kDataPad) return p.rc = set_error(HJD_E_INVALID, "scan bytes exceed the batch capacity");
    DestuffHook hook{SIZE_MAX, gdec_early_pull, this};
    int rc = prepare(data, size, data_area() + data_off, cap - kDataPad, p, mode, raw_off,
                     early && i == 0 && data_off == 0 ? &hook : nullptr);
    if (rc) return p.rc = rc;
    return HJD_OK;
}

int hjd_gdec::stage_frames(const uint8_t* const* datas, const size_t* sizes, int n)
{
    if (n <= 0 || n > caps.max_frames) return set_error(HJD_E_INVALID, "batch of %d frames (capacity %d)", n,
                                                        caps.max_frames);
    frames.assign(static_cast<size_t>(n), Prepared());
    data_used = 0;
    int64_t blocks = 0;
    RawCursor cur;
    // what the frames after i need at least in the data area, whichever path
    // they take: a frame with a device-destuffed scan is placed only if the
    // rest still fit, so a batch sized by its file bytes never fails on
    // placement.  A single-scan file needs its entropy-coded bytes plus pad
    // (destuffed or raw), a multi-scan file data_need() of its size; so a
    // batch sized by its scan bytes (hjd_gdec_create) keeps the device destuff
    // for its pinned files wherever their raw scans fit.
    std::vector<uint64_t> tail(static_cast<size_t>(n) + 1, 0);
    for (int i = n - 1; i >= 0; --i) {
        hjd_internal::ScanHeader h;
        const bool one_scan = datas[i] && hjd_internal::parse_scan_header(datas[i], sizes[i], &h) == HJD_OK &&
                              h.extra_scans == 0 && h.scan_offset <= sizes[i];
        tail[i] = tail[i + 1] + (one_scan ? align_up(sizes[i] - h.scan_offset + kDataPad, 16) : data_need(sizes[i]));
    }
    for (int i = 0; i < n; ++i) {
        if (data_used >= data_cap()) return set_error(HJD_E_INVALID, "scan bytes exceed the batch capacity");
        int mode;
        uint64_t raw_off;
        bool fits;
        int rc = plan_raw(datas[i], sizes[i], cur, mode, raw_off, fits, data_cap() - data_used, tail[i + 1], true);
        if (rc) return set_error(rc, "frame %d: %s", i, hjd_last_error());
        if (!fits) return set_error(HJD_E_INVALID, "scan bytes exceed the batch capacity");
        rc = prepare_frame(i, datas[i], sizes[i], data_used, data_cap() - data_used, mode, raw_off);
        if (rc) return set_error(rc, "frame %d: %s", i, hjd_last_error());
        data_used = align_up(frames[i].data_end(), 16);
        blocks += frames[i].out_blocks;
    }
    if (blocks > caps.max_blocks)
        return set_error(HJD_E_INVALID, "batch needs %lld blocks (capacity %lld)", static_cast<long long>(blocks),
                         static_cast<long long>(caps.max_blocks));
    return HJD_OK;
}

int hjd_gdec::assemble(uint8_t* blob, int16_t* coefs, int64_t* block_offsets, void* const* d_outs,
                       const int32_t* pitches, EntBatchDev& d)
{
    const int n = static_cast<int>(frames.size());
    const uint32_t S = batch_sub_bits ? batch_sub_bits : static_cast<uint32_t>(caps.sub_bits);
    // entropy frames: the n JPEGs' (first) scans, then the further scans of
    // multi-scan files (scan_file: their JPEG), all writing the JPEG's blocks
    std::vector<const Prepared*> ents;
    std::vector<int> ent_file;
    scan_file.clear();
    for (int i = 0; i < n; ++i) {
        ents.push_back(&frames[i]);
        ent_file.push_back(i);
    }
    for (int i = 0; i < n; ++i)
        for (const Prepared& q : frames[i].more) {
            ents.push_back(&q);
            ent_file.push_back(i);
            scan_file.push_back(i);
        }
    const int ne = static_cast<int>(ents.size());
    std::vector<uint64_t> file_coef(static_cast<size_t>(n), 0);
    uint64_t coef_off = 0;
    for (int i = 0; i < n; ++i) {
        file_coef[i] = coef_off;
        coef_off += static_cast<uint64_t>(frames[i].out_blocks);
    }
    size_t ntab = 0, nseg = 0, nwg = 0;
    for (const Prepared* p : ents) {
        ntab += static_cast<size_t>(p->ntab);
        nseg += p->seg_end.size();
        const uint32_t ns = (p->data_bits + S - 1) / S;
        nwg += frame_groups(ns);
    }
    HdrOffsets& o = H;
    o.frames = 0;
    o.tabs = align_up(sizeof(EntFrame) * ne, kAlign);
    o.seg = align_up(o.tabs + sizeof(HuffLut) * ntab, kAlign);
    o.wg = align_up(o.seg + 4 * nseg, kAlign);
    o.recs = align_up(o.wg + 4 * nwg, kAlign);
    o.qt = align_up(o.recs + (d_outs ? sizeof(FrameRecord) * n : 0), kAlign);
    size_t ntiles = 0;
    for (const Prepared& p : frames)
        if (p.destuff != kDestuffHost)
            ntiles += (raw_region_len(static_cast<uint32_t>(p.raw_off & 15), p.raw_len) + kTileBytes - 1) / kTileBytes;
    o.rawf = align_up(o.qt + (d_outs ? 192 * 4 * static_cast<size_t>(n) : 0), kAlign);
    o.tilef = align_up(o.rawf + (ntiles ? sizeof(RawFrame) * ne : 0), kAlign);
    // per entropy frame status words, zero in the header's upload (no memset)
    o.status = align_up(o.tilef + 4 * ntiles, kAlign);
    o.used = align_up(o.status + 4 * (2 * static_cast<size_t>(ne) + 1), kAlign);
    if (o.used > caps.hdr_cap || ntiles > static_cast<size_t>(caps.max_tiles))
        return set_error(HJD_E_INVALID, "batch header exceeds its capacity");

    EntFrame* ef = reinterpret_cast<EntFrame*>(h_stage + o.frames);
    memset(h_stage + o.status, 0, 4 * (2 * static_cast<size_t>(ne) + 1));
    HuffLut* tb = reinterpret_cast<HuffLut*>(h_stage + o.tabs);
    uint32_t* seg = reinterpret_cast<uint32_t*>(h_stage + o.seg);
    uint32_t* wgf = reinterpret_cast<uint32_t*>(h_stage + o.wg);
    uint32_t sub_base = 0, wg_base = 0, seg_base = 0, tab_base = 0;
    for (int e = 0; e < ne; ++e) {
        const Prepared& p = *ents[e];
        const Prepared& file = frames[ent_file[e]];
        EntFrame F;
        memset(&F, 0, sizeof(F));
        F.data_off = p.data_off;
        F.coef_off = file_coef[ent_file[e]];
        F.data_bits = p.data_bits;
        F.nsub = (p.data_bits + S - 1) / S;
        F.sub_base = sub_base;
        F.wg_base = wg_base;
        F.seg_base = seg_base;
        F.nseg = static_cast<uint32_t>(p.seg_end.size());
        F.nblocks = static_cast<uint32_t>(p.nblocks);
        F.tab_base = tab_base;
        F.ntab = static_cast<uint8_t>(p.ntab);
        F.bpm = static_cast<uint8_t>(p.bpm);
        F.sampling = static_cast<uint8_t>(file.sampling);
        F.layout = static_cast<uint8_t>(p.layout);
        memcpy(F.jinfo, p.jinfo, sizeof(F.jinfo));
        F.seg_blocks = F.nseg > 1 ? static_cast<uint32_t>(p.restart_mcus * p.bpm) : 0u;
        F.geo = p.geo;
        F.mcu_w = p.mcu_w;
        F.nout = static_cast<uint32_t>(file.out_blocks);
        ef[e] = F;
        memcpy(tb + tab_base, p.tabs, sizeof(HuffLut) * p.ntab);
        memcpy(seg + seg_base, p.seg_end.data(), 4 * p.seg_end.size());
        const uint32_t nw = frame_groups(F.nsub);
        for (uint32_t g = 0; g < nw; ++g) wgf[wg_base + g] = static_cast<uint32_t>(e);
        sub_base += F.nsub;
        wg_base += nw;
        seg_base += F.nseg;
        tab_base += p.ntab;
    }
    if (block_offsets)
        for (int i = 0; i < n; ++i) block_offsets[i] = static_cast<int64_t>(file_coef[i]);
    if (coef_off > static_cast<uint64_t>(caps.max_blocks) || sub_base > caps.max_subs || wg_base > caps.max_wgs)
        return set_error(HJD_E_INVALID, "batch exceeds the decoder's capacity");

    for (int k = 0; k < kClasses; ++k) {
        nrec[k] = 0;
        tasks[k] = 0;
        out_base[k] = nullptr;
    }
    if (d_outs) {   // pixel-kernel records grouped by sampling class (one launch each)
        FrameRecord* recs = reinterpret_cast<FrameRecord*>(h_stage + o.recs);
        int32_t* qtn = reinterpret_cast<int32_t*>(h_stage + o.qt);
        const int obytes = hjd_internal::out_format_bytes(out_format);
        const uintptr_t amask = out_format == HJD_OUT_BGRX ? 15 : 3;
        for (int i = 0; i < n; ++i) {
            const Prepared& p = frames[i];
            if (!d_outs[i] || !pitches || pitches[i] < obytes * p.width || (pitches[i] & 3) ||
                (reinterpret_cast<uintptr_t>(d_outs[i]) & amask))
                return set_error(HJD_E_INVALID,
                                 "frame %d: bad output buffer or pitch (BGRX: 16-byte aligned, >= 4*width; "
                                 "BGR24: 4-byte aligned, >= 3*width)", i);
            ++nrec[sampling_class(p.sampling)];
        }
        int r[kClasses];
        for (int k = 0, acc = 0; k < kClasses; acc += nrec[k], ++k) r[k] = acc;
        for (int i = 0; i < n; ++i) {
            const Prepared& p = frames[i];
            const int sidx = sampling_class(p.sampling);
            if (!out_base[sidx]) out_base[sidx] = static_cast<uint8_t*>(d_outs[i]);
            const int qti[3] = {3 * i, 3 * i + 1, 3 * i + 2};
            FrameRecord rec;
            const int64_t t = hjd_internal::make_frame_record(
                p.width, p.height, p.sampling, static_cast<int64_t>(ef[i].coef_off),
                static_cast<int64_t>(static_cast<uint8_t*>(d_outs[i]) - out_base[sidx]), pitches[i], qti, &rec,
                out_format);
            if (t < 0) return static_cast<int>(t);
            rec.task_begin = tasks[sidx];
            tasks[sidx] += t;
            recs[r[sidx]++] = rec;
            for (int c = 0; c < 3; ++c)
                for (int k = 0; k < 64; ++k) qtn[(3 * i + c) * 64 + kZigzag[k]] = p.qt[c][k];
        }
    }

    d.ntiles = static_cast<uint32_t>(ntiles);
    uint32_t max_nsub = 0;
    for (int e = 0; e < ne; ++e) max_nsub = ef[e].nsub > max_nsub ? ef[e].nsub : max_nsub;
    d.chain_chunks = (max_nsub + kChainChunk - 1) / kChainChunk;
    if (d.chain_chunks == 0) d.chain_chunks = 1;
    d.chainfn = nullptr;
    d.chain_broken = nullptr;
    d.chain_epoch = 0;
    d.agg2 = nullptr;
    d.host_status = nullptr;
    d.spec = nullptr;
    d.cand = nullptr;
    d.cmap = nullptr;
    d.cslot = nullptr;
    d.spec_lead = 0;
    d.nsub_total = sub_base;
    d.rawf = nullptr;
    d.tile_frame = nullptr;
    if (ntiles) {
        RawFrame* rf = reinterpret_cast<RawFrame*>(h_stage + o.rawf);
        uint32_t* tf = reinterpret_cast<uint32_t*>(h_stage + o.tilef);
        uint32_t tbase = 0;
        for (int e = 0; e < ne; ++e) {   // further scans are host-destuffed (ntiles 0)
            const Prepared& p = *ents[e];
            RawFrame r{p.raw_off, p.raw_len, static_cast<uint32_t>(p.raw_off & 15), tbase, 0, 0, 0};
            if (p.destuff != kDestuffHost) {
                r.ntiles = (raw_region_len(r.begin, p.raw_len) + kTileBytes - 1) / kTileBytes;
                for (uint32_t k = 0; k < r.ntiles; ++k) tf[tbase + k] = static_cast<uint32_t>(e);
                tbase += r.ntiles;
            }
            rf[e] = r;
        }
        d.rawf = reinterpret_cast<RawFrame*>(blob + o.rawf);
        d.tile_frame = reinterpret_cast<const uint32_t*>(blob + o.tilef);
    }
    d.frames = reinterpret_cast<const EntFrame*>(blob + o.frames);
    d.tabs = reinterpret_cast<const HuffLut*>(blob + o.tabs);
    d.seg_end = reinterpret_cast<const uint32_t*>(blob + o.seg);
    d.wg_frame = reinterpret_cast<const uint32_t*>(blob + o.wg);
    d.data = blob + caps.data;
    d.coefs = coefs;
    d.nframes = static_cast<uint32_t>(ne);
    d.nwg = wg_base;
    d.sub_bits = S;
    d.ntab_max = 1;
    for (const Prepared* p : ents) d.ntab_max = std::max<uint32_t>(d.ntab_max, static_cast<uint32_t>(p->ntab));
    d.ntab_total = tab_base;
    d.steps_g = nullptr;
    return HJD_OK;
}

namespace {

int gdec_alloc(hjd_gdec* g)
{
    const size_t total = g->caps.data + g->data_cap();
    if (!g->gpu) {
        g->h_stage = static_cast<uint8_t*>(calloc(1, total));
        if (!g->h_stage) return set_error(HJD_E_NOMEM, "staging allocation");
        return HJD_OK;
    }
    HJD_HIP(hipSetDevice(g->device));
    HJD_HIP(hipHostMalloc(reinterpret_cast<void**>(&g->h_stage), total, hipHostMallocDefault));
    HJD_HIP(hipHostMalloc(reinterpret_cast<void**>(&g->h_status),
                          4 * kMaxScans * static_cast<size_t>(g->caps.max_frames), hipHostMallocDefault));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_blob), total));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_entries), 8 * static_cast<size_t>(g->caps.max_subs)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_stats), sizeof(SubStats) * static_cast<size_t>(g->caps.max_subs)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_mids), 8 * static_cast<size_t>(g->caps.max_subs)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_stats1), sizeof(SubStats) * static_cast<size_t>(g->caps.max_subs)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_wentries), 8 * kWarm * static_cast<size_t>(g->caps.max_wgs)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_linked), 4 * static_cast<size_t>(g->caps.max_wgs)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_agg), sizeof(SubStats) * static_cast<size_t>(g->caps.max_wgs)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_coefs), 128 * static_cast<size_t>(g->caps.max_blocks)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_raw), g->data_cap()));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_tiles), 12 * static_cast<size_t>(g->caps.max_tiles)));
    HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_steps),
                      (static_cast<size_t>(kMaxTables) * kMaxScans * static_cast<size_t>(g->caps.max_frames)) << kStepBits));
    if (g->spec) {
        const size_t n = static_cast<size_t>(g->caps.max_subs);
        HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_spec), sizeof(SpecRec) * kMaxBpm * n));
        HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_cand), sizeof(CandRec) * kCandRow * n));
        HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_cmap), kSlotRow * n));
        HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_cslot), n + 16));
        // chunk functions: [entropy frame][chunks of the largest frame]
        const size_t ef = kMaxScans * static_cast<size_t>(g->caps.max_frames);
        g->chain_fn_rows = static_cast<int64_t>(ef * (n / kChainChunk + 1));
        HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_chainfn), 4 * kLbWords * static_cast<size_t>(g->chain_fn_rows)));
        HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_chain_broken), 4 * ef));
        HJD_HIP(hipMemset(g->d_chain_broken, 0, 4 * ef));
        HJD_HIP(hipMemset(g->d_chainfn, 0, 4 * kLbWords * static_cast<size_t>(g->chain_fn_rows)));
        HJD_HIP(hipMalloc(reinterpret_cast<void**>(&g->d_agg2), sizeof(SubStats) * static_cast<size_t>(g->caps.max_wgs)));
    }
    HJD_HIP(hipEventCreateWithFlags(&g->staged, hipEventDisableTiming));
    HJD_HIP(hipEventCreateWithFlags(&g->done, hipEventDisableTiming));
    return HJD_OK;
}

// Entropy kernels on `stream`; coefficients land in b.coefs.
int launch_entropy(hjd_gdec* g, const EntBatchDev& b, hipStream_t s)
{
    if (b.nwg == 0) return HJD_OK;
    if (b.ntiles) {
        hipLaunchKernelGGL(destuff_count_kernel, dim3(b.ntiles), dim3(kTileThreads), 0, s, b);
        HJD_HIP(hipGetLastError());
        hipLaunchKernelGGL(destuff_scan_kernel, dim3(b.nframes), dim3(kTileThreads), 0, s, b);
        HJD_HIP(hipGetLastError());
        hipLaunchKernelGGL(destuff_write_kernel, dim3(b.ntiles), dim3(kTileThreads), 0, s, b);
        HJD_HIP(hipGetLastError());
    }
    // the step tables depend on the Huffman tables only: a batch whose tables
    // (in batch order) are the previous batch's reuses them
    const uint8_t* tabs_h = g->h_stage + g->H.tabs;
    const size_t tabs_n = sizeof(HuffLut) * b.ntab_total;
    if (g->steps_tabs.size() != tabs_n || memcmp(g->steps_tabs.data(), tabs_h, tabs_n) != 0) {
        hipLaunchKernelGGL(ent_steps_kernel, dim3(b.ntab_total, kStepGroups), dim3(kStepsThreads), 0, s, b);
        HJD_HIP(hipGetLastError());
        g->steps_tabs.assign(tabs_h, tabs_h + tabs_n);
    }
    if (b.spec) {   // speculative sync: latency decoders
        const size_t tl = (sizeof(HuffLut) + (1u << kStepBits)) * b.ntab_max;
        hipLaunchKernelGGL(ent_spec_kernel, dim3(b.nwg, kMaxBpm), dim3(kGroupSubs), tl, s, b);
        HJD_HIP(hipGetLastError());
        hipLaunchKernelGGL(ent_cand_kernel, dim3(b.nwg, kMaxBpm), dim3(kGroupSubs), tl, s, b);
        HJD_HIP(hipGetLastError());
        if (b.chain_broken)   // chunks in parallel (+ group records; a broken frame's last chunk walks it)
            hipLaunchKernelGGL(ent_chain_lb_kernel, dim3(b.chain_chunks, b.nframes), dim3(kChainThreads), 0, s, b);
        else   // every frame walked
            hipLaunchKernelGGL(ent_chain_kernel, dim3(b.nframes), dim3(kChainThreads), 0, s, b);
        HJD_HIP(hipGetLastError());
    } else {
        hipLaunchKernelGGL(ent_sync_kernel, dim3(b.nwg), dim3(kGroupSubs), sync_lds_bytes(b.ntab_max), s, b);
        HJD_HIP(hipGetLastError());
        hipLaunchKernelGGL(ent_link_kernel, dim3((b.nwg + 255) / 256), dim3(256), 0, s, b);
        HJD_HIP(hipGetLastError());
    }
    if (!b.spec) {   // the chain kernel repairs its chains itself: never a fallback
        hipLaunchKernelGGL(ent_fallback_kernel, dim3(b.nframes), dim3(64), 0, s, b);
        HJD_HIP(hipGetLastError());
    }
    constexpr size_t kStageBytes = sizeof(int16_t) * kWriteThreads * kStageStride;
    hipLaunchKernelGGL(ent_write_kernel, dim3(b.nwg, write_pieces(b)), dim3(kWriteThreads),
                       kStageBytes + sizeof(HuffLut) * b.ntab_max, s, b);
    HJD_HIP(hipGetLastError());
    return HJD_OK;
}

// Upload the staged frames and run the entropy kernels (+ the pixel kernel
// when d_outs is given) on stream s.
struct HostCopy {
    void* host;          // destination (pinned host memory recommended)
    int32_t host_pitch;
    int32_t width, height;
};

// Latency decoders: the staged bytes of a batch whose scans were all
// destuffed on the host (its header, then its data area) are pulled from the
// pinned staging by one kernel instead of two DMA copies: 1 MB moves in 23 us
// against 31 us by DMA (tools/h2d_probe.hip, profiles/r06y_h2d_probe.json;
// 64 workgroups beat 256 and 1024), and the kernel replaces the copy calls.
// Staging and blob share their layout, so a segment is an offset and a length
// (16-B multiples: the header is kAlign-aligned, a data run ends in its pad).
constexpr uint64_t kDenseBitsPerBlock = 200;   // (a q90 FHD 4:2:0 frame: 164; q95: 232; q100: 436)
// the round-based S of a dense scan: the first tier whose bits per block bound
// it (best S measured per FHD frame: q95 232 / 243 -> 1024, q97 286 / 301 and
// q98 322 -> 2048, q99 388 and q100 436 -> 8192; profiles/r06zz_dense_sub_bits.json)
constexpr struct { uint64_t bits_per_block; uint32_t sub_bits; } kDenseTiers[] = {
    {260, 1024}, {360, 2048}, {0, 8192}};   // (the last: everything denser)
constexpr int kPullSegs = 4;
constexpr int kPullBlocks = 64;
constexpr int kPullThreads = 256;
struct PullSegs {
    uint64_t off[kPullSegs];     // 16-B words
    uint64_t words[kPullSegs];
    uint32_t n;
};

__global__ __launch_bounds__(kPullThreads) void pull_kernel(const u32x4* src, u32x4* dst, PullSegs p)
{
    const uint64_t stride = static_cast<uint64_t>(gridDim.x) * kPullThreads;
    for (uint32_t k = 0; k < p.n; ++k)
        for (uint64_t w = blockIdx.x * static_cast<uint64_t>(kPullThreads) + threadIdx.x; w < p.words[k]; w += stride)
            dst[p.off[k] + w] = src[p.off[k] + w];
}

// DestuffHook::fire of a latency decoder's lone image: pull the destuffed
// bytes that are final so far (16-B words) while the host destuffs the rest;
// gdec_issue pulls the remainder with the header.  One early pull per call
// (each costs a launch on the host, ~5 us: two measured no better).
void gdec_early_pull(DestuffHook* h, size_t done)
{
    hjd_gdec* g = static_cast<hjd_gdec*>(h->ctx);
    h->next = SIZE_MAX;
    const size_t upto = done & ~static_cast<size_t>(15);
    if (upto <= g->prepulled) return;
    PullSegs segs{};
    segs.off[0] = (g->caps.data + g->prepulled) / 16;   // frame 0: data_off 0
    segs.words[0] = (upto - g->prepulled) / 16;
    segs.n = 1;
    if (hipSetDevice(g->device) != hipSuccess) return;
    if (g->pending && hipStreamWaitEvent(g->early_stream, g->done, 0) != hipSuccess) return;
    hipLaunchKernelGGL(pull_kernel, dim3(kPullBlocks), dim3(kPullThreads), 0, g->early_stream,
                       reinterpret_cast<const u32x4*>(g->h_stage), reinterpret_cast<u32x4*>(g->d_blob), segs);
    if (hipGetLastError() == hipSuccess) g->prepulled = upto;
}

int gdec_issue(hjd_gdec* g, void* const* d_outs, const int32_t* pitches, int16_t* coefs_out, int64_t* block_offsets,
               hipStream_t s, const HostCopy* host = nullptr)
{
    HJD_HIP(hipSetDevice(g->device));
    const int n = static_cast<int>(g->frames.size());
    int16_t* coefs = coefs_out ? coefs_out : g->d_coefs;
    // Dense scans sync slowly: at S = 512 a q95 FHD frame breaks the
    // speculative chain ~200 times and a q100 one ~3,600 times, each break a
    // serial single-thread repair (8 ms and worse per image).  Above
    // kDenseBitsPerBlock a latency decoder takes the round-based sync instead,
    // at longer subsequences the denser the scan (kDenseTiers: q95 FHD 4:2:0
    // 1.4 ms at S = 1024; q98 2.4 at 2048 against 6.0 at 1024; q100 7.6 at 8192
    // against 14 at 2048; tools/fhd_env_sweep.py).  Never shorter than the
    // decoder's S (its capacity is sized for that).
    bool spec = g->spec;
    g->batch_sub_bits = 0;
    if (spec) {
        uint64_t bits = 0, blocks = 0;
        for (const Prepared& p : g->frames) {
            bits += p.data_bits;
            blocks += static_cast<uint64_t>(p.nblocks);
            for (const Prepared& q : p.more) {
                bits += q.data_bits;
                blocks += static_cast<uint64_t>(q.nblocks);
            }
        }
        if (bits > kDenseBitsPerBlock * blocks) {
            spec = false;
            const char* e = getenv("HJD_DENSE_SUB_BITS");   // tuning: the dense scans' S
            constexpr size_t nt = sizeof(kDenseTiers) / sizeof(kDenseTiers[0]);
            size_t t = 0;
            while (t + 1 < nt && bits > kDenseTiers[t].bits_per_block * blocks) ++t;
            const uint32_t want = e ? static_cast<uint32_t>(atoi(e)) : kDenseTiers[t].sub_bits;
            g->batch_sub_bits = std::max(want, static_cast<uint32_t>(g->caps.sub_bits));
        }
    }
    g->batch_spec = spec;
    EntBatchDev b;
    int rc = g->assemble(g->d_blob, coefs, block_offsets, d_outs, pitches, b);
    if (rc) return rc;
    b.entries = g->d_entries;
    b.stats = g->d_stats;
    b.mids = g->d_mids;
    b.stats1 = g->d_stats1;
    b.wentries = g->d_wentries;
    b.linked = g->d_linked;
    b.agg = g->d_agg;
    b.status = reinterpret_cast<uint32_t*>(g->d_blob + g->H.status);
    if (b.nwg) b.host_status = g->h_status;   // the write kernel delivers the status words
    b.raw = g->d_raw;
    b.tiles = g->d_tiles;
    b.steps_g = g->d_steps;
    if (spec) {
        b.spec = g->d_spec;
        b.cand = g->d_cand;
        b.cmap = g->d_cmap;
        b.cslot = g->d_cslot;
        b.spec_lead = spec_lead_bits(g->lead_step);
        if (static_cast<int64_t>(b.chain_chunks) * b.nframes <= g->chain_fn_rows) {
            b.chainfn = g->d_chainfn;
            b.chain_broken = g->d_chain_broken;
            b.agg2 = g->d_agg2;
            g->chain_epoch = g->chain_epoch % 0xFFFFFFu + 1u;   // 1 .. 2^24 - 1
            b.chain_epoch = g->chain_epoch;
        }
    }
    // the device buffers are reused: order this call after the previous one
    // (which may have been issued on another stream)
    if (g->pending) HJD_HIP(hipStreamWaitEvent(s, g->done, 0));
    bool pull = g->spec;   // latency decoders, every scan host-destuffed (one data run)
    for (const Prepared& p : g->frames) pull = pull && p.destuff == kDestuffHost;
    PullSegs segs{};
    if (pull) {
        segs.off[0] = 0;
        segs.words[0] = g->H.used / 16;
        segs.n = 1;
    } else {
        HJD_HIP(hipMemcpyAsync(g->d_blob, g->h_stage, g->H.used, hipMemcpyHostToDevice, s));
    }
    // scan bytes: runs of consecutive frames staged the same way move in one copy
    // (host-destuffed -> data area; raw in staging -> raw area); raw bytes in the
    // caller's pinned memory go straight from there to the raw area.
    int64_t moved = static_cast<int64_t>(g->H.used), host_bytes = 0;
    std::vector<void*> bd, bs;          // caller-pinned raw scans: one batched DMA submission
    std::vector<size_t> bn;
    std::vector<std::pair<int, int>> bf;   // frames [first, last) each copy covers
    for (int i = 0; i < n;) {
        const Prepared& p = g->frames[i];
        const size_t len = p.destuff == kDestuffHost ? p.data_bits / 8 : p.raw_len;
        host_bytes += p.destuff == kDestuffHost ? static_cast<int64_t>(p.raw_len) + static_cast<int64_t>(len)
                    : p.destuff == kDestuffFromStaging ? 2 * static_cast<int64_t>(len) : 0;
        if (p.destuff == kDestuffFromCaller) {
            // a run of scans placed at their distance in the caller's memory moves in one DMA
            int j = i + 1;
            size_t span = len;
            while (j < n && g->frames[j].destuff == kDestuffFromCaller && g->frames[j].raw_src > p.raw_src &&
                   g->frames[j].raw_off - p.raw_off == static_cast<uint64_t>(g->frames[j].raw_src - p.raw_src)) {
                span = static_cast<size_t>(g->frames[j].raw_src - p.raw_src) + g->frames[j].raw_len;
                ++j;
            }
            bd.push_back(g->d_raw + p.raw_off);
            bs.push_back(const_cast<uint8_t*>(p.raw_src));
            bn.push_back(span);
            bf.emplace_back(i, j);
            moved += static_cast<int64_t>(span);
            i = j;
            continue;
        }
        if (p.destuff == kDestuffFromStaging) {
            HJD_HIP(hipMemcpyAsync(g->d_raw + p.raw_off, g->h_stage + g->caps.data + p.data_off, len,
                                   hipMemcpyHostToDevice, s));
            moved += static_cast<int64_t>(len);
            ++i;
            continue;
        }
        int j = i + 1;                   // host-destuffed: one copy per run of frames (all their scans)
        size_t hi = p.data_end();
        for (const Prepared& q : p.more) host_bytes += static_cast<int64_t>(q.data_bits / 8);
        while (j < n && g->frames[j].destuff == kDestuffHost) {
            const Prepared& q = g->frames[j];
            hi = q.data_end();
            host_bytes += static_cast<int64_t>(q.raw_len) + q.data_bits / 8;
            for (const Prepared& r : q.more) host_bytes += static_cast<int64_t>(r.data_bits / 8);
            ++j;
        }
        uint8_t* dst = g->d_blob + g->caps.data + p.data_off;
        if (pull && segs.n < kPullSegs) {
            const size_t pre = i == 0 ? g->prepulled : 0;   // (frame 0 starts the data area)
            segs.off[segs.n] = (g->caps.data + p.data_off + pre) / 16;
            segs.words[segs.n] = (hi - p.data_off - pre + 15) / 16;
            ++segs.n;
        } else {
            HJD_HIP(hipMemcpyAsync(dst, g->h_stage + g->caps.data + p.data_off, hi - p.data_off, hipMemcpyHostToDevice, s));
        }
        moved += static_cast<int64_t>(hi - p.data_off);
        i = j;
    }
    if (pull) {
        hipLaunchKernelGGL(pull_kernel, dim3(kPullBlocks), dim3(kPullThreads), 0, s,
                           reinterpret_cast<const u32x4*>(g->h_stage), reinterpret_cast<u32x4*>(g->d_blob), segs);
        HJD_HIP(hipGetLastError());
    }
    // (hipMemcpyBatchAsync would submit these at once, but the HIP runtime this
    // library shares with PyTorch -- DESIGN.md s8 -- predates it)
    for (size_t k = 0; k < bd.size(); ++k) {
        if (hipMemcpyAsync(bd[k], bs[k], bn[k], hipMemcpyHostToDevice, s) == hipSuccess) continue;
        // A merged span can cross from one pinned allocation into another (the
        // caller's buffers merely lie close together), which the DMA rejects
        // before queueing anything: copy those scans one by one.
        (void)hipGetLastError();
        if (bf[k].second - bf[k].first < 2)
            return set_error(HJD_E_HIP, "hipMemcpyAsync of a pinned scan (%zu bytes) failed", bn[k]);
        for (int f = bf[k].first; f < bf[k].second; ++f) {
            const Prepared& q = g->frames[f];
            HJD_HIP(hipMemcpyAsync(g->d_raw + q.raw_off, const_cast<uint8_t*>(q.raw_src), q.raw_len,
                                   hipMemcpyHostToDevice, s));
        }
    }
    g->last_h2d = moved;
    g->last_host_scan_bytes = host_bytes;
    // (pulled: the staging is free when `done` fires -- an event between the
    // pull and the first entropy kernel delayed that kernel by ~6 us, and a
    // latency decoder's next call waits for `done` anyway)
    if (!pull) HJD_HIP(hipEventRecord(g->staged, s));
    g->staged_by_done = pull;
    g->pending = true;
    // a multi-scan file's non-interleaved scans leave its MCU-padding blocks
    // uncoded: they must read as zeros (as the host decoder's)
    {
        size_t first = 0;
        for (int i = 0; i < n; ++i) {
            const Prepared& p = g->frames[i];
            if (!p.more.empty())
                HJD_HIP(hipMemsetAsync(coefs + first * 64, 0, static_cast<size_t>(p.out_blocks) * 128, s));
            first += static_cast<size_t>(p.out_blocks);
        }
    }
    rc = launch_entropy(g, b, s);
    if (rc) return rc;
    if (d_outs) {
        int r0 = 0;
        for (int sidx = 0; sidx < hjd_gdec::kClasses; ++sidx) {
            if (!g->nrec[sidx]) continue;
            rc = hjd_internal::launch_decode(
                g->device, g->num_cu, hjd_gdec::kClassSampling[sidx], HJD_IN_Q16_ZIGZAG, 0, coefs,
                reinterpret_cast<const int32_t*>(g->d_blob + g->H.qt),
                reinterpret_cast<const FrameRecord*>(g->d_blob + g->H.recs) + r0, g->nrec[sidx], g->tasks[sidx],
                g->out_base[sidx], s, 0, g->out_format);
            if (rc) return rc;
            r0 += g->nrec[sidx];
        }
    }
    if (host && d_outs) {   // D2H sink: pixels of host-output frames back to the caller's memory
        for (int i = 0; i < n; ++i) {
            if (!host[i].host) continue;
            HJD_HIP(hipMemcpy2DAsync(host[i].host, static_cast<size_t>(host[i].host_pitch), d_outs[i],
                                     static_cast<size_t>(pitches[i]),
                                     static_cast<size_t>(host[i].width) * hjd_internal::out_format_bytes(g->out_format),
                                     static_cast<size_t>(host[i].height), hipMemcpyDeviceToHost, s));
        }
    }
    if (!b.host_status)
        HJD_HIP(hipMemcpyAsync(g->h_status, b.status, 4 * static_cast<size_t>(b.nframes), hipMemcpyDeviceToHost, s));
    HJD_HIP(hipEventRecord(g->done, s));
    g->nframes_issued = n;
    return HJD_OK;
}

// Stage n JPEGs on the calling thread, then issue.
int gdec_run(hjd_gdec* g, const uint8_t* const* datas, const size_t* sizes, int n, void* const* d_outs,
             const int32_t* pitches, int16_t* coefs_out, int64_t* block_offsets, hipStream_t s)
{
    if (!g || !g->gpu || !datas || !sizes) return set_error(HJD_E_INVALID, "NULL argument");
    const auto t0 = std::chrono::steady_clock::now();
    int rc = g->wait_staging();
    if (rc) return rc;
    const auto t1 = std::chrono::steady_clock::now();
    g->early = g->spec && n == 1;   // a lone image may be pulled while it is destuffed
    g->early_stream = s;
    g->prepulled = 0;
    rc = g->stage_frames(datas, sizes, n);
    g->early = false;
    if (rc) {
        if (g->prepulled) (void)hipStreamSynchronize(s);   // an early pull still reads the staging
        return rc;
    }
    const auto t2 = std::chrono::steady_clock::now();
    rc = gdec_issue(g, d_outs, pitches, coefs_out, block_offsets, s);
    if (rc) return rc;
    const auto t3 = std::chrono::steady_clock::now();
    g->host_us[0] += std::chrono::duration<double, std::micro>(t1 - t0).count();
    g->host_us[1] += std::chrono::duration<double, std::micro>(t2 - t1).count();
    g->host_us[2] += std::chrono::duration<double, std::micro>(t3 - t2).count();
    ++g->host_calls;
    // The caller may reuse its bytes once this returns (include/hjd_host.h):
    // scans read by DMA straight from the caller's pinned memory must have
    // landed first.  Only the uploads are waited for, not the kernels.
    for (const Prepared& p : g->frames)
        if (p.destuff == kDestuffFromCaller) {
            HJD_HIP(hipEventSynchronize(g->staged));
            break;
        }
    return HJD_OK;
}

}  // namespace

extern "C" {

// Subsequence length when the caller passes 0.  Longer subsequences mean fewer
// guessed starts to repair but fewer workgroups.  Measured on 4K q90 4:2:0
// batches (profiles/r01_entropy_subbits.json, sync + write kernels):
// - 64 frames: S = 4096 is 5-8 % faster than 2048;
// - 32 frames: S = 4096 is 6 % slower;
// - 8 frames: S = 4096 is 34 % slower.
// Hence 4096 for decoders sized for >= 48 frames per call (the stream's
// 48-frame batches: profiles/r01_stream_batch_ab.json).  A decoder for one or
// two images is latency-bound by the serial chain of a subsequence: one FHD
// q90 JPEG, end to end, took 1.16 ms at S = 1024 against 1.35 ms at 2048
// (512: 1.04 ms, but its 4096-bit warm-up overlap fails to link often enough
// at 256 to fall back; profiles/r02_fhd_jpeg_subbits.json), so 1024 there.
// With the sync kernel's step tables: 1.05 ms at 1024, 0.96 at 512, 1.21 at 2048.
// HJD_SUB_BITS overrides it (tuning hook, tools/gpu_subbits_sweep.sh).
static int default_sub_bits(int max_frames)
{
    static const int env = [] {
        const char* e = getenv("HJD_SUB_BITS");
        return e ? atoi(e) : 0;
    }();
    if (env) return env;
    return max_frames >= 48 ? 2 * kDefaultSubBits : max_frames <= 2 ? kDefaultSubBits / 2 : kDefaultSubBits;
}

// The stream's decoders: batches of several slots overlap on the GPU, so the
// parallelism a single batch lacks at long subsequences comes from the other
// slots, and fewer guessed starts to repair wins.  Measured end to end on the
// config-5 stream (profiles/r02_stream_subbits.json): S = 8192 at 32-48
// frames per batch x 8 slots gives 97-101 Gpx/s against 91-94 at S = 4096;
// 16384 and 64-96-frame batches are slower.
// Speculative sync (ent_spec/cand/sync_spec kernels) for latency decoders:
// one or two frames per call, where the round-based sync's serial rounds are
// the critical path and most of the GPU is idle.  HJD_SYNC_SPEC=0/1 overrides.
static bool spec_sync_default(int max_frames)
{
    const char* e = getenv("HJD_SYNC_SPEC");
    if (e) return atoi(e) != 0;
    return max_frames <= 2;
}

static int stream_sub_bits(int max_frames)
{
    const char* e = getenv("HJD_SUB_BITS");
    if (e) return atoi(e);
    return max_frames >= 24 ? 4 * kDefaultSubBits : default_sub_bits(max_frames);
}

int hjd_gdec_create(hjd_ctx* ctx, int max_frames, int64_t max_scan_bytes, int64_t max_blocks, int sub_bits,
                    hjd_gdec** out)
{
    if (!ctx || !out || max_frames <= 0 || max_scan_bytes <= 0 || max_blocks <= 0)
        return set_error(HJD_E_INVALID, "invalid gdec arguments");
    const bool spec = spec_sync_default(max_frames);
    // the speculative sync's critical path is a few runs of S (+ the lead-in)
    // bits, no longer ~7 serial rounds: shorter subsequences pay there.  One
    // FHD q90 JPEG end to end (profiles/r03_fhd420_jpeg_spec_sweep.json):
    // 0.65 ms at S = 512 / lead-in 512, 0.71 at 1024, 0.69-0.76 at 768.
    if (sub_bits == 0) sub_bits = spec && !getenv("HJD_SUB_BITS") ? kDefaultSubBits / 4 : default_sub_bits(max_frames);
    if (sub_bits < 32 || sub_bits > (1 << 20)) return set_error(HJD_E_INVALID, "sub_bits out of range [32, 2^20]");
    *out = nullptr;
    hjd_gdec* g = new (std::nothrow) hjd_gdec;
    if (!g) return set_error(HJD_E_NOMEM, "gdec allocation");
    g->ctx = ctx;
    g->device = hjd_ctx_device(ctx);
    g->num_cu = hjd_internal::ctx_num_cu(ctx);
    g->caps = make_caps(max_frames, max_scan_bytes, max_blocks, sub_bits);
    g->spec = spec;
    const int rc = gdec_alloc(g);
    if (rc) {
        hjd_gdec_destroy(g);
        return rc;
    }
    *out = g;
    return HJD_OK;
}

int hjd_gdec_destroy(hjd_gdec* g)
{
    if (!g) return HJD_OK;
    if (g->host_calls && getenv("HJD_GDEC_HOST_TIMES"))
        fprintf(stderr, "hjd_gdec host us/call over %lld calls: wait_staging %.1f stage %.1f issue %.1f\n",
                static_cast<long long>(g->host_calls), g->host_us[0] / g->host_calls, g->host_us[1] / g->host_calls,
                g->host_us[2] / g->host_calls);
    if (!g->gpu) {
        free(g->h_stage);
        delete g;
        return HJD_OK;
    }
    (void)hipSetDevice(g->device);
    if (g->done) (void)hipEventSynchronize(g->done);
    if (g->h_stage) (void)hipHostFree(g->h_stage);
    if (g->h_status) (void)hipHostFree(g->h_status);
    void* dev[] = {g->d_blob, g->d_entries, g->d_stats, g->d_mids, g->d_stats1, g->d_wentries, g->d_linked, g->d_agg,
                   g->d_coefs, g->d_raw, g->d_tiles, g->d_spec, g->d_cand, g->d_cmap, g->d_cslot,
                   g->d_steps, g->d_chainfn, g->d_chain_broken, g->d_agg2};
    for (void* p : dev)
        if (p) (void)hipFree(p);
    if (g->staged) (void)hipEventDestroy(g->staged);
    if (g->done) (void)hipEventDestroy(g->done);
    delete g;
    return HJD_OK;
}

int hjd_gdec_decode(hjd_gdec* g, const uint8_t* const* datas, const size_t* sizes, int n, void* const* d_outs,
                    const int32_t* pitches, void* stream)
{
    if (!d_outs) return set_error(HJD_E_INVALID, "d_outs is NULL");
    return gdec_run(g, datas, sizes, n, d_outs, pitches, nullptr, nullptr, static_cast<hipStream_t>(stream));
}

int hjd_gdec_decode_coefs(hjd_gdec* g, const uint8_t* const* datas, const size_t* sizes, int n, int16_t* d_coefs,
                          int64_t* block_offsets, void* stream)
{
    if (!d_coefs || (reinterpret_cast<uintptr_t>(d_coefs) & 15))
        return set_error(HJD_E_INVALID, "d_coefs must be a 16-byte aligned device pointer");
    return gdec_run(g, datas, sizes, n, nullptr, nullptr, d_coefs, block_offsets, static_cast<hipStream_t>(stream));
}

int hjd_gdec_last_bytes(hjd_gdec* g, int64_t* host_scan_bytes, int64_t* h2d_bytes)
{
    if (!g) return set_error(HJD_E_INVALID, "gdec is NULL");
    if (host_scan_bytes) *host_scan_bytes = g->last_host_scan_bytes;
    if (h2d_bytes) *h2d_bytes = g->last_h2d;
    return HJD_OK;
}

int hjd_gdec_set_output_format(hjd_gdec* g, int out_format)
{
    if (!g) return set_error(HJD_E_INVALID, "gdec is NULL");
    if (!hjd_internal::out_format_bytes(out_format)) return set_error(HJD_E_INVALID, "unknown output format %d", out_format);
    g->out_format = out_format;   // applies to the next decode; an issued one keeps its format
    return HJD_OK;
}

int hjd_gdec_sync(hjd_gdec* g, int32_t* status)
{
    if (!g || !g->gpu) return set_error(HJD_E_INVALID, "gdec is NULL");
    if (!g->pending) return HJD_OK;
    HJD_HIP(hipSetDevice(g->device));
    HJD_HIP(hipEventSynchronize(g->done));
    for (size_t e = 0; e < g->scan_file.size(); ++e)   // a JPEG's further scans
        g->h_status[g->scan_file[e]] |= g->h_status[g->nframes_issued + e];
    int bad = 0;
    bool repaired = false;
    for (int i = 0; i < g->nframes_issued; ++i) {
        const uint32_t s = g->h_status[i] & ~kStatusFallback;
        if (status) status[i] = static_cast<int32_t>(g->h_status[i]);
        if (s) ++bad;
        repaired = repaired || (g->h_status[i] & kStatusFallback);
    }
    if (g->batch_spec) {   // the lead-in of the next batches (spec_lead_bits)
        if (repaired) {
            if (g->lead_stepped_down) g->lead_hold = std::min(2 * g->lead_hold, kLeadBatchesMax);
            g->lead_step = std::min(g->lead_step + 1, kLeadSteps - 1);
            g->lead_left = g->lead_hold;
            g->lead_stepped_down = false;
        } else {
            g->lead_stepped_down = false;
            if (g->lead_step && --g->lead_left == 0) {
                g->lead_left = --g->lead_step ? g->lead_hold : 0;
                g->lead_stepped_down = true;
            }
        }
    }
    g->pending = false;
    if (bad) return set_error(HJD_E_INVALID, "%d of %d frames had corrupt entropy data", bad, g->nframes_issued);
    return HJD_OK;
}

// Tuning hook: for every subsequence start k*S (k >= 1), decode from the guess
// (k*S, 0, 0) and report after how many bits past k*S its state first equals
// the true decode's state at the same unit boundary (hist[min(bits/64, nbins-1)];
// never-synced within max_bits go to the last bin).
int hjd_debug_entropy_syncstats(const uint8_t* data, size_t size, int sub_bits, int max_bits, int64_t* hist, int nbins)
{
    if (!data || !hist || nbins < 2 || sub_bits < 32) return set_error(HJD_E_INVALID, "invalid arguments");
    std::vector<uint8_t> buf(size + 64);
    Prepared p;
    int rc = prepare(data, size, buf.data(), size + 32, p);
    if (rc) return rc;
    EntFrame F;
    memset(&F, 0, sizeof(F));
    F.data_bits = p.data_bits;
    F.nseg = static_cast<uint32_t>(p.seg_end.size());
    F.bpm = static_cast<uint8_t>(p.bpm);
    memcpy(F.jinfo, p.jinfo, sizeof(F.jinfo));
    EntBatchDev b;
    memset(&b, 0, sizeof(b));
    b.data = buf.data();
    b.seg_end = p.seg_end.data();
    BlockInfo blocks[kMaxBpm];
    fill_blocks(blocks, F);
    const RunCtx c = make_ctx(b, F, p.tabs, blocks);
    // true states at every unit boundary: decode one unit at a time (stop = pos + 1)
    std::vector<uint16_t> truth(p.data_bits + 1, 0xFFFF);
    uint64_t cur = pack_state(0, 0, 0, 0);
    while (st_seg(cur) < F.nseg) {
        truth[st_pos(cur)] = static_cast<uint16_t>(st_j(cur) << 8 | st_z(cur));
        SubStats st = stats_identity();
        const uint64_t nx = run<false>(c, cur, st_pos(cur) + 1, st, nullptr);
        if (st_pos(nx) <= st_pos(cur) && st_seg(nx) == st_seg(cur)) break;
        cur = nx;
    }
    for (int i = 0; i < nbins; ++i) hist[i] = 0;
    const uint32_t S = static_cast<uint32_t>(sub_bits);
    // HJD_SYNC_PHASES=n: guesses (k*S, j, 0) for j < n; the first of them to
    // meet the true decode counts (speculation over block-in-MCU positions)
    const char* ph = getenv("HJD_SYNC_PHASES");
    const uint32_t nph = std::max(1, std::min(ph ? atoi(ph) : 1, static_cast<int>(F.bpm)));
    // HJD_SYNC_OFFSETS=m: also guesses m-1 bit positions before k*S (offsets
    // 7, 19, 37, 61, ... bits), each with the n phases
    const char* os = getenv("HJD_SYNC_OFFSETS");
    const uint32_t noff = std::max(1, os ? atoi(os) : 1);
    static const uint32_t kOffs[] = {0, 7, 19, 37, 61, 91, 127, 169, 217, 271, 331, 397};
    for (uint32_t k = 1; static_cast<uint64_t>(k) * S < p.data_bits; ++k) {
        int bin = nbins - 1;
        for (uint32_t oi = 0; oi < std::min<uint32_t>(noff, 12); ++oi) {
            if (kOffs[oi] > k * S) continue;
            for (uint32_t j0 = 0; j0 < nph; ++j0) {
                uint64_t g = guess_entry(c, k * S - kOffs[oi]);
                g = pack_state(st_pos(g), j0, 0, st_seg(g));
                while (st_pos(g) < static_cast<uint64_t>(k) * S + static_cast<uint32_t>(max_bits) && st_seg(g) < F.nseg) {
                    const uint32_t q = st_pos(g);
                    if (truth[q] == (st_j(g) << 8 | st_z(g))) {
                        bin = std::min<int>(bin, q > k * S ? static_cast<int>((q - k * S) / 64) : 0);
                        break;
                    }
                    SubStats st = stats_identity();
                    g = run<false>(c, g, q + 1, st, nullptr);
                }
            }
        }
        hist[bin]++;
    }
    return HJD_OK;
}

// Test hook for the sync-mode step decode: every run a sync kernel makes uses
// the AC step tables (several units per lookup) and must give exactly the
// state and statistics of the unit-by-unit decode.  Runs the first scan from
// guessed entries (k*S - o, j, 0) for every block-in-MCU j and a few offsets o,
// and from true unit boundaries, to stops S bits on, both ways; counts runs
// and mismatches (exit state, block count, flags or DC sums).
int hjd_debug_entropy_sync_check(const uint8_t* data, size_t size, int sub_bits, int64_t* runs, int64_t* mismatches)
{
    if (!data || !runs || !mismatches || sub_bits < 16) return set_error(HJD_E_INVALID, "invalid arguments");
    std::vector<uint8_t> buf(size + 256);
    Prepared p;
    int rc = prepare(data, size, buf.data(), size + 64, p);
    if (rc) return rc;
    EntFrame F;
    memset(&F, 0, sizeof(F));
    F.data_bits = p.data_bits;
    F.nseg = static_cast<uint32_t>(p.seg_end.size());
    F.bpm = static_cast<uint8_t>(p.bpm);
    F.ntab = static_cast<uint8_t>(p.ntab);
    memcpy(F.jinfo, p.jinfo, sizeof(F.jinfo));
    EntBatchDev b;
    memset(&b, 0, sizeof(b));
    b.data = buf.data();
    b.seg_end = p.seg_end.data();
    BlockInfo blocks[kMaxBpm];
    fill_blocks(blocks, F);
    std::vector<uint8_t> steps(static_cast<size_t>(F.ntab) << kStepBits);
    fill_steps(steps.data(), p.tabs, F.ntab, 0, 1);
    const RunCtx cs = make_ctx(b, F, p.tabs, blocks, steps.data());
    const RunCtx cu = make_ctx(b, F, p.tabs, blocks);
    const uint32_t S = static_cast<uint32_t>(sub_bits);
    int64_t n = 0, bad = 0;
    auto check = [&](uint64_t entry, uint32_t stop) {
        SubStats a = stats_identity(), u = stats_identity();
        const uint64_t xa = run<false>(cs, entry, stop, a, nullptr);
        const uint64_t xu = run<false>(cu, entry, stop, u, nullptr);
        ++n;
        if (xa != xu || a.nblk != u.nblk || a.flags != u.flags || a.dc[0] != u.dc[0] || a.dc[1] != u.dc[1] ||
            a.dc[2] != u.dc[2])
            ++bad;
    };
    static const uint32_t kOffs[] = {0, 5, 19, 61, 200};
    for (uint32_t k = 0; static_cast<uint64_t>(k) * S < p.data_bits; ++k)
        for (uint32_t o : kOffs) {
            if (o > k * S) continue;
            const uint64_t g = guess_entry(cu, k * S - o);
            for (uint32_t j = 0; j < F.bpm; ++j) check(pack_state(st_pos(g), j, 0, st_seg(g)), k * S + S);
        }
    // true unit boundaries, sampled
    uint64_t cur = pack_state(0, 0, 0, 0);
    for (uint32_t i = 0; st_seg(cur) < F.nseg; ++i) {
        if (i % 7 == 0) check(cur, st_pos(cur) + S / 2 + (i % 5) * 37);
        SubStats st = stats_identity();
        const uint64_t nx = run<false>(cu, cur, st_pos(cur) + 1, st, nullptr);
        if (st_pos(nx) <= st_pos(cur) && st_seg(nx) == st_seg(cur)) break;
        cur = nx;
    }
    *runs = n;
    *mismatches = bad;
    return HJD_OK;
}

// Test hooks for the destuff step alone: the host routine (destuff()) and the
// three device kernels on one raw scan, so arbitrary byte strings (stuffing,
// fill bytes, RSTn in and out of order, truncation) can be compared directly.
int hjd_debug_destuff_host(const uint8_t* scan, size_t n, uint8_t* out, size_t cap, uint32_t* seg_end, int max_seg,
                           int* nseg, int64_t* out_bytes)
{
    if (!scan || !out || !seg_end || !nseg || !out_bytes) return set_error(HJD_E_INVALID, "NULL argument");
    std::vector<uint32_t> seg;
    size_t len = 0;
    const int rc = destuff(scan, scan + n, out, cap, seg, len);
    if (rc) return rc;
    *nseg = static_cast<int>(seg.size());
    for (int i = 0; i < static_cast<int>(seg.size()) && i < max_seg; ++i) seg_end[i] = seg[i];
    *out_bytes = static_cast<int64_t>(len);
    return HJD_OK;
}

int hjd_debug_destuff_gpu(hjd_ctx* ctx, const uint8_t* scan, size_t n, int nseg, uint8_t* out, size_t cap,
                          uint32_t* seg_end, int64_t* out_bytes, uint32_t* status)
{
    if (!ctx || !scan || !out || !seg_end || !out_bytes || !status || n == 0 || nseg < 1 || cap < n + kDataPad)
        return set_error(HJD_E_INVALID, "invalid destuff arguments");
    HJD_HIP(hipSetDevice(hjd_ctx_device(ctx)));
    const uint32_t ntiles = static_cast<uint32_t>((n + kTileBytes - 1) / kTileBytes);
    const size_t area = align_up(n + kDataPad, 16);
    EntFrame F;
    memset(&F, 0, sizeof(F));
    F.nseg = static_cast<uint32_t>(nseg);
    F.data_bits = static_cast<uint32_t>(n * 8);
    RawFrame R{0, static_cast<uint32_t>(n), 0, 0, ntiles, 0, 0};
    std::vector<uint32_t> tf(ntiles, 0);
    uint8_t *d_raw = nullptr, *d_out = nullptr;
    EntFrame* d_f = nullptr;
    RawFrame* d_r = nullptr;
    uint32_t *d_tf = nullptr, *d_tiles = nullptr, *d_seg = nullptr, *d_status = nullptr;
    hipError_t e = hipSuccess;
    auto ok = [&](hipError_t x) { if (e == hipSuccess) e = x; return e == hipSuccess; };
    if (ok(hipMalloc(&d_raw, area)) && ok(hipMalloc(&d_out, area)) && ok(hipMalloc(&d_f, sizeof(F))) &&
        ok(hipMalloc(&d_r, sizeof(R))) && ok(hipMalloc(&d_tf, 4 * ntiles)) && ok(hipMalloc(&d_tiles, 12 * ntiles)) &&
        ok(hipMalloc(&d_seg, 4 * static_cast<size_t>(nseg))) && ok(hipMalloc(&d_status, 4)) &&
        ok(hipMemcpy(d_raw, scan, n, hipMemcpyHostToDevice)) && ok(hipMemcpy(d_f, &F, sizeof(F), hipMemcpyHostToDevice)) &&
        ok(hipMemcpy(d_r, &R, sizeof(R), hipMemcpyHostToDevice)) &&
        ok(hipMemcpy(d_tf, tf.data(), 4 * ntiles, hipMemcpyHostToDevice)) && ok(hipMemset(d_status, 0, 4)) &&
        ok(hipMemset(d_seg, 0xEE, 4 * static_cast<size_t>(nseg))) && ok(hipMemset(d_out, 0xEE, area))) {
        EntBatchDev b;
        memset(&b, 0, sizeof(b));
        b.frames = d_f;
        b.seg_end = d_seg;
        b.data = d_out;
        b.status = d_status;
        b.nframes = 1;
        b.sub_bits = 4096;
        b.raw = d_raw;
        b.rawf = d_r;
        b.tile_frame = d_tf;
        b.tiles = d_tiles;
        b.ntiles = ntiles;
        hipLaunchKernelGGL(destuff_count_kernel, dim3(ntiles), dim3(kTileThreads), 0, 0, b);
        hipLaunchKernelGGL(destuff_scan_kernel, dim3(1), dim3(kTileThreads), 0, 0, b);
        hipLaunchKernelGGL(destuff_write_kernel, dim3(ntiles), dim3(kTileThreads), 0, 0, b);
        EntFrame Fo;
        if (ok(hipGetLastError()) && ok(hipDeviceSynchronize()) &&
            ok(hipMemcpy(&Fo, d_f, sizeof(Fo), hipMemcpyDeviceToHost)) &&
            ok(hipMemcpy(out, d_out, area, hipMemcpyDeviceToHost)) &&
            ok(hipMemcpy(seg_end, d_seg, 4 * static_cast<size_t>(nseg), hipMemcpyDeviceToHost)) &&
            ok(hipMemcpy(status, d_status, 4, hipMemcpyDeviceToHost)))
            *out_bytes = Fo.data_bits / 8;
    }
    for (void* p : {static_cast<void*>(d_raw), static_cast<void*>(d_out), static_cast<void*>(d_f),
                    static_cast<void*>(d_r), static_cast<void*>(d_tf), static_cast<void*>(d_tiles),
                    static_cast<void*>(d_seg), static_cast<void*>(d_status)})
        if (p) (void)hipFree(p);
    if (e != hipSuccess) return set_error(HJD_E_HIP, "destuff test hook: %s", hipGetErrorString(e));
    return HJD_OK;
}

int hjd_debug_entropy_emulate(const uint8_t* data, size_t size, int sub_bits, int16_t* coefs,
                              int64_t capacity_blocks, int32_t* status)
{
    if (!data || !coefs) return set_error(HJD_E_INVALID, "NULL argument");
    if (sub_bits == 0) sub_bits = kDefaultSubBits;
    if (sub_bits < 32 || sub_bits > (1 << 20)) return set_error(HJD_E_INVALID, "sub_bits out of range [32, 2^20]");
    hjd_gdec g;
    g.gpu = false;
    g.caps = make_caps(1, static_cast<int64_t>(size), std::max<int64_t>(capacity_blocks, 1), sub_bits);
    const char* se = getenv("HJD_SYNC_SPEC");   // the emulation takes the round-based sync unless asked
    g.spec = se && atoi(se) != 0;
    int rc = gdec_alloc(&g);
    if (rc) return rc;
    struct Free {
        hjd_gdec* g;
        ~Free() { free(g->h_stage); g->h_stage = nullptr; }
    } guard{&g};
    const uint8_t* datas[1] = {data};
    const size_t sizes[1] = {size};
    rc = g.stage_frames(datas, sizes, 1);
    if (rc) return rc;
    if (g.frames[0].out_blocks > capacity_blocks)
        return set_error(HJD_E_INVALID, "capacity %lld < %lld blocks", static_cast<long long>(capacity_blocks),
                         static_cast<long long>(g.frames[0].out_blocks));
    EntBatchDev b;
    rc = g.assemble(g.h_stage, coefs, nullptr, nullptr, nullptr, b);
    if (rc) return rc;
    const int64_t total = g.frames[0].out_blocks;
    g.e_entries.assign(static_cast<size_t>(g.caps.max_subs), 0);
    g.e_stats.assign(static_cast<size_t>(g.caps.max_subs), stats_identity());
    g.e_mids.assign(static_cast<size_t>(g.caps.max_subs), 0);
    g.e_stats1.assign(static_cast<size_t>(g.caps.max_subs), stats_identity());
    g.e_wentries.assign(static_cast<size_t>(g.caps.max_wgs) * kWarm, 0);
    g.e_linked.assign(static_cast<size_t>(g.caps.max_wgs), 0);
    g.e_agg.assign(static_cast<size_t>(g.caps.max_wgs), stats_identity());
    g.e_status.assign(b.nframes, 0);
    if (g.spec) {
        const size_t n = static_cast<size_t>(g.caps.max_subs);
        g.e_spec.assign(n * kMaxBpm, SpecRec());
        g.e_cand.assign(n * kCandRow, CandRec());
        g.e_cmap.assign(n * kSlotRow, static_cast<uint8_t>(kNoCand));
        b.spec = g.e_spec.data();
        b.cand = g.e_cand.data();
        b.cmap = g.e_cmap.data();
        g.e_cslot.assign(n + 16, 0);
        b.cslot = g.e_cslot.data();
        b.spec_lead = spec_lead_bits(0);
    }
    b.entries = g.e_entries.data();
    b.stats = g.e_stats.data();
    b.mids = g.e_mids.data();
    b.stats1 = g.e_stats1.data();
    b.wentries = g.e_wentries.data();
    b.linked = g.e_linked.data();
    b.agg = g.e_agg.data();
    b.status = g.e_status.data();
    memset(coefs, 0, static_cast<size_t>(total) * 128);
    emulate(b);
    for (uint32_t e = 1; e < b.nframes; ++e) g.e_status[0] |= g.e_status[e];   // the JPEG's further scans
    if (status) *status = static_cast<int32_t>(g.e_status[0]);
    if (g.e_status[0] & ~kStatusFallback) return set_error(HJD_E_INVALID, "corrupt entropy data (status %u)", g.e_status[0]);
    return HJD_OK;
}

}  // extern "C"

// ---------------------------------------------------------------------------
// GPU-entropy stream: submit JPEGs one by one; worker threads parse and
// destuff them into the pinned staging of the open batch (nslots batches
// rotate, each on its own HIP stream, so one batch's upload overlaps another's
// kernels); the thread that completes a closed batch issues it.
// ---------------------------------------------------------------------------
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <thread>

namespace {

struct GBatch {
    int slot = 0;
    int nframes = 0;
    size_t bytes = 0;
    int64_t blocks = 0;
    int prepared = 0;
    bool closed = false;
    bool issued = false;
    std::vector<void*> outs;         // device destination, or null for a host-output frame
    std::vector<int32_t> pitches;
    std::vector<void*> host_outs;    // host destination (D2H sink), or null
    RawCursor raw;                   // raw-area placement of device-destuffed scans
};

struct GJob {
    GBatch* batch;
    int index;
    const uint8_t* data;
    size_t size;
    size_t data_off;
    size_t cap;
    int mode;                        // kDestuff*
    uint64_t raw_off;
};

}  // namespace

struct hjd_gstream {
    hjd_ctx* ctx = nullptr;
    int device = 0;
    std::vector<hjd_gdec*> slots;
    std::vector<hipStream_t> streams;
    std::vector<uint8_t*> scratch;       // per slot: device pixels of host-output frames (D2H sink)
    std::vector<size_t> scratch_bytes;
    std::vector<GBatch*> slot_batch;   // batch currently owning each slot (nullptr = free)
    int next_slot = 0;
    GBatch* open = nullptr;

    std::mutex mu;
    std::mutex api_mu;          // serialises submit/sync callers (batch opening drops `mu` while it waits)
    std::condition_variable cv_jobs, cv_state;
    std::deque<GJob> queue;
    bool stop = false;
    std::vector<std::thread> workers;
    int64_t batches_in_flight = 0;     // created and not yet issued

    std::atomic<int64_t> images{0}, pixels{0}, prep_ns{0}, h2d_bytes{0}, batches{0}, host_scan_bytes{0};
    int first_error = HJD_OK;
    std::string first_error_msg;
    int local_cpus = 0;   // CPUs of the GPU's NUMA node the workers are bound to (0: unbound)
    int out_format = HJD_OUT_BGRX;

    void record_error(int rc, const std::string& msg)
    {
        if (first_error == HJD_OK) {
            first_error = rc;
            first_error_msg = msg;
        }
    }
    int open_batch(std::unique_lock<std::mutex>& lk);
    void issue_locked(GBatch* b);
    void worker();
};

// Caller holds mu.  Waits for the next slot's previous batch to be issued and
// its uploads to finish before reusing the slot's pinned staging.
int hjd_gstream::open_batch(std::unique_lock<std::mutex>& lk)
{
    const int s = next_slot;
    next_slot = (next_slot + 1) % static_cast<int>(slots.size());
    cv_state.wait(lk, [&] { return !slot_batch[s] || slot_batch[s]->issued; });
    if (slot_batch[s]) {
        delete slot_batch[s];
        slot_batch[s] = nullptr;
        hjd_gdec* g = slots[s];
        if (g->pending) {
            lk.unlock();
            const hipError_t e = hipEventSynchronize(g->staged_by_done ? g->done : g->staged);
            lk.lock();
            if (e != hipSuccess) return set_error(HJD_E_HIP, "hipEventSynchronize: %s", hipGetErrorString(e));
        }
        // statuses of the slot's previous batch
        if (g->pending) {
            lk.unlock();
            const int rc = hjd_gdec_sync(g, nullptr);
            const std::string msg = rc ? hjd_last_error() : "";
            lk.lock();
            if (rc) record_error(rc, msg);
        }
    }
    GBatch* b = new GBatch;
    b->slot = s;
    slot_batch[s] = b;
    open = b;
    ++batches_in_flight;
    return HJD_OK;
}

// Caller holds mu; b is closed and fully prepared.
void hjd_gstream::issue_locked(GBatch* b)
{
    if (b->issued) return;
    hjd_gdec* g = slots[b->slot];
    // drop frames whose preparation failed (already recorded)
    std::vector<void*> outs;
    std::vector<int32_t> pitches;
    std::vector<HostCopy> host;
    std::vector<Prepared> keep;
    size_t used = 0, scratch_need = 0;
    for (int i = 0; i < b->nframes; ++i) {
        Prepared& p = g->frames[i];
        if (p.rc != HJD_OK) continue;
        used = std::max(used, align_up(p.data_end(), 16));
        images++;
        pixels += static_cast<int64_t>(p.width) * p.height;
        if (b->host_outs[i]) {
            host.push_back(HostCopy{b->host_outs[i], b->pitches[i], p.width, p.height});
            outs.push_back(reinterpret_cast<void*>(scratch_need));   // offset, rebased below
            pitches.push_back(align_up(static_cast<size_t>(hjd_internal::out_format_bytes(out_format)) * p.width, 16));
            scratch_need += align_up(static_cast<size_t>(pitches.back()) * p.height, 256);
        } else {
            host.push_back(HostCopy{nullptr, 0, p.width, p.height});
            outs.push_back(b->outs[i]);
            pitches.push_back(b->pitches[i]);
        }
        keep.push_back(std::move(p));
    }
    g->frames.swap(keep);
    g->data_used = used;
    int rc = HJD_OK;
    if (scratch_need > scratch_bytes[b->slot]) {   // grows rarely; the slot's previous batch is complete
        if (scratch[b->slot]) (void)hipFree(scratch[b->slot]);
        scratch[b->slot] = nullptr;
        scratch_bytes[b->slot] = 0;
        if (hipMalloc(reinterpret_cast<void**>(&scratch[b->slot]), scratch_need) != hipSuccess)
            rc = set_error(HJD_E_NOMEM, "device scratch for host outputs (%zu bytes)", scratch_need);
        else
            scratch_bytes[b->slot] = scratch_need;
    }
    for (size_t i = 0; i < outs.size(); ++i)
        if (host[i].host) outs[i] = scratch[b->slot] + reinterpret_cast<size_t>(outs[i]);
    if (rc) record_error(rc, hjd_last_error());
    if (!g->frames.empty() && rc == HJD_OK) {
        rc = gdec_issue(g, outs.data(), pitches.data(), nullptr, nullptr, streams[b->slot], host.data());
        if (rc) record_error(rc, hjd_last_error());
        h2d_bytes += g->last_h2d;
        host_scan_bytes += g->last_host_scan_bytes;
        batches++;
    }
    b->issued = true;
    --batches_in_flight;
    cv_state.notify_all();
}

void hjd_gstream::worker()
{
    (void)hipSetDevice(device);
    for (;;) {
        GJob job;
        {
            std::unique_lock<std::mutex> lk(mu);
            cv_jobs.wait(lk, [&] { return stop || !queue.empty(); });
            if (queue.empty()) return;
            job = queue.front();
            queue.pop_front();
        }
        hjd_gdec* g = slots[job.batch->slot];
        const auto t0 = std::chrono::steady_clock::now();
        const int rc = g->prepare_frame(job.index, job.data, job.size, job.data_off, job.cap, job.mode, job.raw_off);
        prep_ns += std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
        const std::string msg = rc ? hjd_last_error() : "";
        std::unique_lock<std::mutex> lk(mu);
        if (rc) record_error(rc, msg);
        GBatch* b = job.batch;
        ++b->prepared;
        if (b->closed && b->prepared == b->nframes) issue_locked(b);
        cv_state.notify_all();
    }
}

extern "C" {

int hjd_gstream_create(hjd_ctx* ctx, int max_frames, int64_t max_scan_bytes, int64_t max_blocks, int nslots,
                       int nthreads, hjd_gstream** out)
{
    if (!ctx || !out || nslots < 2 || nslots > 16) return set_error(HJD_E_INVALID, "invalid gstream arguments (nslots 2..16)");
    *out = nullptr;
    if (nthreads <= 0) nthreads = hjd_internal::default_worker_threads(hjd_ctx_device(ctx));
    hjd_gstream* st = new (std::nothrow) hjd_gstream;
    if (!st) return set_error(HJD_E_NOMEM, "gstream allocation");
    st->ctx = ctx;
    st->device = hjd_ctx_device(ctx);
    st->slots.assign(nslots, nullptr);
    st->streams.assign(nslots, nullptr);
    st->scratch.assign(nslots, nullptr);
    st->scratch_bytes.assign(nslots, 0);
    st->slot_batch.assign(nslots, nullptr);
    // NUMA locality: pinned staging is allocated, and the
    // workers run, on the CPUs of the GPU's NUMA node (HJD_NUMA=0 disables).
    const char* numa_env = getenv("HJD_NUMA");
    const hjd_internal::CpuSet local = (numa_env && numa_env[0] == '0') ? hjd_internal::CpuSet{}
                                                                       : hjd_internal::device_local_cpus(st->device);
    const std::vector<int> prev = hjd_internal::bind_current_thread(local);
    for (int s = 0; s < nslots; ++s) {
        int rc = hjd_gdec_create(ctx, max_frames, max_scan_bytes, max_blocks, stream_sub_bits(max_frames),
                                 &st->slots[s]);
        if (rc == HJD_OK && hipStreamCreateWithFlags(&st->streams[s], hipStreamNonBlocking) != hipSuccess)
            rc = set_error(HJD_E_HIP, "hipStreamCreate");
        if (rc) {
            hjd_internal::restore_current_thread(prev);
            hjd_gstream_destroy(st);
            return rc;
        }
    }
    hjd_internal::restore_current_thread(prev);
    st->local_cpus = static_cast<int>(local.cpus.size());
    for (int t = 0; t < nthreads; ++t)
        st->workers.emplace_back([st, local] {
            hjd_internal::bind_current_thread(local);
            st->worker();
        });
    *out = st;
    return HJD_OK;
}

static int gstream_submit(hjd_gstream* st, const uint8_t* data, size_t size, void* d_out, void* h_out,
                          int32_t out_pitch)
{
    hjd_internal::ScanHeader h;
    int rc = hjd_internal::parse_scan_header(data, size, &h);
    if (rc) return rc;
    if (out_pitch < hjd_internal::out_format_bytes(st->out_format) * h.width)
        return set_error(HJD_E_INVALID, "output pitch too small");
    const size_t need = h.extra_scans > 0 ? data_need(size) : align_up(size + kDataPad, 16);
    std::lock_guard<std::mutex> api(st->api_mu);
    std::unique_lock<std::mutex> lk(st->mu);
    hjd_gdec* g0 = st->slots[0];
    if (need > g0->data_cap() || h.nblocks > g0->caps.max_blocks)
        return set_error(HJD_E_INVALID, "JPEG larger than one batch's capacity");
    int mode = kDestuffHost;
    uint64_t raw_off = 0;
    bool fits = true;
    if (st->open) {
        GBatch* b = st->open;
        hjd_gdec* g = st->slots[b->slot];
        RawCursor cur = b->raw;
        rc = g->plan_raw(data, size, cur, mode, raw_off, fits, g->data_cap(), 0, false);
        if (rc) return rc;
        if (!fits || b->nframes == g->caps.max_frames || b->bytes + need > g->data_cap() ||
            b->blocks + h.nblocks > g->caps.max_blocks) {
            b->closed = true;
            st->open = nullptr;
            if (b->prepared == b->nframes) st->issue_locked(b);
        } else {
            b->raw = cur;
        }
    }
    if (!st->open) {
        rc = st->open_batch(lk);
        if (rc) return rc;
        GBatch* b = st->open;
        rc = st->slots[b->slot]->plan_raw(data, size, b->raw, mode, raw_off, fits, g0->data_cap(), 0, false);
        if (rc) return rc;
        if (!fits) return set_error(HJD_E_INVALID, "JPEG larger than one batch's capacity");
    }
    GBatch* b = st->open;
    hjd_gdec* g = st->slots[b->slot];
    if (b->nframes == 0) g->frames.assign(static_cast<size_t>(g->caps.max_frames), Prepared());
    GJob job{b, b->nframes, data, size, b->bytes, need, mode, raw_off};
    b->outs.push_back(d_out);
    b->host_outs.push_back(h_out);
    b->pitches.push_back(out_pitch);
    b->nframes++;
    b->bytes += need;
    b->blocks += h.nblocks;
    st->queue.push_back(job);
    lk.unlock();
    st->cv_jobs.notify_one();
    return HJD_OK;
}

int hjd_gstream_submit(hjd_gstream* st, const uint8_t* data, size_t size, void* d_out, int32_t out_pitch)
{
    const uintptr_t amask = st && st->out_format == HJD_OUT_BGR24 ? 3 : 15;
    if (!st || !data || !d_out || out_pitch <= 0 || (out_pitch & 3) || (reinterpret_cast<uintptr_t>(d_out) & amask))
        return set_error(HJD_E_INVALID, "invalid submit arguments (d_out must be 16-byte (BGR24: 4-byte) aligned)");
    return gstream_submit(st, data, size, d_out, nullptr, out_pitch);
}

int hjd_gstream_submit_host(hjd_gstream* st, const uint8_t* data, size_t size, void* h_out, int32_t out_pitch)
{
    if (!st || !data || !h_out || out_pitch <= 0) return set_error(HJD_E_INVALID, "invalid submit arguments");
    return gstream_submit(st, data, size, nullptr, h_out, out_pitch);
}

int hjd_gstream_set_output_format(hjd_gstream* st, int out_format)
{
    if (!st) return set_error(HJD_E_INVALID, "gstream is NULL");
    if (!hjd_internal::out_format_bytes(out_format)) return set_error(HJD_E_INVALID, "unknown output format %d", out_format);
    std::lock_guard<std::mutex> api(st->api_mu);
    std::lock_guard<std::mutex> lk(st->mu);
    if (st->open || st->batches_in_flight)
        return set_error(HJD_E_STATE, "output format can only change between hjd_gstream_sync and the next submit");
    st->out_format = out_format;
    for (hjd_gdec* g : st->slots) g->out_format = out_format;
    return HJD_OK;
}

static void bmp_header_bpp(int32_t width, int32_t height, int bpp, uint8_t header[54])
{
    // src/decoder.cpp:372-394 (bmp_create): BITMAPFILEHEADER + BITMAPINFOHEADER,
    // BI_RGB, negative height = top-down rows; rows padded to 4 bytes.
    auto put16 = [&](int o, uint32_t v) { header[o] = v & 0xFF; header[o + 1] = (v >> 8) & 0xFF; };
    auto put32 = [&](int o, uint32_t v) { put16(o, v & 0xFFFF); put16(o + 2, v >> 16); };
    memset(header, 0, 54);
    const uint64_t row = (static_cast<uint64_t>(width) * (bpp / 8) + 3) & ~uint64_t(3);
    const uint64_t size = 54 + row * static_cast<uint64_t>(height);
    put16(0, 0x4d42);
    put32(2, static_cast<uint32_t>(size));
    put32(10, 54);
    put32(14, 40);
    put32(18, static_cast<uint32_t>(width));
    put32(22, static_cast<uint32_t>(-height));
    put16(26, 1);
    put16(28, static_cast<uint32_t>(bpp));
}

int hjd_bmp_header(int32_t width, int32_t height, uint8_t header[54])
{
    if (!header || width <= 0 || height <= 0) return set_error(HJD_E_INVALID, "invalid BMP geometry");
    bmp_header_bpp(width, height, 32, header);   // the reference's 32-bpp BGRX file
    return HJD_OK;
}

int hjd_bmp_header_bgr24(int32_t width, int32_t height, uint8_t header[54])
{
    if (!header || width <= 0 || height <= 0) return set_error(HJD_E_INVALID, "invalid BMP geometry");
    bmp_header_bpp(width, height, 24, header);
    return HJD_OK;
}

int hjd_gstream_sync(hjd_gstream* st, int64_t stats[5])
{
    if (!st) return set_error(HJD_E_INVALID, "gstream is NULL");
    std::lock_guard<std::mutex> api(st->api_mu);
    {
        std::unique_lock<std::mutex> lk(st->mu);
        if (st->open) {
            GBatch* b = st->open;
            b->closed = true;
            st->open = nullptr;
            if (b->prepared == b->nframes) st->issue_locked(b);
        }
        st->cv_state.wait(lk, [&] { return st->batches_in_flight == 0; });
    }
    for (size_t s = 0; s < st->slots.size(); ++s) {
        hjd_gdec* g = st->slots[s];
        if (!g->pending) continue;
        const int rc = hjd_gdec_sync(g, nullptr);
        if (rc) {
            std::lock_guard<std::mutex> lk(st->mu);
            st->record_error(rc, hjd_last_error());
        }
    }
    if (stats) {
        stats[0] = st->images;
        stats[1] = st->pixels;
        stats[2] = st->prep_ns;
        stats[3] = st->h2d_bytes;
        stats[4] = st->batches;
    }
    std::lock_guard<std::mutex> lk(st->mu);
    if (st->first_error != HJD_OK) {
        const int rc = st->first_error;
        st->first_error = HJD_OK;
        return set_error(rc, "%s", st->first_error_msg.c_str());
    }
    return HJD_OK;
}

// Host-side stream preparation alone, no GPU (bench.py --host-prep-only: the
// host ceiling of the multi-GPU config-5 stream).  One call =
// one per-GPU worker pool: nthreads threads bound to NUMA node `node` (-1:
// unbound) prepare `frames` JPEGs.  The sources are an arena of `arena_bytes`
// (the pool's files replicated back to back, first-touched on that node, read
// in order) and each frame lands in the next slot of a staging ring of
// `ring_bytes`: with both larger than the node's L3 the traffic is DRAM's, as
// for a loader streaming fresh files.
//   mode 0: the host-destuff path (header, tables, destuff into staging);
//   mode 1: the GPU-destuff path (header and tables only);
//   mode 2: a plain memcpy of each file into staging (the DRAM reference).
// out[0] wall ns, out[1] summed thread CPU ns, out[2] JPEG bytes, out[3] frames.
int hjd_debug_host_prep(const uint8_t* const* datas, const size_t* sizes, int n, int mode, int nthreads, int node,
                        int64_t frames, int64_t arena_bytes, int64_t ring_bytes, int32_t* barrier, int parties,
                        int64_t out[4])
{
    if (!datas || !sizes || n <= 0 || nthreads <= 0 || frames <= 0 || !out || mode < 0 || mode > 2)
        return set_error(HJD_E_INVALID, "invalid host-prep arguments");
    const hjd_internal::CpuSet cpus = hjd_internal::node_cpus(node);
    size_t maxsz = 0, total = 0;
    for (int i = 0; i < n; ++i) {
        maxsz = std::max(maxsz, sizes[i]);
        total += sizes[i];
    }
    const size_t reps = std::max<size_t>(1, static_cast<size_t>(arena_bytes) / std::max<size_t>(total, 1));
    const size_t slot = align_up(maxsz + 4 * kDataPad, 4096);
    const size_t nslot = std::max<size_t>(static_cast<size_t>(nthreads),
                                          static_cast<size_t>(ring_bytes) / slot);
    std::vector<const uint8_t*> src;
    std::vector<size_t> src_size;
    uint8_t* arena = nullptr;
    uint8_t* ring = nullptr;
    {   // arena and ring first-touched by a thread on the pool's node
        std::thread t([&] {
            hjd_internal::bind_current_thread(cpus);
            arena = static_cast<uint8_t*>(malloc(total * reps));
            ring = static_cast<uint8_t*>(malloc(slot * nslot));
            if (!arena || !ring) return;
            size_t pos = 0;
            for (size_t r = 0; r < reps; ++r)
                for (int i = 0; i < n; ++i) {
                    memcpy(arena + pos, datas[i], sizes[i]);
                    src.push_back(arena + pos);
                    src_size.push_back(sizes[i]);
                    pos += sizes[i];
                }
            memset(ring, 0, slot * nslot);
        });
        t.join();
    }
    if (!arena || !ring) {
        free(arena);
        free(ring);
        return set_error(HJD_E_NOMEM, "host-prep arena");
    }
    if (barrier && parties > 1) {   // concurrent pools start their timed phase together
        __atomic_add_fetch(barrier, 1, __ATOMIC_SEQ_CST);
        while (__atomic_load_n(barrier, __ATOMIC_SEQ_CST) < parties) std::this_thread::yield();
    }
    std::atomic<int64_t> next{0}, cpu_ns{0}, bytes{0};
    std::atomic<int> err{HJD_OK};
    auto worker = [&] {
        hjd_internal::bind_current_thread(cpus);
        timespec c0, c1;
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c0);
        int64_t my_bytes = 0;
        Prepared pf;
        for (;;) {
            const int64_t k = next.fetch_add(1);
            if (k >= frames) break;
            const size_t i = static_cast<size_t>(k) % src.size();
            uint8_t* dst = ring + slot * (static_cast<size_t>(k) % nslot);
            int rc = HJD_OK;
            if (mode == 2) memcpy(dst, src[i], src_size[i]);
            else rc = prepare(src[i], src_size[i], dst, slot - kDataPad, pf,
                              mode == 0 ? kDestuffHost : kDestuffFromCaller, 0);
            if (rc) err = rc;
            my_bytes += static_cast<int64_t>(src_size[i]);
        }
        clock_gettime(CLOCK_THREAD_CPUTIME_ID, &c1);
        cpu_ns += (c1.tv_sec - c0.tv_sec) * 1000000000ll + (c1.tv_nsec - c0.tv_nsec);
        bytes += my_bytes;
    };
    const auto t0 = std::chrono::steady_clock::now();
    std::vector<std::thread> th;
    for (int t = 0; t < nthreads; ++t) th.emplace_back(worker);
    for (auto& t : th) t.join();
    out[0] = std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count();
    out[1] = cpu_ns;
    out[2] = bytes;
    out[3] = frames;
    free(arena);
    free(ring);
    return err == HJD_OK ? HJD_OK : set_error(err, "host prep failed: %s", hjd_last_error());
}

int hjd_gstream_host_bytes(hjd_gstream* st, int64_t* host_scan_bytes)
{
    if (!st || !host_scan_bytes) return set_error(HJD_E_INVALID, "NULL argument");
    *host_scan_bytes = st->host_scan_bytes;
    return HJD_OK;
}

int hjd_host_register(void* ptr, size_t size)
{
    if (!ptr || !size) return set_error(HJD_E_INVALID, "NULL or empty host range");
    HJD_HIP(hipHostRegister(ptr, size, hipHostRegisterDefault));
    return HJD_OK;
}

int hjd_host_unregister(void* ptr)
{
    if (!ptr) return set_error(HJD_E_INVALID, "NULL host pointer");
    HJD_HIP(hipHostUnregister(ptr));
    return HJD_OK;
}

int hjd_gstream_destroy(hjd_gstream* st)
{
    if (!st) return HJD_OK;
    (void)hjd_gstream_sync(st, nullptr);
    {
        std::lock_guard<std::mutex> lk(st->mu);
        st->stop = true;
    }
    st->cv_jobs.notify_all();
    for (auto& t : st->workers) t.join();
    for (size_t s = 0; s < st->slots.size(); ++s) {
        delete st->slot_batch[s];
        if (st->slots[s]) hjd_gdec_destroy(st->slots[s]);
        if (st->streams[s]) (void)hipStreamDestroy(st->streams[s]);
        if (st->scratch[s]) (void)hipFree(st->scratch[s]);
    }
    delete st;
    return HJD_OK;
}

}  // extern "C"
