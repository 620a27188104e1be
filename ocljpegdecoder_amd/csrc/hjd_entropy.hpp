// hjd_entropy.hpp -- GPU entropy (Huffman) decoding of baseline JPEG scans:
// the state machine shared by the gfx950 kernels (hjd_entropy.hip) and the
// host emulation used by the CPU tests.
//
// What it replaces: the reference decodes the whole scan on one host thread
// (src/decoder.cpp:221-365: DC/AC symbol loop :221-260, restart handling
// :288-307, MCU/block order :308-344; bit reader src/bitstream.h:310-365;
// Huffman lookup src/huffman.h:277-314).  SURVEY.md s8(f) rank 3.
//
// Parallel formulation (self-synchronising decode, our design):
//   * the host strips byte stuffing and RST markers while copying the scan
//     into pinned memory; the device sees one contiguous bit string per frame
//     plus the bit offset where each restart interval ("segment") ends;
//   * the bit string is cut into fixed "subsequences" of S bits; the decoder
//     state at a unit boundary (before a DC or AC Huffman symbol) is
//     (pos, j = block of the MCU, z = next coefficient index);
//   * the ENTRY of subsequence k is the first unit boundary at pos >= k*S; a
//     RUN decodes from an entry until the first unit boundary >= (k+1)*S and
//     returns that state (the EXIT), which is the next subsequence's entry;
//   * runs started from a guessed entry (k*S, 0, 0) usually fall into step
//     with the true decode within a few hundred bits (JPEG Huffman codes
//     self-synchronise); the kernels then verify the chain entry(k+1) ==
//     run(entry(k)) from the known frame start, re-running only where it
//     breaks, so the result never depends on the guess being right;
//   * segment ends are found without counting MCUs: at a unit boundary with
//     fewer than 8 bits left in the segment and all of them 1 (the T.81
//     F.1.2.3 pad), the segment is over -- no Huffman code is all ones, so
//     valid data can never look like that earlier.
#pragma once
#include <stdint.h>

#ifndef __HIPCC__
#define __host__
#define __device__
#define __forceinline__ inline
#endif

namespace hjd {
namespace ent {

constexpr int kLutBits = 10;                    // first-level lookup width
// sync-mode AC step table width (>= kLutBits, <= 15); same-box: 11 bits best on the
// stream, 12 on a lone batch (profiles/r02_entropy_step_bits_ab.json)
constexpr int kStepBits = 11;
constexpr int kMaxTables = 6;                   // DC+AC per component at most
constexpr int kGroupSubs = 256;                 // subsequences per workgroup (one per thread)
constexpr int kWarm = 8;                        // leading subsequences a group shares with its predecessor
constexpr int kOwn = kGroupSubs - kWarm;        // subsequences a group is responsible for
constexpr int kDefaultSubBits = 2048;           // S
// int16 per lane in the staging buffer: one 16-coefficient quarter + 8 B pad.
// 40 B (8-B aligned, accessed as 8-B pieces) keeps the write kernel's LDS
// (256 slots + the tables) under 20 KiB, i.e. 8 groups per CU.
constexpr int kStageStride = 20;

// A decoded unit (one Huffman symbol + its extra bits) in table form, 16 bits:
//   [4:0]  total: code length + extra bits s (the bits the unit consumes, >= 1)
//   [8:5]  s (extra bits = magnitude category)
//   [15:9] zk: how far the unit moves z, the next coefficient index --
//          DC 1 (127: a DC symbol > 11, an error), AC value r + 1 (the run
//          plus the coefficient), ZRL (r = 15, s = 0) 16, EOB (s = 0, r != 15)
//          64, which ends the block from any z.
// Precomputing these per code makes the device's symbol step branch-free on
// its common path (no DC/AC/EOB/ZRL cases).
__host__ __device__ __forceinline__ uint32_t unit_entry(uint32_t len, uint32_t sym, bool dc)
{
    const uint32_t s = sym & 15, r = sym >> 4;
    const uint32_t zk = dc ? (sym > 11 ? 127u : 1u) : (s ? r + 1 : (r == 15 ? 16u : 64u));
    return (len + s) | (s << 5) | (zk << 9);
}
constexpr uint32_t kZkDcError = 127;

// One Huffman table in device form (2448 B, 16-B multiple).
struct HuffLut {
    uint16_t lut[1 << kLutBits];   // unit_entry() for codes <= kLutBits bits, 0: longer code
    int32_t maxcode[17];           // largest code of each length, -1 if none (T.81 F.2.2.3)
    int32_t delta[17];             // valptr[len] - mincode[len]
    uint8_t vals[256];
    uint8_t pad[8];
};
static_assert(sizeof(HuffLut) == 2448, "HuffLut layout");

// Per-frame record of an entropy batch (device, 80 B).
struct EntFrame {
    uint64_t data_off;    // byte offset of the destuffed bit string in the batch data area (16-B aligned)
    uint64_t coef_off;    // first output block in the coefficient buffer
    uint32_t data_bits;   // destuffed length in bits (= end of the last segment)
    uint32_t nsub;        // subsequences of this frame
    uint32_t sub_base;    // first global subsequence index
    uint32_t wg_base;     // first global workgroup index (kGroupSubs subsequences each)
    uint32_t seg_base;    // first entry in the segment-end table
    uint32_t nseg;        // restart intervals (1 without DRI)
    uint32_t nblocks;     // blocks the scan must produce
    uint32_t tab_base;    // first HuffLut of this frame
    uint8_t ntab, bpm, sampling;
    uint8_t layout;       // kLayoutMcu / kLayoutRaster (where the scan's blocks go, see block_dest)
    uint16_t jinfo[6];    // per bitstream block j of an MCU: dc slot | ac slot << 3 | comp << 6 | out slot << 8
    uint32_t seg_blocks;  // blocks of a full restart interval (DRI MCUs x bpm); 0 without restarts
    uint32_t geo;         // out_bpm | comp_lh << 4 | comp_lv << 6 | comp_bw << 8 (geo_make)
    uint32_t mcu_w;       // MCUs per row of the image
    uint32_t nout;        // blocks of the image (= nblocks for a single scan)
};
static_assert(sizeof(EntFrame) == 80, "EntFrame layout");

// Scan layouts.  A "frame" of the entropy kernels is one scan: the reference's
// single interleaved scan, or one scan of a sequential file with several
// (an extension; its scans write into the same coefficient frame).
//   kLayoutMcu:    the scan's MCUs are the image's, holding bpm <= out_bpm of
//                  its blocks (all of them for the single scan);
//   kLayoutRaster: one component's blocks in raster order over its own block
//                  grid (comp_bw wide; T.81 A.2.2), one block per "MCU".
constexpr uint32_t kLayoutMcu = 0, kLayoutRaster = 1;
__host__ __device__ __forceinline__ uint32_t geo_make(uint32_t out_bpm, uint32_t lh, uint32_t lv, uint32_t bw)
{
    return out_bpm | (lh << 4) | (lv << 6) | (bw << 8);
}

// Per-subsequence statistics of a run; combined with an ordered, segmented
// operator to get each subsequence's block index and DC predictors.
struct SubStats {
    uint32_t nblk : 30;   // DC units decoded (= blocks started)
    uint32_t flags : 2;   // kReset | kError
    int32_t dc[3];        // sum of DC differences per component since the last reset in this run
};
static_assert(sizeof(SubStats) == 16, "SubStats layout");

constexpr uint32_t kReset = 1;      // a restart (or the frame start) happened inside the run
constexpr uint32_t kError = 2;      // invalid symbol / overrun (fatal only for the verified chain)

// Frame status bits (device -> host).
constexpr uint32_t kStatusFallback = 1;   // verification needed the sequential path
constexpr uint32_t kStatusCorrupt = 2;    // invalid entropy data on the verified chain
constexpr uint32_t kStatusCount = 4;      // block count != expected

__host__ __device__ __forceinline__ SubStats stats_identity()
{
    SubStats s;
    s.nblk = 0;
    s.flags = 0;
    s.dc[0] = s.dc[1] = s.dc[2] = 0;
    return s;
}

// a then b
__host__ __device__ __forceinline__ SubStats stats_combine(const SubStats& a, const SubStats& b)
{
    SubStats r;
    r.nblk = a.nblk + b.nblk;
    const bool rb = (b.flags & kReset) != 0;
    for (int c = 0; c < 3; ++c) r.dc[c] = rb ? b.dc[c] : a.dc[c] + b.dc[c];
    r.flags = a.flags | b.flags;
    return r;
}

// ---- decoder state --------------------------------------------------------
// bits 0-31 pos, 32-38 z, 39-41 j, 42-63 restart-interval (segment) index.
// States compare in full: a run is a deterministic function of all 64 bits,
// which is what makes "two chains that agree at a boundary agree from there
// on" hold.  The segment index is not redundant: a run from a wrong entry can
// decode through a restart pad as data and stop past the segment end without
// taking the restart, leaving (pos, z, j) that may coincide with the true
// state's but a stale segment index (and DC predictors that were never
// reset).  The one pair of equivalent states that differ only in the index,
// a segment start seen from either side, costs at most one extra re-run.

__host__ __device__ __forceinline__ uint64_t pack_state(uint32_t pos, uint32_t j, uint32_t z, uint32_t seg)
{
    return static_cast<uint64_t>(pos) | (static_cast<uint64_t>(z) << 32) | (static_cast<uint64_t>(j) << 39) |
           (static_cast<uint64_t>(seg) << 42);
}
__host__ __device__ __forceinline__ uint32_t st_pos(uint64_t s) { return static_cast<uint32_t>(s); }
__host__ __device__ __forceinline__ uint32_t st_z(uint64_t s) { return static_cast<uint32_t>(s >> 32) & 127; }
__host__ __device__ __forceinline__ uint32_t st_j(uint64_t s) { return static_cast<uint32_t>(s >> 39) & 7; }
__host__ __device__ __forceinline__ uint32_t st_seg(uint64_t s) { return static_cast<uint32_t>(s >> 42); }
__host__ __device__ __forceinline__ bool same_state(uint64_t a, uint64_t b) { return a == b; }

__host__ __device__ __forceinline__ uint32_t bswap32(uint32_t x)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_perm(0u, x, 0x00010203u);
#else
    return __builtin_bswap32(x);
#endif
}

// First segment whose end is > pos (nseg if pos is at/after the data end).
__host__ __device__ __forceinline__ uint32_t find_segment(const uint32_t* seg_end, uint32_t nseg, uint32_t pos)
{
    uint32_t lo = 0, hi = nseg;
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (seg_end[mid] > pos) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}

// Bitstream block j of an MCU: scan components in SOS order, H*V blocks each
// (src/decoder.cpp:308-344); `out slot` is its place in the MCU-major output
// (Y blocks, then Cb, then Cr, as hjd_frame expects).
__host__ __device__ __forceinline__ uint32_t jinfo_make(int dc_slot, int ac_slot, int comp, int out_slot)
{
    return static_cast<uint32_t>(dc_slot | (ac_slot << 3) | (comp << 6) | (out_slot << 8));
}

// What the symbol step needs about bitstream block j of an MCU: the byte
// offsets of its DC and AC tables from RunCtx::tabs, its component as 0/1
// multipliers (the DC sums accumulate with multiply-adds, no branch), and its
// jinfo.  One 32-B record per j, in LDS on the device, read when j changes.
struct alignas(16) BlockInfo {
    uint32_t tdc, tac;
    int32_t m0, m1, m2;
    uint32_t ji;
    uint32_t sac;   // first entry of the AC table's step table (RunCtx::steps)
    uint32_t pad;
};
static_assert(sizeof(BlockInfo) == 32, "BlockInfo layout");

__host__ __device__ __forceinline__ BlockInfo block_info(uint32_t ji)
{
    BlockInfo b;
    b.tdc = (ji & 7) * static_cast<uint32_t>(sizeof(HuffLut));
    b.tac = ((ji >> 3) & 7) * static_cast<uint32_t>(sizeof(HuffLut));
    const uint32_t comp = (ji >> 6) & 3;
    b.m0 = comp == 0;
    b.m1 = comp == 1;
    b.m2 = comp == 2;
    b.ji = ji;
    b.sac = ((ji >> 3) & 7) << kStepBits;
    b.pad = 0;
    return b;
}

constexpr int kMaxBpm = 6;   // blocks per MCU of the supported samplings (4:2:0)

// Everything a run needs about its frame.  `tabs` points at the frame's
// tables and `blocks` at its block_info() records (both LDS on the device),
// `data` at its destuffed bytes (4-B aligned).
struct RunCtx {
    const uint8_t* data;
    const uint32_t* seg_end;   // bit offsets, nseg entries
    const HuffLut* tabs;
    const BlockInfo* blocks;   // [bpm]
    uint32_t nseg, data_bits;
    int bpm;
    uint32_t seg_blocks;       // EntFrame::seg_blocks
    const uint8_t* steps;      // [table][1 << kStepBits] AC step entries (LDS), or null: one unit per step
    uint32_t layout, geo, mcu_w;   // EntFrame: where the scan's blocks go (block_dest)
};

// Write mode: where the scan's block lands in the image's MCU-major
// coefficients.  (u, v): kLayoutMcu -- the scan MCU and the block's j in it;
// kLayoutRaster -- the block's column and row in the component's grid.
__host__ __device__ __forceinline__ uint32_t block_dest(const RunCtx& c, uint32_t u, uint32_t v, uint32_t slot)
{
    const uint32_t out_bpm = c.geo & 15;
    if (c.layout == kLayoutMcu) return u * out_bpm + slot;
    const uint32_t lh = (c.geo >> 4) & 3, lv = (c.geo >> 6) & 3;
    const uint32_t mcu = (v >> lv) * c.mcu_w + (u >> lh);
    return mcu * out_bpm + slot + ((v & ((1u << lv) - 1)) << lh) + (u & ((1u << lh) - 1));
}

// AC step entry (sync mode): the AC units that a kStepBits-bit peek decodes
// completely, taken in one step, since a sync run needs no AC values --
// only how far they move pos and z.  One byte: [3:0] bits consumed, [7:4] 15
// if the last unit is an EOB (the block ends), else how far the units move z
// (<= 14; the units before an EOB also move it by <= 14).  0: the first
// unit's code or extra bits reach past the peek (or it moves z by 15 or more);
// one byte per entry keeps the sync kernel's LDS small.
constexpr uint32_t kStepEnds = 15;
__host__ __device__ __forceinline__ uint32_t step_bits(uint32_t e) { return e & 15; }
__host__ __device__ __forceinline__ uint32_t step_zadv(uint32_t e) { return e >> 4; }   // kStepEnds: EOB

// Step entry of an AC table for the kStepBits-bit prefix p: units decoded from
// p alone, in order, until one does not fit, an EOB (taken, last) or z would
// move by more than 14.  Every unit is one the LUT decodes (codes <= kLutBits bits).
__host__ __device__ __forceinline__ uint8_t step_entry(const HuffLut& t, uint32_t p)
{
    uint32_t o = 0, zadv = 0;
    while (o < static_cast<uint32_t>(kStepBits)) {
        const uint32_t e = t.lut[((p << o) & ((1u << kStepBits) - 1)) >> (kStepBits - kLutBits)];
        const uint32_t total = e & 31, zk = e >> 9;
        if (e == 0 || o + total > static_cast<uint32_t>(kStepBits)) break;
        if (zk == 64) {   // EOB: the block ends
            o += total;
            zadv = kStepEnds;
            break;
        }
        if (zadv + zk >= kStepEnds) break;
        zadv += zk;
        o += total;
    }
    return static_cast<uint8_t>(o | zadv << 4);
}

// The record of bitstream block j.
__host__ __device__ __forceinline__ BlockInfo block_of(const RunCtx& c, uint32_t j) { return c.blocks[j]; }

// (x >> off) & ((1 << w) - 1), w <= 31 (v_bfe_u32); off + w <= 32
__host__ __device__ __forceinline__ uint32_t ubfe(uint32_t x, uint32_t off, uint32_t w)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_ubfe(x, off, w);
#else
    return (x >> off) & ((1u << w) - 1);
#endif
}

// a * b + c for |a|, |b| < 2^23 (v_mad_i32_i24; b is a 0/1 multiplier here).
// asm: the compiler otherwise widens the pattern to v_mad_u64_u32.
__host__ __device__ __forceinline__ int32_t mad24(int32_t a, int32_t b, int32_t c)
{
#ifdef __HIP_DEVICE_COMPILE__
    int32_t r;
    asm("v_mad_i32_i24 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
    return r;
#else
    return a * b + c;
#endif
}

// Output side of a write-mode run.
struct RunOut {
    int16_t* coefs;        // frame's first block
    int16_t* stage;        // this lane's 64-coefficient staging slot (LDS on the device)
    uint32_t blk;          // index (in scan order) of the next block this run owns
    uint32_t nblocks;      // blocks of the scan
    uint32_t nout;         // blocks of the image (destinations must stay below)
    int32_t pred[3];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// Write-mode staging: only the quarter of the block being filled (16
// coefficients, z order) lives in LDS; quarters are flushed with two 16-B
// stores as z moves past them, so every block is still written exactly once
// as 8 x 16 B, while the LDS per lane is 40 B instead of a whole block.
__host__ __device__ __forceinline__ void zero_quarter(int16_t* stage)
{
    u32x2* p = reinterpret_cast<u32x2*>(stage);
    const u32x2 zv = {0u, 0u};
    p[0] = zv;
    p[1] = zv;
    p[2] = zv;
    p[3] = zv;
}

// Store the staged quarter q to the block, zeros for quarters q+1 .. qn-1,
// and clear the stage.
__host__ __device__ __forceinline__ void flush_quarters(int16_t* blk, int16_t* stage, uint32_t q, uint32_t qn)
{
    u32x4* d = reinterpret_cast<u32x4*>(blk);
    u32x2* sp = reinterpret_cast<u32x2*>(stage);
    const u32x2 a = sp[0], b = sp[1], c = sp[2], e = sp[3];
    d[2 * q] = u32x4{a.x, a.y, b.x, b.y};
    d[2 * q + 1] = u32x4{c.x, c.y, e.x, e.y};
    const u32x4 zv = {0u, 0u, 0u, 0u};
    for (uint32_t i = q + 1; i < qn; ++i) {
        d[2 * i] = zv;
        d[2 * i + 1] = zv;
    }
    zero_quarter(stage);
}

// Raw (little-endian) 16-B chunk of the frame's bit string.
__host__ __device__ __forceinline__ u32x4 load_chunk(const RunCtx& c, uint32_t ci)
{
    return reinterpret_cast<const u32x4*>(c.data)[ci];
}

// Word k (0..3) of a chunk: a two-level select, no indexed registers.
__host__ __device__ __forceinline__ uint32_t pick(const u32x4& v, uint32_t k)
{
    const uint32_t lo = (k & 1) ? v.y : v.x, hi = (k & 1) ? v.w : v.z;
    return (k & 2) ? hi : lo;
}

__host__ __device__ __forceinline__ u32x4 bswap4(const u32x4& v)
{
    u32x4 s;
    s.x = bswap32(v.x);
    s.y = bswap32(v.y);
    s.z = bswap32(v.z);
    s.w = bswap32(v.w);
    return s;
}

// Per-lane bit window: w0:w1 are the (byte-swapped) words wi, wi+1 under the
// read position; the following words come from the swapped 16-B chunk `cur`
// (word ci next), and `r`, the raw chunk after it, is in flight -- a lead of
// 4-8 words (~26-52 symbols), enough to hide an HBM miss (each lane streams
// its own lines, so every line crossing misses the caches).  r is only read
// (swapped into cur) when cur runs out, four advances after its load was
// issued, so the wait lands there, and every definition of r is a load, so
// the new load can target r's registers.  An advance moves one word and picks
// one: no shifted queue, so divergent advances cost few instructions.
struct BitWindow {
    uint32_t w0, w1;
    u32x4 cur, r;
    uint32_t ci, next, wi;

    __host__ __device__ __forceinline__ void advance(const RunCtx& c)
    {
        w0 = w1;
        w1 = pick(cur, ci);
#ifdef __HIP_DEVICE_COMPILE__
        // take the word before cur can be replaced: otherwise the select sinks
        // below the refill and cur is copied around it
        asm volatile("" : "+v"(w1)::"memory");
#endif
        ++wi;
        if (++ci == 4) {
            cur = bswap4(r);
            ci = 0;
            r = load_chunk(c, next++);
        }
    }

    __host__ __device__ __forceinline__ void seek(const RunCtx& c, uint32_t word)
    {
        const uint32_t q = word >> 2, k = word & 3;
        const u32x4 a = load_chunk(c, q), b = load_chunk(c, q + 1);
        const bool lo = k < 2;   // word + 2 is still in a
        r = load_chunk(c, lo ? q + 1 : q + 2);
        next = lo ? q + 2 : q + 3;
        w0 = bswap32(pick(a, k));
        w1 = bswap32(k < 3 ? pick(a, k + 1) : b.x);
        wi = word;
        cur = bswap4(lo ? a : b);
        ci = lo ? k + 2 : k - 2;
    }
};

__host__ __device__ __forceinline__ uint32_t funnel(uint32_t w0, uint32_t w1, uint32_t off)
{
    return static_cast<uint32_t>(((static_cast<uint64_t>(w0) << 32) | w1) >> (32 - off));
}

// Unit entry of a code longer than the LUT (T.81 F.2.2.3): the length is the
// first l with code_l <= MAXCODE[l]; the six compares use independent loads
// and selects instead of a dependent loop.  An invalid code sets kError and
// consumes 16 bits as a zero symbol.
__host__ __device__ __forceinline__ uint32_t long_code_entry(const HuffLut& t, uint32_t peek, bool dc, uint32_t& flags)
{
    static_assert(kLutBits == 10, "long-code lengths 11..16");
    const int32_t c11 = static_cast<int32_t>(peek >> 21), c12 = static_cast<int32_t>(peek >> 20);
    const int32_t c13 = static_cast<int32_t>(peek >> 19), c14 = static_cast<int32_t>(peek >> 18);
    const int32_t c15 = static_cast<int32_t>(peek >> 17), c16 = static_cast<int32_t>(peek >> 16);
    const bool p11 = c11 <= t.maxcode[11], p12 = c12 <= t.maxcode[12], p13 = c13 <= t.maxcode[13];
    const bool p14 = c14 <= t.maxcode[14], p15 = c15 <= t.maxcode[15], p16 = c16 <= t.maxcode[16];
    const uint32_t len = p11 ? 11u : p12 ? 12u : p13 ? 13u : p14 ? 14u : p15 ? 15u : 16u;
    const int32_t code = static_cast<int32_t>(peek >> (32 - len));
    uint32_t sym = t.vals[(code + t.delta[len]) & 255];
    if (!(p11 || p12 || p13 || p14 || p15 || p16)) {
        flags |= kError;
        sym = 0;
    }
    return unit_entry(len, sym, dc);
}

// Decode one run: from `entry` until the first unit boundary >= stop (write
// mode: and until the block this run owns is complete).  Accumulates `st`
// (must start as the identity).  Returns the exit state.  Per-component sums
// live in scalars (selects, not indexed arrays: no scratch on the device).
// kMarks > 0 (sync mode): the run also passes marks mpos[0] < mpos[1] ... <=
// stop and records, at the first unit boundary >= each, the state (mstate)
// and the statistics since the previous mark (mstats; `st` then holds those
// after the last mark) -- exactly what separate runs split there would give,
// without a window reload per piece.  The marks are taken between passes of
// the unit loop (one pass per mark), not inside it: a mark test in the loop
// made every unit dearer (gfx950, same box: spec 118 vs 100 us, cand 147 vs
// 115 us per FHD frame; profiles/r06yz_fhd420_kernel_medians.json).
template <bool kWrite, int kMarks = 0>
__host__ __device__ __forceinline__ uint64_t run(const RunCtx& c, uint64_t entry, uint32_t stop, SubStats& st,
                                                 RunOut* out, const uint32_t* mpos = nullptr,
                                                 uint64_t* mstate = nullptr, SubStats* mstats = nullptr)
{
    static_assert(!kWrite || kMarks == 0, "marks: sync mode only");
    int mi = 0;
    uint32_t pos = st_pos(entry);
    uint32_t z = st_z(entry);
    uint32_t j = st_j(entry);
    uint32_t seg = st_seg(entry);
    int32_t nblk = static_cast<int32_t>(st.nblk), d0 = st.dc[0], d1 = st.dc[1], d2 = st.dc[2];
    uint32_t flags = st.flags;
    int32_t p0 = 0, p1 = 0, p2 = 0;
    // write mode, kept incrementally: the scan block index, its j in the scan
    // MCU (blk % bpm) and its block_dest coordinates (bu, bv)
    uint32_t blk = 0, blk_j = 0, bu = 0, bv = 0;
    if (kWrite) {
        p0 = out->pred[0];
        p1 = out->pred[1];
        p2 = out->pred[2];
        blk = out->blk;
        if (c.layout == kLayoutMcu) {
            bu = blk / static_cast<uint32_t>(c.bpm);
            blk_j = blk - bu * static_cast<uint32_t>(c.bpm);
        } else {
            bv = blk / (c.geo >> 8);
            bu = blk - bv * (c.geo >> 8);
        }
    }
    uint64_t result;
    if (seg >= c.nseg) {
        result = pack_state(c.data_bits, 0, 0, c.nseg);
    } else {
        // An entry exactly at a segment start restarts the DC prediction itself:
        // (e, seg s-1) and (e, seg s) compare equal, and only the former reaches
        // the restart through the jump below.
        if (pos == 0 || (seg > 0 && pos == c.seg_end[seg - 1])) {
            flags |= kReset;
            d0 = d1 = d2 = 0;
            p0 = p1 = p2 = 0;
            // write mode: a restart interval starts with block seg * seg_blocks
            // (T.81 B.2.1: every interval but the last holds DRI MCUs)
            if (kWrite && c.seg_blocks && blk != seg * c.seg_blocks) flags |= kError;
        }
        uint32_t seg_end = c.seg_end[seg];
        if (seg_end < pos) flags |= kError;   // consumed before the window loads are issued
        BitWindow bw;
        bool owned = false;                            // write mode: current block started in this run
        int16_t* cur = nullptr;                        // write mode: its destination (null: not written)
        uint32_t quarter = 0;                          // write mode: quarter of the block being staged
        BlockInfo bi = block_of(c, j);
        result = 0;
        bool done = false;
        bw.seek(c, pos >> 5);
        for (;; ++mi) {   // one pass per mark, then to stop
            const uint32_t lim = mi < kMarks ? mpos[mi] : stop;
            // One loop: a nested re-seek loop (so the window never merges with a
            // seek) measured 13% slower -- its extra exits cost more exec-mask
            // bookkeeping per unit than the merge copies.
            for (;;) {
                if (pos >= lim && (!kWrite || !owned)) break;
                const uint32_t nwi = pos >> 5;
                if (nwi != bw.wi) {
                    if (nwi == bw.wi + 1) bw.advance(c);
                    else bw.seek(c, nwi);   // an overrun of a restart pad moved pos back
                }
                const uint32_t peek = funnel(bw.w0, bw.w1, pos & 31);
                // ---- restart-interval end: < 8 bits left, all ones (or overrun) ----
                const int32_t left = static_cast<int32_t>(seg_end - pos);
                if (left < 8) {
                    const bool ones = left <= 0 || (peek >> (32 - left)) == (1u << left) - 1;
                    if (ones) {
                        if (left < 0 || (kWrite && owned)) flags |= kError;   // overrun / block cut by the pad
                        pos = seg_end;
                        ++seg;
                        // write mode: the interval just closed must have held
                        // exactly DRI MCUs (the host decoder counts them and resyncs
                        // at the marker; a count that differs is corrupt data)
                        if (kWrite && c.seg_blocks && seg < c.nseg && blk != seg * c.seg_blocks) flags |= kError;
                        j = 0;
                        z = 0;
                        bi = block_of(c, 0);
                        owned = false;
                        cur = nullptr;
                        flags |= kReset;
                        d0 = d1 = d2 = 0;
                        p0 = p1 = p2 = 0;
                        if (seg >= c.nseg) {
                            result = pack_state(c.data_bits, 0, 0, c.nseg);
                            done = true;
                            break;
                        }
                        seg_end = c.seg_end[seg];
                        // consume the load inside this rare branch, so the loop
                        // head does not wait for every outstanding memory op
                        if (seg_end < pos) flags |= kError;
                        continue;
                    }
                }
                const bool dc = z == 0;
                // ---- sync mode: the AC units the peek holds, in one step ----
                // Taken only where single units would give the same state: all of
                // them end at or before `stop`, >= 8 bits before the segment end (no pad
                // check in between), and z stays <= 63 (no index-63 error case).
                // (A branch-free form that computes the step and the unit outcome in
                // every lane and selects measured slower: DESIGN.md s10.1.)
                if (!kWrite && c.steps && !dc) {
                    const uint32_t se = c.steps[bi.sac + (peek >> (32 - kStepBits))];
                    const uint32_t nb = step_bits(se), za = step_zadv(se);
                    const bool ends = za == kStepEnds;
                    // an EOB entry's units before the EOB move z by <= 14: z <= 49 keeps them <= 63
                    if (se != 0 && z + (ends ? 14 : za) <= 63 && left >= static_cast<int32_t>(nb) + 8 && pos + nb <= lim) {
                        pos += nb;
                        if (ends) {
                            z = 0;
                            j = j + 1 == static_cast<uint32_t>(c.bpm) ? 0 : j + 1;
                            bi = block_of(c, j);
                        } else {
                            z += za;
                        }
                        continue;
                    }
                }
                // ---- one unit: Huffman symbol + extra bits (unit_entry fields) ----
                const HuffLut& t = *reinterpret_cast<const HuffLut*>(reinterpret_cast<const char*>(c.tabs) +
                                                                     (dc ? bi.tdc : bi.tac));
                uint32_t e = t.lut[peek >> (32 - kLutBits)];
                if (e == 0) e = long_code_entry(t, peek, dc, flags);
                const uint32_t total = e & 31, s = (e >> 5) & 15;
                uint32_t zk = e >> 9;
                if (zk == kZkDcError) {   // DC symbol > 11
                    flags |= kError;
                    zk = 1;
                }
                // extra bits -> value (T.81 F.2.2.1 EXTEND); s = 0 gives 0
                const uint32_t bits = ubfe(peek, 32 - total, s);
                const uint32_t m = (1u << s) - 1;
                const int32_t v = bits <= (m >> 1) ? static_cast<int32_t>(bits - m) : static_cast<int32_t>(bits);
                pos += total;
                const uint32_t zn = z + zk;
                if (zn > 64 && zk != 64) flags |= kError;   // AC coefficient or ZRL past index 63 (not EOB)
                // DC unit: a block starts (per-component sums by 0/1 multipliers, no branch)
                const int32_t dv = dc ? v : 0;
                nblk += dc ? 1 : 0;
                d0 = mad24(dv, bi.m0, d0);
                d1 = mad24(dv, bi.m1, d1);
                d2 = mad24(dv, bi.m2, d2);
                if (kWrite) {
                    if (dc) {
                        owned = true;
                        p0 = mad24(v, bi.m0, p0);
                        p1 = mad24(v, bi.m1, p1);
                        p2 = mad24(v, bi.m2, p2);
                        // MCU-major destination; on valid data blk % bpm == j.  Blocks past
                        // the scan's count are ignored (as the host decoder stops there).
                        const uint32_t dst = block_dest(c, bu, bv, bi.ji >> 8);
                        cur = nullptr;
                        if (blk < out->nblocks) {
                            if (dst < out->nout && blk_j == j) {
                                cur = out->coefs + static_cast<uint64_t>(dst) * 64;
                                zero_quarter(out->stage);
                                out->stage[0] = static_cast<int16_t>(p0 * bi.m0 + p1 * bi.m1 + p2 * bi.m2);
                                quarter = 0;
                            } else {
                                flags |= kError;   // a restart interval ended inside an MCU
                            }
                        }
                    } else if (s != 0 && zn <= 64 && cur) {
                        const uint32_t zi = zn - 1;   // the coefficient's index: z + run
                        const uint32_t qz = zi >> 4;
                        if (qz != quarter) {
                            flush_quarters(cur, out->stage, quarter, qz);
                            quarter = qz;
                        }
                        out->stage[zi & 15] = static_cast<int16_t>(v);
                    }
                }
                if (zn >= 64) {   // EOB, ZRL or a coefficient reaching the end, or an error
                    if (kWrite && owned) {
                        if (cur) flush_quarters(cur, out->stage, quarter, 4);   // the rest of the block
                        blk += 1;
                        if (c.layout == kLayoutMcu) {
                            const bool wrap = blk_j + 1 == static_cast<uint32_t>(c.bpm);
                            blk_j = wrap ? 0 : blk_j + 1;
                            bu += wrap ? 1 : 0;
                        } else {
                            const bool wrap = bu + 1 == (c.geo >> 8);
                            bu = wrap ? 0 : bu + 1;
                            bv += wrap ? 1 : 0;
                        }
                        owned = false;
                        cur = nullptr;
                    }
                    z = 0;
                    j = j + 1 == static_cast<uint32_t>(c.bpm) ? 0 : j + 1;
                    bi = block_of(c, j);
                } else {
                    z = zn;
                }
            }
            if (done || mi >= kMarks) break;   // the end of the data, or past the last mark
            // mark mi: its state and the statistics since the previous one
            mstate[mi] = pack_state(pos, j, z, seg);
            mstats[mi].nblk = static_cast<uint32_t>(nblk);
            mstats[mi].flags = flags;
            mstats[mi].dc[0] = d0;
            mstats[mi].dc[1] = d1;
            mstats[mi].dc[2] = d2;
            nblk = d0 = d1 = d2 = 0;
            flags = 0;
        }
        if (!done) result = pack_state(pos, j, z, seg);
    }
    // marks the run did not reach (the data ended first): the exit state, and
    // the statistics so far for the first of them (as separate runs would give)
    for (; kMarks && mi < kMarks; ++mi) {
        mstate[mi] = result;
        mstats[mi].nblk = static_cast<uint32_t>(nblk);
        mstats[mi].flags = flags;
        mstats[mi].dc[0] = d0;
        mstats[mi].dc[1] = d1;
        mstats[mi].dc[2] = d2;
        nblk = d0 = d1 = d2 = 0;
        flags = 0;
    }
    st.nblk = static_cast<uint32_t>(nblk);
    st.dc[0] = d0;
    st.dc[1] = d1;
    st.dc[2] = d2;
    st.flags = flags;
    if (kWrite) {
        out->pred[0] = p0;
        out->pred[1] = p1;
        out->pred[2] = p2;
        out->blk = blk;
    }
    return result;
}

// ---- slot maps of the speculative sync's chain kernel ----------------------
// A slot map is 20 bytes (5 dwords): byte s = the slot of the next
// subsequence that slot s leads to, < 20, or 0xFF (none; absorbing).
// Composition r = g . f, r[s] = g[f[s]], as three byte permutes per dword
// (v_perm_b32 picks 4 bytes out of 8 by the selector bytes 0..7; selector
// bytes >= 13 give 0xFF) and a per-byte select on bits 3 and 4 of f's bytes:
// bytes 0-7 of g from (g0, g1), 8-15 from (g2, g3) with the selector's bit 3
// flipped, 16-19 from g4 with bit 4 flipped; a 0xFF selector has bit 4 set and
// flips to 0xEF, which the permute turns into 0xFF.
__host__ __device__ __forceinline__ uint32_t byte_perm(uint32_t hi, uint32_t lo, uint32_t sel)
{
#ifdef __HIP_DEVICE_COMPILE__
    return __builtin_amdgcn_perm(hi, lo, sel);
#else
    uint32_t r = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t k = (sel >> (8 * i)) & 0xFF;
        uint32_t b;
        if (k < 4) b = (lo >> (8 * k)) & 0xFF;
        else if (k < 8) b = (hi >> (8 * (k - 4))) & 0xFF;
        else if (k == 12) b = 0;
        else if (k >= 13) b = 0xFF;
        else {   // 8..11: sign of a 16-bit half (unused here)
            const uint32_t w = k < 10 ? lo : hi;
            b = ((w >> ((k & 1) ? 31 : 15)) & 1) ? 0xFF : 0;
        }
        r |= b << (8 * i);
    }
    return r;
#endif
}

__host__ __device__ __forceinline__ void slot_compose(const uint32_t (&f)[5], const uint32_t (&g)[5], uint32_t (&r)[5])
{
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const uint32_t idx = f[i];
        const uint32_t lo = byte_perm(g[1], g[0], idx);
        const uint32_t mid = byte_perm(g[3], g[2], idx ^ 0x08080808u);
        const uint32_t hi = byte_perm(g[4], g[4], idx ^ 0x10101010u);
        const uint32_t m3 = ((idx >> 3) & 0x01010101u) * 0xFFu;   // bytes >= 8 (bit 3)
        const uint32_t m4 = ((idx >> 4) & 0x01010101u) * 0xFFu;   // bytes >= 16 and 0xFF (bit 4)
        r[i] = (hi & m4) | (~m4 & ((mid & m3) | (lo & ~m3)));
    }
}

}  // namespace ent
}  // namespace hjd
