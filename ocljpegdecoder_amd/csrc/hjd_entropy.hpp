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
constexpr int kMaxTables = 6;                   // DC+AC per component at most
constexpr int kGroupSubs = 256;                 // subsequences per workgroup (one per thread)
constexpr int kWarm = 8;                        // leading subsequences a group shares with its predecessor
constexpr int kOwn = kGroupSubs - kWarm;        // subsequences a group is responsible for
constexpr int kDefaultSubBits = 2048;           // S
constexpr int kStageStride = 24;                // int16 per lane in the staging buffer: one 16-coefficient quarter (+pad)

// One Huffman table in device form (2448 B, 16-B multiple).
struct HuffLut {
    uint16_t lut[1 << kLutBits];   // (len << 8) | symbol for codes <= kLutBits bits, 0: longer code
    int32_t maxcode[17];           // largest code of each length, -1 if none (T.81 F.2.2.3)
    int32_t delta[17];             // valptr[len] - mincode[len]
    uint8_t vals[256];
    uint8_t pad[8];
};
static_assert(sizeof(HuffLut) == 2448, "HuffLut layout");

// Per-frame record of an entropy batch (device, 64 B).
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
    uint8_t ntab, bpm, sampling, pad0;
    uint16_t jinfo[6];    // per bitstream block j of an MCU: dc slot | ac slot << 3 | comp << 6 | out slot << 8
};
static_assert(sizeof(EntFrame) == 64, "EntFrame layout");

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

// Everything a run needs about its frame.  `tabs` points at the frame's
// tables (LDS on the device), `data` at its destuffed bytes (4-B aligned).
struct RunCtx {
    const uint8_t* data;
    const uint32_t* seg_end;   // bit offsets, nseg entries
    const HuffLut* tabs;
    uint32_t nseg, data_bits;
    int bpm;
    uint64_t jinfo_q;    // jinfo[0..3], 16 bits each
    uint32_t jinfo_hi;   // jinfo[4..5]
};

// Blend (not select) between the two words so the context stays in registers.
__host__ __device__ __forceinline__ uint32_t jinfo_of(const RunCtx& c, uint32_t j)
{
    const uint64_t m = 0ull - static_cast<uint64_t>(j < 4);
    const uint64_t q = (c.jinfo_q & m) | (static_cast<uint64_t>(c.jinfo_hi) & ~m);
    return static_cast<uint32_t>(q >> ((j & 3) * 16)) & 0xFFFF;
}

// Output side of a write-mode run.
struct RunOut {
    int16_t* coefs;        // frame's first block
    int16_t* stage;        // this lane's 64-coefficient staging slot (LDS on the device)
    uint32_t blk;          // index of the next block this run owns
    uint32_t nblocks;
    int32_t pred[3];
};

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Write-mode staging: only the quarter of the block being filled (16
// coefficients, z order) lives in LDS; quarters are flushed with two 16-B
// stores as z moves past them, so every block is still written exactly once
// as 8 x 16 B, while the LDS per lane is 48 B instead of a whole block.
__host__ __device__ __forceinline__ void zero_quarter(int16_t* stage)
{
    u32x4* p = reinterpret_cast<u32x4*>(stage);
    const u32x4 zv = {0u, 0u, 0u, 0u};
    p[0] = zv;
    p[1] = zv;
}

// Store the staged quarter q to the block, zeros for quarters q+1 .. qn-1,
// and clear the stage.
__host__ __device__ __forceinline__ void flush_quarters(int16_t* blk, int16_t* stage, uint32_t q, uint32_t qn)
{
    u32x4* d = reinterpret_cast<u32x4*>(blk);
    u32x4* sp = reinterpret_cast<u32x4*>(stage);
    d[2 * q] = sp[0];
    d[2 * q + 1] = sp[1];
    const u32x4 zv = {0u, 0u, 0u, 0u};
    for (uint32_t i = q + 1; i < qn; ++i) {
        d[2 * i] = zv;
        d[2 * i + 1] = zv;
    }
    sp[0] = zv;
    sp[1] = zv;
}

// Raw (little-endian) 16-B chunk of the frame's bit string.
__host__ __device__ __forceinline__ u32x4 load_chunk(const RunCtx& c, uint32_t ci)
{
    return reinterpret_cast<const u32x4*>(c.data)[ci];
}

// Per-lane bit window: w0:w1 are the (byte-swapped) words under the read
// position; q holds the following words and r the next raw 16-B chunk, still
// in flight -- about 18 symbols of lead, enough to hide an HBM miss (each lane
// streams its own lines, so every line crossing misses the caches).  r is only
// consumed (swapped into q) four word-advances after its load is issued, so
// the wait lands there; only fixed register moves, no indexed registers.
struct BitWindow {
    uint32_t w0, w1, q0, q1, q2, q3, q4, q5;
    u32x4 r;
    uint32_t nq, next, wi;

    __host__ __device__ __forceinline__ void advance(const RunCtx& c)
    {
        w0 = w1;
        w1 = q0;
        q0 = q1;
        q1 = q2;
        q2 = q3;
        q3 = q4;
        q4 = q5;
        ++wi;
        if (--nq == 0) {
            q0 = bswap32(r.x);
            q1 = bswap32(r.y);
            q2 = bswap32(r.z);
            q3 = bswap32(r.w);
            nq = 4;
            r = load_chunk(c, next++);
        }
    }

    __host__ __device__ __forceinline__ void seek(const RunCtx& c, uint32_t word)
    {
        const uint32_t ci = word >> 2;
        const u32x4 a = load_chunk(c, ci), b = load_chunk(c, ci + 1);
        r = load_chunk(c, ci + 2);
        next = ci + 3;
        w0 = bswap32(a.x);
        w1 = bswap32(a.y);
        q0 = bswap32(a.z);
        q1 = bswap32(a.w);
        q2 = bswap32(b.x);
        q3 = bswap32(b.y);
        q4 = bswap32(b.z);
        q5 = bswap32(b.w);
        nq = 6;
        wi = ci * 4;
        for (uint32_t i = 0; i < (word & 3); ++i) advance(c);
    }
};

__host__ __device__ __forceinline__ uint32_t funnel(uint32_t w0, uint32_t w1, uint32_t off)
{
    return static_cast<uint32_t>(((static_cast<uint64_t>(w0) << 32) | w1) >> (32 - off));
}

// Decode one run: from `entry` until the first unit boundary >= stop (write
// mode: and until the block this run owns is complete).  Accumulates `st`
// (must start as the identity).  Returns the exit state.  Per-component sums
// live in scalars (selects, not indexed arrays: no scratch on the device).
template <bool kWrite>
__host__ __device__ __forceinline__ uint64_t run(const RunCtx& c, uint64_t entry, uint32_t stop, SubStats& st,
                                                 RunOut* out)
{
    uint32_t pos = st_pos(entry);
    uint32_t z = st_z(entry);
    uint32_t j = st_j(entry);
    uint32_t seg = st_seg(entry);
    int32_t nblk = static_cast<int32_t>(st.nblk), d0 = st.dc[0], d1 = st.dc[1], d2 = st.dc[2];
    uint32_t flags = st.flags;
    int32_t p0 = 0, p1 = 0, p2 = 0;
    uint32_t blk = 0;
    if (kWrite) {
        p0 = out->pred[0];
        p1 = out->pred[1];
        p2 = out->pred[2];
        blk = out->blk;
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
        }
        uint32_t seg_end = c.seg_end[seg];
        if (seg_end < pos) flags |= kError;   // consumed before the window loads are issued
        BitWindow bw;
        bw.seek(c, pos >> 5);
        bool owned = false;                            // write mode: current block started in this run
        int16_t* cur = nullptr;                        // write mode: its destination (null: not written)
        uint32_t quarter = 0;                          // write mode: quarter of the block being staged
        uint32_t ji = jinfo_of(c, j);
        result = 0;
        bool done = false;
        while (!done) {
            if (pos >= stop && (!kWrite || !owned)) break;
            const uint32_t nwi = pos >> 5;
            if (nwi != bw.wi) {
                if (nwi == bw.wi + 1) bw.advance(c);
                else bw.seek(c, nwi);
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
                    j = 0;
                    z = 0;
                    ji = jinfo_of(c, 0);
                    owned = false;
                    cur = nullptr;
                    flags |= kReset;
                    d0 = d1 = d2 = 0;
                    p0 = p1 = p2 = 0;
                    if (seg >= c.nseg) {
                        result = pack_state(c.data_bits, 0, 0, c.nseg);
                        done = true;
                    } else {
                        seg_end = c.seg_end[seg];
                        // consume the load inside this rare branch, so the loop
                        // head does not wait for every outstanding memory op
                        if (seg_end < pos) flags |= kError;
                    }
                    continue;
                }
            }
            // ---- one Huffman symbol + its extra bits ----
            const uint32_t comp = (ji >> 6) & 3;
            const bool dc = z == 0;
            const HuffLut& t = c.tabs[dc ? (ji & 7) : ((ji >> 3) & 7)];
            const uint32_t e = t.lut[peek >> (32 - kLutBits)];
            uint32_t len, sym;
            if (e != 0) {
                len = e >> 8;
                sym = e & 0xFF;
            } else {
                // Codes longer than the LUT (T.81 F.2.2.3): the length is the first
                // l with code_l <= MAXCODE[l]; the six compares use independent
                // loads and selects instead of a dependent loop.
                static_assert(kLutBits == 10, "long-code lengths 11..16");
                const int32_t c11 = static_cast<int32_t>(peek >> 21), c12 = static_cast<int32_t>(peek >> 20);
                const int32_t c13 = static_cast<int32_t>(peek >> 19), c14 = static_cast<int32_t>(peek >> 18);
                const int32_t c15 = static_cast<int32_t>(peek >> 17), c16 = static_cast<int32_t>(peek >> 16);
                const bool p11 = c11 <= t.maxcode[11], p12 = c12 <= t.maxcode[12], p13 = c13 <= t.maxcode[13];
                const bool p14 = c14 <= t.maxcode[14], p15 = c15 <= t.maxcode[15], p16 = c16 <= t.maxcode[16];
                len = p11 ? 11u : p12 ? 12u : p13 ? 13u : p14 ? 14u : p15 ? 15u : 16u;
                const int32_t code = static_cast<int32_t>(peek >> (32 - len));
                sym = t.vals[(code + t.delta[len]) & 255];
                if (!(p11 || p12 || p13 || p14 || p15 || p16)) {
                    flags |= kError;   // consumes 16 bits as a zero symbol
                    sym = 0;
                }
            }
            const uint32_t s = sym & 15;
            const uint32_t r = dc ? 0 : sym >> 4;
            if (dc && sym > 11) flags |= kError;
            int32_t v = 0;
            if (s) {
                const uint32_t bits = (peek << len) >> (32 - s);
                v = bits < (1u << (s - 1)) ? static_cast<int32_t>(bits) - static_cast<int32_t>((1u << s) - 1)
                                           : static_cast<int32_t>(bits);
            }
            pos += len + s;
            if (dc) {
                nblk += 1;
                d0 += comp == 0 ? v : 0;
                d1 += comp == 1 ? v : 0;
                d2 += comp == 2 ? v : 0;
                if (kWrite) {
                    owned = true;
                    p0 += comp == 0 ? v : 0;
                    p1 += comp == 1 ? v : 0;
                    p2 += comp == 2 ? v : 0;
                    // MCU-major destination; on valid data blk % bpm == j.  Blocks past
                    // the frame's count are ignored (as the host decoder stops there).
                    const uint32_t dst = blk - j + (ji >> 8);
                    cur = nullptr;
                    if (blk < out->nblocks) {
                        if (dst < out->nblocks && blk % static_cast<uint32_t>(c.bpm) == j) {
                            cur = out->coefs + static_cast<uint64_t>(dst) * 64;
                            zero_quarter(out->stage);
                            out->stage[0] = static_cast<int16_t>(comp == 0 ? p0 : (comp == 1 ? p1 : p2));
                            quarter = 0;
                        } else {
                            flags |= kError;   // a restart interval ended inside an MCU
                        }
                    }
                }
                z = 1;
            } else if (s == 0) {
                z = r == 15 ? z + 16 : 64;       // ZRL / EOB
            } else {
                z += r;
                if (z > 63) {
                    flags |= kError;
                    z = 64;
                } else {
                    if (kWrite && cur) {
                        const uint32_t qz = z >> 4;
                        if (qz != quarter) {
                            flush_quarters(cur, out->stage, quarter, qz);
                            quarter = qz;
                        }
                        out->stage[z & 15] = static_cast<int16_t>(v);
                    }
                    ++z;
                }
            }
            if (z >= 64) {
                if (kWrite && owned) {
                    if (cur) flush_quarters(cur, out->stage, quarter, 4);   // the rest of the block
                    blk += 1;
                    owned = false;
                    cur = nullptr;
                }
                z = 0;
                j = j + 1 == static_cast<uint32_t>(c.bpm) ? 0 : j + 1;
                ji = jinfo_of(c, j);
            }
        }
        if (!done) result = pack_state(pos, j, z, seg);
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

}  // namespace ent
}  // namespace hjd
