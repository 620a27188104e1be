// jpeg_host.cpp -- host JPEG front end: markers + Huffman decode (include/hjd_host.h).
//
// Produces the fused kernel's input (int16 quantised zigzag coefficients,
// MCU-major) from a baseline JPEG.  Covers the reference's L2/L3
// (src/parser.cpp:7-419, src/decoder.cpp:72-365) with a fresh table-driven
// design: kFastBits first-level lookups per Huffman table (canonical
// MAXCODE/VALPTR search for longer codes, JPEG Annex F.2.2.3), up to two AC
// units per lookup, a de-stuffed copy of the scan read with a branch-free
// refill (a byte-wise reader for the rest), restart-marker resynchronisation,
// two files per thread with interleaved steps, and a thread pool that decodes
// independent files in parallel.
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "hjd.h"
#include "hjd_host.h"
#include "hjd_internal.h"

using hjd_internal::set_error;

namespace {

// first-level lookup width: 11 bits, +10 % per thread over 9 (EPYC 9575F, 4K q90;
// profiles/r05d_host_huffman_lookup_bits_ab.json: 10 and 12 gain less; with the
// two-unit table too, profiles/README.md r05r)
constexpr int kFastBits = 11;
constexpr int kFast = 1 << kFastBits;
constexpr int kMaxBlocksPerMcu = 6;   // 4:2:0 and 4:1:1 (4 luma + 2 chroma)
// fast_ac flag of symbol 0x00 (AC end of block; a zero DC difference), value 0:
// the block's EOB costs one lookup (+1.5 % per thread, profiles/r05e_host_huffman_eob_ab.json)
constexpr int32_t kFastEob = 0x8000;

struct HuffTable {
    bool defined = false;
    uint8_t counts[16];      // the DHT spec, kept for the GPU tables (hjd_entropy.hip)
    int nsym = 0;
    uint16_t fast[kFast];    // (length << 8) | symbol for codes of <= kFastBits bits; 0 = slow path
    // AC: (value << 16) | (run << 5) | (code + extra bits) when those fit kFastBits, else 0
    int32_t fast_ac[kFast];
    // AC tables: up to two units per lookup (build_pairs; the de-stuffed reader's steps)
    uint32_t fast2[kFast];
    int32_t maxcode[18];     // largest code of each length (-1: none)
    int32_t valptr[17];
    int32_t mincode[17];
    uint8_t vals[256];
    // what the arrays above were last built from (counts / vals / nsym) and how:
    // a DHT with the same spec reuses them (build_table)
    bool built = false, built_fast = false, built_ac = false;
};

// A frame's eight Huffman tables (~165 KB with their lookup arrays) live in
// per-thread heap storage, not in Frame on the stack, and stay built across
// files: the config-5 pool repeats one set of tables in every file.  Set 0 and
// 1 hold decode_two's two frames (decode_one uses 0), set 2 the header-only
// parses, so a parse never clobbers the tables of a decode on the same thread.
struct TableSet {
    HuffTable dc[4], ac[4];
};

TableSet& table_set(int i)
{
    thread_local std::unique_ptr<TableSet[]> sets;
    if (!sets) sets.reset(new TableSet[3]);
    return sets[i];
}

struct Component {
    int id = 0, h = 1, v = 1, tq = 0;
    int td = 0, ta = 0;      // DC / AC Huffman table ids (from SOS)
};

// One scan's header (T.81 B.2.3): its components (frame indices) and, for a
// progressive scan, the spectral band ss..se and successive-approximation bits.
struct ScanSpec {
    int ns = 0;
    int comp[3] = {0, 1, 2};
    int ss = 0, se = 63, ah = 0, al = 0;
    size_t offset = 0;       // first byte of the entropy-coded segment
};

struct Frame {
    int width = 0, height = 0, ncomp = 0;
    int process = -1;        // 0 = baseline (SOF0), 1 = extended sequential (SOF1), 2 = progressive (SOF2)
    Component comp[3];
    int32_t qt[4][64] = {};
    int qt_prec[4] = {-1, -1, -1, -1};
    HuffTable* dc;                   // [4] each, in table_set(set)
    HuffTable* ac;
    int restart_interval = 0;
    int scan_order[3] = {0, 1, 2};   // frame component index of each scan component (first scan)
    size_t scan_offset = 0;
    int sampling = -1;
    ScanSpec scan;                   // the scan parse_segments stopped at
    bool decode_tables;              // build the host decoder's lookup tables (false: header parse only)

    // decode: table set 0 or 1; header-only parse (no lookup tables): set 2
    explicit Frame(int set, bool tables = true) : decode_tables(tables)
    {
        TableSet& ts = table_set(tables ? set : 2);
        dc = ts.dc;
        ac = ts.ac;
        for (int i = 0; i < 4; ++i) dc[i].defined = ac[i].defined = false;
    }
    Frame(const Frame&) = delete;
    Frame& operator=(const Frame&) = delete;
};

inline int be16(const uint8_t* p) { return (p[0] << 8) | p[1]; }

// fast = false: the canonical tables only (header parses for the GPU entropy
// path, which builds its own device tables from counts / symbols).
// fast2 entries: bits 0-4 the bits taken (0: not covered), bit 5 the block
// ends after them (an end of block among the units), bits 6-9 the zero run
// before the first coefficient, bits 10-13 the distance from the first
// coefficient to the second (0: one coefficient, written twice), bits 14-22 and
// 23-31 the two values (9-bit signed).  A lookup covers: an end of block; a
// nonzero coefficient; a coefficient and an end of block; or two coefficients
// (second run <= 14) -- whatever of that is complete within the kFastBits
// looked at, with |value| <= 255.
constexpr uint32_t kPairEnd = 1u << 5;

inline uint32_t pair_entry(int bits, bool end, int run1, int dist, int v1, int v2)
{
    return static_cast<uint32_t>(bits) | (end ? kPairEnd : 0) | (static_cast<uint32_t>(run1) << 6) |
           (static_cast<uint32_t>(dist) << 10) | ((static_cast<uint32_t>(v1) & 0x1FF) << 14) |
           ((static_cast<uint32_t>(v2) & 0x1FF) << 23);
}

// One unit at the top of `bits` (kFastBits wide, `avail` of them real): its
// symbol, code length and extended value, if code and value bits fit `avail`.
inline bool unit_at(const HuffTable& t, uint32_t bits, int avail, int& rs, int& used, int& value)
{
    const uint16_t e = t.fast[bits & (kFast - 1)];
    if (!e) return false;
    const int len = e >> 8, size = (e & 0xFF) & 15;
    rs = e & 0xFF;
    if (len + size > avail) return false;
    used = len + size;
    const int v = static_cast<int>((bits >> (kFastBits - used)) & ((1u << size) - 1));
    value = size == 0 ? 0 : v < (1 << (size - 1)) ? v - (1 << size) + 1 : v;
    return true;
}

void build_pairs(HuffTable& t)
{
    for (int idx = 0; idx < kFast; ++idx) {
        uint32_t& out = t.fast2[idx];
        out = 0;
        int rs1, u1, v1;
        if (!unit_at(t, static_cast<uint32_t>(idx), kFastBits, rs1, u1, v1)) continue;
        if (rs1 == 0) {   // end of block
            out = pair_entry(u1, true, 0, 0, 0, 0);
            continue;
        }
        if ((rs1 & 15) == 0 || v1 < -255 || v1 > 255) continue;   // ZRL / wide values: the one-unit path
        const int r1 = rs1 >> 4;
        out = pair_entry(u1, false, r1, 0, v1, v1);
        int rs2, u2, v2;
        const uint32_t rest = (static_cast<uint32_t>(idx) << u1) & (kFast - 1);
        if (!unit_at(t, rest, kFastBits - u1, rs2, u2, v2)) continue;
        if (rs2 == 0) {
            out = pair_entry(u1 + u2, true, r1, 0, v1, v1);
        } else if ((rs2 & 15) != 0 && (rs2 >> 4) <= 14 && v2 >= -255 && v2 <= 255) {
            out = pair_entry(u1 + u2, false, r1, (rs2 >> 4) + 1, v1, v2);
        }
    }
}

int build_table(HuffTable& t, const uint8_t counts[16], const uint8_t* symbols, int nsym, bool fast, bool ac)
{
    if (t.built && t.built_fast == fast && t.built_ac == ac && t.nsym == nsym && memcmp(t.counts, counts, 16) == 0 &&
        memcmp(t.vals, symbols, static_cast<size_t>(nsym)) == 0) {
        t.defined = true;   // the spec these arrays were built from
        return 0;
    }
    t.built = false;
    if (fast) memset(t.fast, 0, sizeof(t.fast));
    memcpy(t.counts, counts, 16);
    t.nsym = nsym;
    int code = 0, k = 0;
    for (int len = 1; len <= 16; ++len) {
        const int n = counts[len - 1];
        t.valptr[len] = k;
        t.mincode[len] = code;
        for (int i = 0; i < n; ++i, ++k, ++code) {
            if (k >= nsym) return -1;
            if (code >= (1 << len)) return -1;   // over-subscribed table
            t.vals[k] = symbols[k];
            if (fast && len <= kFastBits) {
                const int shift = kFastBits - len;
                for (int j = 0; j < (1 << shift); ++j)
                    t.fast[(code << shift) | j] = static_cast<uint16_t>((len << 8) | symbols[k]);
            }
        }
        t.maxcode[len] = n ? code - 1 : -1;
        code <<= 1;
    }
    t.maxcode[17] = 0x7fffffff;
    t.defined = true;
    t.built = true;
    t.built_fast = fast;
    t.built_ac = ac;
    if (!fast) return 0;
    // combined AC entries: symbol and its extra bits in one lookup (nonzero
    // coefficients whose code + magnitude bits fit the kFastBits index)
    memset(t.fast_ac, 0, sizeof(t.fast_ac));
    for (int idx = 0; idx < kFast; ++idx) {
        const uint16_t e = t.fast[idx];
        if (!e) continue;
        const int len = e >> 8, rs = e & 0xFF, run = rs >> 4, size = rs & 15;
        if (rs == 0) {   // EOB (AC) / a zero difference (DC): bit 15 marks it, value 0
            t.fast_ac[idx] = kFastEob | len;
            continue;
        }
        if (size == 0 || len + size > kFastBits) continue;
        const int bits = (idx >> (kFastBits - len - size)) & ((1 << size) - 1);
        const int value = bits < (1 << (size - 1)) ? bits - (1 << size) + 1 : bits;
        t.fast_ac[idx] = static_cast<int32_t>((static_cast<uint32_t>(value) << 16) | (run << 5) | (len + size));
    }
    if (ac) build_pairs(t);
    return 0;
}

int parse_sof(const uint8_t* s, int sl, int marker, Frame& f)
{
    if (f.process >= 0) return set_error(HJD_E_INVALID, "second SOF marker");
    if (sl < 6) return set_error(HJD_E_INVALID, "truncated SOF");
    if (s[0] != 8) return set_error(HJD_E_INVALID, "unsupported bit depth %d", s[0]);
    f.process = marker - 0xC0;
    f.height = be16(s + 1);
    f.width = be16(s + 3);
    f.ncomp = s[5];
    if (f.ncomp != 3 && f.ncomp != 1)
        return set_error(HJD_E_INVALID, "unsupported number of components %d", f.ncomp);
    if (sl < 6 + 3 * f.ncomp) return set_error(HJD_E_INVALID, "truncated SOF");
    if (f.width <= 0 || f.height <= 0) return set_error(HJD_E_INVALID, "invalid dimensions");
    for (int c = 0; c < f.ncomp; ++c) {
        f.comp[c].id = s[6 + 3 * c];
        f.comp[c].h = s[7 + 3 * c] >> 4;
        f.comp[c].v = s[7 + 3 * c] & 15;
        f.comp[c].tq = s[8 + 3 * c];
        if (f.comp[c].tq > 3) return set_error(HJD_E_INVALID, "bad quantisation table id");
        if (f.comp[c].h < 1 || f.comp[c].h > 4 || f.comp[c].v < 1 || f.comp[c].v > 4)
            return set_error(HJD_E_INVALID, "bad sampling factors");
    }
    // src/decoder.cpp:58-69 accepts H2V2/H1V1/H1V1 and all-H1V1; H2V1/H1V1/H1V1
    // (4:2:2) and one component (gray) are this library's extensions
    // (SURVEY.md s8(f) rank 4).  A one-component scan is non-interleaved:
    // its MCU is one block whatever the sampling factors (T.81 A.2.2).
    const Component* c = f.comp;
    const bool chroma11 = f.ncomp == 3 && c[1].h == 1 && c[1].v == 1 && c[2].h == 1 && c[2].v == 1;
    if (f.ncomp == 1)
        f.sampling = HJD_GRAY;
    else if (chroma11 && c[0].h == 2 && c[0].v == 2)
        f.sampling = HJD_YUV420;
    else if (chroma11 && c[0].h == 1 && c[0].v == 1)
        f.sampling = HJD_YUV444;
    else if (chroma11 && c[0].h == 2 && c[0].v == 1)
        f.sampling = HJD_YUV422;
    else if (chroma11 && c[0].h == 4 && c[0].v == 1)
        f.sampling = HJD_YUV411_H4V1;
    else if (chroma11 && c[0].h == 1 && c[0].v == 2)
        f.sampling = HJD_YUV440;
    else
        return set_error(HJD_E_INVALID, "unsupported sampling (4:2:0, 4:4:4, 4:2:2, 4:1:1, 4:4:0 or gray)");
    return HJD_OK;
}

// SOS (src/parser.cpp:132-154; T.81 B.2.3).  The reference takes one scan
// holding every component; sequential files with several scans (one or two
// components each) and progressive scans (G.1.1.1.1 band rules) are this
// library's extensions.
int parse_sos(const uint8_t* s, int sl, Frame& f, ScanSpec& sc)
{
    if (f.process < 0) return set_error(HJD_E_INVALID, "SOS before SOF");
    if (sl < 1) return set_error(HJD_E_INVALID, "truncated SOS");
    const int ns = s[0];
    if (ns < 1 || ns > f.ncomp || sl < 1 + 2 * ns + 3) return set_error(HJD_E_INVALID, "bad SOS component count");
    sc.ns = ns;
    for (int i = 0; i < ns; ++i) {
        const int cid = s[1 + 2 * i], tdta = s[2 + 2 * i];
        int fc = -1;
        for (int c = 0; c < f.ncomp; ++c)
            if (f.comp[c].id == cid) fc = c;
        if (fc < 0) return set_error(HJD_E_INVALID, "scan component %d not in frame", cid);
        for (int j = 0; j < i; ++j)
            if (sc.comp[j] == fc) return set_error(HJD_E_INVALID, "component %d twice in one scan", cid);
        sc.comp[i] = fc;
        f.comp[fc].td = tdta >> 4;
        f.comp[fc].ta = tdta & 15;
        if (f.comp[fc].td > 3 || f.comp[fc].ta > 3) return set_error(HJD_E_INVALID, "bad Huffman table id");
    }
    const uint8_t* tail = s + 1 + 2 * ns;
    sc.ss = tail[0];
    sc.se = tail[1];
    sc.ah = tail[2] >> 4;
    sc.al = tail[2] & 15;
    const bool prog = f.process == 2;
    if (!prog) {
        if (sc.ss != 0 || sc.se != 63 || sc.ah != 0 || sc.al != 0)
            return set_error(HJD_E_INVALID, "not a sequential scan (Ss/Se/Ah/Al)");
    } else {
        const bool dc = sc.ss == 0;
        if ((dc && sc.se != 0) || (!dc && (sc.se < sc.ss || sc.se > 63 || ns != 1)) || sc.al > 13 ||
            (sc.ah != 0 && sc.ah != sc.al + 1))
            return set_error(HJD_E_INVALID, "bad progressive scan (Ss=%d Se=%d Ah=%d Al=%d Ns=%d)", sc.ss, sc.se,
                             sc.ah, sc.al, ns);
    }
    for (int i = 0; i < ns; ++i) {
        const Component& c = f.comp[sc.comp[i]];
        if (f.qt_prec[c.tq] < 0) return set_error(HJD_E_INVALID, "missing quantisation table");
        const bool need_dc = sc.ss == 0 && sc.ah == 0, need_ac = sc.se > 0;
        if (need_dc && !f.dc[c.td].defined) return set_error(HJD_E_INVALID, "missing DC Huffman table");
        if (need_ac && !f.ac[c.ta].defined) return set_error(HJD_E_INVALID, "missing AC Huffman table");
    }
    return HJD_OK;
}

// Marker segments from d[p] up to the next SOS (returns HJD_OK with f.scan set
// and *p past the SOS) or, after the first scan, EOI / end of data (*eoi).
int parse_segments(const uint8_t* d, size_t n, size_t* pp, Frame& f, bool after_scan, bool* eoi)
{
    size_t p = *pp;
    *eoi = false;
    for (;;) {
        while (p < n && d[p] != 0xFF) ++p;           // tolerate garbage between segments
        while (p < n && d[p] == 0xFF) ++p;           // fill bytes
        if (p >= n) {
            if (after_scan) { *eoi = true; return HJD_OK; }   // missing EOI: take what was decoded
            return set_error(HJD_E_INVALID, "no SOS marker");
        }
        const uint8_t m = d[p++];
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;   // no length
        if (m == 0xD9) {
            if (after_scan) { *eoi = true; *pp = p; return HJD_OK; }
            return set_error(HJD_E_INVALID, "EOI before SOS");
        }
        if (p + 2 > n) return set_error(HJD_E_INVALID, "truncated marker segment");
        const int len = be16(d + p);
        if (len < 2 || p + len > n) return set_error(HJD_E_INVALID, "bad segment length");
        const uint8_t* s = d + p + 2;
        const int sl = len - 2;
        switch (m) {
        case 0xDB: {   // DQT (src/parser.cpp:47-100; 16-bit entries big-endian per T.81 B.2.4.1)
            int q = 0;
            while (q < sl) {
                const int pq = s[q] >> 4, tq = s[q] & 15;
                if (pq > 1 || tq > 3) return set_error(HJD_E_INVALID, "bad DQT table %d precision %d", tq, pq);
                if (q + 1 + 64 * (pq + 1) > sl) return set_error(HJD_E_INVALID, "truncated DQT");
                for (int i = 0; i < 64; ++i)
                    f.qt[tq][i] = pq ? be16(s + q + 1 + 2 * i) : s[q + 1 + i];
                f.qt_prec[tq] = pq;
                q += 1 + 64 * (pq + 1);
            }
            break;
        }
        case 0xC0: case 0xC1: case 0xC2: {   // SOF0 (src/parser.cpp:102-130); SOF1/SOF2: extensions
            const int rc = parse_sof(s, sl, m, f);
            if (rc) return rc;
            break;
        }
        case 0xC3: case 0xC5: case 0xC6: case 0xC7:
        case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
            return set_error(HJD_E_INVALID, "only Huffman-coded sequential or progressive JPEG is supported");
        case 0xC4: {   // DHT (src/parser.cpp:170-270)
            int q = 0;
            while (q < sl) {
                if (q + 17 > sl) return set_error(HJD_E_INVALID, "truncated DHT");
                const int tc = s[q] >> 4, th = s[q] & 15;
                if (tc > 1 || th > 3) return set_error(HJD_E_INVALID, "bad DHT class/id");
                int nsym = 0;
                for (int i = 0; i < 16; ++i) nsym += s[q + 1 + i];
                if (nsym > 256 || q + 17 + nsym > sl) return set_error(HJD_E_INVALID, "bad DHT size");
                HuffTable& t = tc ? f.ac[th] : f.dc[th];
                if (build_table(t, s + q + 1, s + q + 17, nsym, f.decode_tables, tc == 1))
                    return set_error(HJD_E_INVALID, "invalid Huffman table");
                q += 17 + nsym;
            }
            break;
        }
        case 0xDD:     // DRI (src/parser.cpp:156-168)
            if (sl < 2) return set_error(HJD_E_INVALID, "truncated DRI");
            f.restart_interval = be16(s);
            break;
        case 0xDA: {   // SOS
            const int rc = parse_sos(s, sl, f, f.scan);
            if (rc) return rc;
            f.scan.offset = p + len;
            *pp = p + len;
            return HJD_OK;
        }
        default:       // APPn, COM, DNL, ...: skip (src/parser.cpp:295-322 skips APPn)
            break;
        }
        p += len;
    }
}

// Headers up to the first SOS.
int parse(const uint8_t* d, size_t n, Frame& f)
{
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) return set_error(HJD_E_INVALID, "SOI missing");
    size_t p = 2;
    bool eoi = false;
    const int rc = parse_segments(d, n, &p, f, false, &eoi);
    if (rc) return rc;
    for (int i = 0; i < f.scan.ns; ++i) f.scan_order[i] = f.scan.comp[i];
    f.scan_offset = f.scan.offset;
    return HJD_OK;
}

// One interleaved sequential scan holds the whole image: the reference's
// case (src/decoder.cpp:308-344) and the GPU entropy decoder's.
inline bool single_scan(const Frame& f) { return f.process != 2 && f.scan.ns == f.ncomp; }

void fill_info(const Frame& f, hjd_jpeg_info* info)
{
    memset(info, 0, sizeof(*info));
    info->width = f.width;
    info->height = f.height;
    info->sampling = f.sampling;
    info->restart_interval = f.restart_interval;
    hjd_internal::SamplingGeom g;
    hjd_internal::sampling_geom(f.sampling, &g);   // parse() admitted only known samplings
    info->mcu_w = (f.width - 1) / g.mcu_px_w + 1;
    info->mcu_h = (f.height - 1) / g.mcu_px_h + 1;
    info->nblocks = static_cast<int64_t>(info->mcu_w) * info->mcu_h * g.bpm;
    for (int c = 0; c < 3; ++c) {   // gray: the Y table for all three (only Y is used)
        const int fc = c < f.ncomp ? c : 0;
        memcpy(info->qt[c], f.qt[f.comp[fc].tq], sizeof(info->qt[c]));
        info->qt_precision[c] = f.qt_prec[f.comp[fc].tq];
    }
    info->scan_offset = static_cast<int64_t>(f.scan_offset);
    info->process = f.process;
    info->single_scan = single_scan(f) ? 1 : 0;
}

// Entropy-coded segment reader: 64-bit MSB-first accumulator, FF00 de-stuffing,
// fill bytes (FF FF) skipped as the reference's read_more_data does
// (src/decoder.cpp:94-159), stops feeding (zeros) at the first marker.
struct BitReader {
    const uint8_t* p;
    const uint8_t* end;
    uint64_t acc = 0;
    int nbits = 0;
    bool at_marker = false;
    int64_t virt = 0;   // zero bits fed past the marker / the end of the data

    void refill()
    {
        // fast path: the next 8 bytes hold no 0xFF (no stuffing, no marker) --
        // take as many whole bytes as fit in one big-endian load
        if (!at_marker && end - p >= 8) {
            uint64_t v;
            memcpy(&v, p, 8);
            const uint64_t inv = ~v;   // a 0xFF byte of v is a zero byte of inv
            if (((inv - 0x0101010101010101ull) & ~inv & 0x8080808080808080ull) == 0) {
                const int take = (63 - nbits) >> 3;   // bytes that fit (nbits < 64 after)
                acc |= (__builtin_bswap64(v) >> nbits) & ~(~0ull >> (nbits + 8 * take));
                p += take;
                nbits += 8 * take;
                return;
            }
        }
        while (nbits <= 56) {
            uint64_t b = 0;
            bool real = false;
            if (!at_marker && p < end) {
                if (p[0] != 0xFF) {
                    b = *p++;
                    real = true;
                } else if (p + 1 < end && p[1] == 0x00) {
                    b = 0xFF;
                    p += 2;
                    real = true;
                } else if (p + 1 < end && p[1] == 0xFF) {
                    ++p;                // a fill byte: the pair starts at the next 0xFF
                    continue;           // (src/decoder.cpp:121-134, FF FF -> look at the next byte)
                } else {
                    at_marker = true;   // leave p on the marker
                }
            }
            acc |= b << (56 - nbits);
            nbits += 8;
            if (!real) virt += 8;
        }
    }
    // The decode took bits past the data (the zeros fed after it): the
    // reference's cacheEof (src/bitstream.h:322-331), checked as it does
    // before every component after the first (src/decoder.cpp:310-314).
    bool overrun() const { return virt > nbits; }
    uint32_t peek(int n) const { return static_cast<uint32_t>(acc >> (64 - n)); }
    void skip(int n) { acc <<= n; nbits -= n; }

    // Restart: drop buffered bits, expect RSTn at the next marker.  The
    // reference aligns to the next byte and reads it as the marker
    // (src/decoder.cpp:295-302), so a whole byte of the interval left
    // undecoded (or a decode past the interval's data) fails here too.
    bool restart(int expect)
    {
        bool spare = nbits - virt >= 8 || virt > nbits;
        acc = 0;
        nbits = 0;
        virt = 0;
        if (!at_marker) {
            const uint8_t* q = p;
            while (p + 1 < end && !(p[0] == 0xFF && p[1] != 0x00)) ++p;
            spare |= p != q;
        }
        if (spare) return false;
        while (p < end && p[0] == 0xFF) ++p;   // marker prefix + fill bytes
        if (p >= end || *p != 0xD0 + (expect & 7)) return false;
        ++p;
        at_marker = false;
        return true;
    }
};

inline int decode_symbol(BitReader& br, const HuffTable& t)
{
    if (br.nbits < 16) br.refill();
    const uint16_t e = t.fast[br.peek(kFastBits)];
    if (e) {
        br.skip(e >> 8);
        return e & 0xFF;
    }
    const uint32_t code16 = br.peek(16);
    for (int len = kFastBits + 1; len <= 16; ++len) {
        const int32_t c = static_cast<int32_t>(code16 >> (16 - len));
        if (c <= t.maxcode[len]) {
            br.skip(len);
            return t.vals[t.valptr[len] + c - t.mincode[len]];
        }
    }
    return -1;
}

// receive + extend (T.81 F.2.2.1; src/decoder.cpp:72-92)
inline int receive_extend(BitReader& br, int s)
{
    if (s == 0) return 0;
    if (br.nbits < s) br.refill();
    const int v = static_cast<int>(br.peek(s));
    br.skip(s);
    return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
}

// One block (src/decoder.cpp:221-260).
inline bool decode_block(BitReader& br, const HuffTable& dc, const HuffTable& ac, int& pred, int16_t* out)
{
    if (br.nbits < 16) br.refill();
    const int32_t fd = dc.fast_ac[br.peek(kFastBits)];   // a DC table's symbols are sizes: run 0
    if (fd) {
        br.skip(fd & 31);
        pred += fd >> 16;
    } else {
        const int s = decode_symbol(br, dc);
        if (s < 0 || s > 11) return false;
        pred += receive_extend(br, s);
    }
    if (pred < -32768 || pred > 32767) return false;
    memset(out, 0, 64 * sizeof(int16_t));
    out[0] = static_cast<int16_t>(pred);
    for (int k = 1; k < 64;) {
        if (br.nbits < 16) br.refill();
        const int32_t fe = ac.fast_ac[br.peek(kFastBits)];
        if (fe) {   // run + nonzero coefficient in one lookup
            br.skip(fe & 31);
            if (fe & kFastEob) break;
            k += (fe >> 5) & 15;
            if (k > 63) return false;
            out[k++] = static_cast<int16_t>(fe >> 16);
            continue;
        }
        const int rs = decode_symbol(br, ac);
        if (rs < 0) return false;
        const int r = rs >> 4, sz = rs & 15;
        if (sz == 0) {
            if (r != 15) break;   // EOB
            k += 16;              // ZRL; one past index 63 is corrupt (the reference
            if (k > 64) return false;   // asserts count + 1 <= 64, src/decoder.cpp:244-245)
            continue;
        }
        k += r;
        if (k > 63) return false;
        out[k++] = static_cast<int16_t>(receive_extend(br, sz));
    }
    return true;
}

// The scan's data ended inside MCU m: the reference's "data incomplete"
// (src/decoder.cpp:310-313; load_jpg then stops, src/parser.cpp:384-388).
// One stricter case: the reference checks before each component but not after
// the last one, so a file cut inside the last MCU's last component decodes
// there from whatever its buffer holds past the data; this decoder rejects it.
__attribute__((noinline, cold)) int report_incomplete(int64_t m, int64_t nmcu)
{
    return set_error(HJD_E_INVALID, "entropy data incomplete or truncated (MCU %lld of %lld)",
                     static_cast<long long>(m), static_cast<long long>(nmcu));
}

int decode_scan_bytewise(const uint8_t* d, size_t n, const Frame& f, const hjd_jpeg_info& info, int16_t* coefs)
{
    BitReader br{d + f.scan_offset, d + n};
    int pred[3] = {0, 0, 0};
    // blocks per MCU of each component (gray: one block, non-interleaved scan)
    const int nblk_c[3] = {f.ncomp == 1 ? 1 : f.comp[0].h * f.comp[0].v, 1, 1};
    int blk_base[3];   // block offset of each frame component inside an MCU
    blk_base[0] = 0;
    blk_base[1] = nblk_c[0];
    blk_base[2] = nblk_c[0] + 1;
    const int bpm = f.ncomp == 1 ? 1 : nblk_c[0] + 2;
    const int64_t nmcu = static_cast<int64_t>(info.mcu_w) * info.mcu_h;
    int restarts = 0, since = 0;
    for (int64_t m = 0; m < nmcu; ++m) {
        if (br.overrun()) return report_incomplete(m - 1, nmcu);
        if (f.restart_interval > 0 && since == f.restart_interval) {   // src/decoder.cpp:288-307
            if (!br.restart(restarts)) return set_error(HJD_E_INVALID, "expected RST%d before MCU %lld", restarts & 7,
                                                      static_cast<long long>(m));
            ++restarts;
            since = 0;
            pred[0] = pred[1] = pred[2] = 0;
        }
        ++since;
        int16_t* mcu = coefs + m * bpm * 64;
        for (int si = 0; si < f.ncomp; ++si) {
            const int c = f.scan_order[si];
            const HuffTable& dc = f.dc[f.comp[c].td];
            const HuffTable& ac = f.ac[f.comp[c].ta];
            for (int b = 0; b < nblk_c[c]; ++b)
                if (!decode_block(br, dc, ac, pred[c], mcu + (blk_base[c] + b) * 64))
                    return set_error(HJD_E_INVALID, "corrupt entropy data in MCU %lld", static_cast<long long>(m));
        }
    }
    return br.overrun() ? report_incomplete(nmcu - 1, nmcu) : HJD_OK;
}

// ---- the de-stuffed reader (the single-scan hot path) ----------------------
// BitReader pays a data-dependent branch per symbol (refill when fewer than
// 16 bits are left) and a byte loop at every 0xFF.  The hot path instead
// copies the scan's entropy-coded data once without its byte stuffing
// (copy_until_ff, a few % of the decode) into per-thread scratch, one segment
// per restart interval, each followed by kSegPad zero bytes, and then reads it
// with a branch-free refill: a 64-bit load at the byte cursor, shifted under
// the bits still buffered (the cursor moves by the whole bytes taken, so the
// reader sees zeros past the data, as BitReader does past a marker, and
// stops kSegPad - 8 bytes past it).  A refill leaves at least 56 bits, which
// is what lets FastDec run three symbol steps per refill (the bit budget is at
// FastDec::step).
//
// Reading past the data: while the cursor has not hit its stop, the bits taken
// are exact (8 x bytes moved - bits buffered), and a cursor that moved more
// than 8 bytes past the data means more bits were taken than buffered there;
// so FastReader::left() < 0 exactly when the decode consumed bits past the
// segment's data, the stop included (16 bytes past: left() <= 63 - 128).  The
// check runs where an interval ends (the restart) and after the last MCU
// (FastDec::report), none on the step path: a decode that runs out of data
// goes on over zeros to the segment's end, is then rejected, and the
// byte-wise reader re-runs it for the exact MCU of the error.
//
// The bits a decode sees are the BitReader's exactly: de-stuffed FF00, fill
// bytes in front of a marker dropped, zeros after the marker or the end of
// the data, and a restart moves to the next segment when the marker that ended
// the current one is the expected RSTn.  The one difference would be fill
// bytes INSIDE the data (FF FF 00: BitReader reads the FF00 after the fill
// byte, its restart search stops at the FF FF): destuff_scan declines such a
// scan and it takes the byte-wise path.  tests/test_jpeg_host_pair.py and the
// fuzz harness (tools/fuzz/host_decode_fuzz.cpp) compare the two readers.
constexpr size_t kSegPad = 24;   // zero bytes after each segment: the cursor stops 16 past the data

struct CleanSeg {
    size_t begin, end;   // bytes of CleanScan::buf; kSegPad zero bytes follow `end`
    int marker;          // the marker byte that ended the segment; -1: the data ended
};

struct CleanScan {
    std::unique_ptr<uint8_t[]> buf;
    size_t cap = 0;
    std::vector<CleanSeg> segs;
};

// De-stuff the entropy-coded data from s into cs: max_segs segments at most
// (the scan's restart intervals), stopping at a marker that is not RSTn.
// false: fill bytes inside the data (the byte-wise reader's case).
bool destuff_scan(const uint8_t* s, const uint8_t* end, int64_t max_segs, CleanScan& cs)
{
    const size_t n = static_cast<size_t>(end - s);
    max_segs = std::max<int64_t>(1, std::min<int64_t>(max_segs, static_cast<int64_t>(n / 2) + 1));
    // + 64: copy_until_ff stores whole 64-byte vectors while that many fit
    const size_t need = n + kSegPad * static_cast<size_t>(max_segs) + kSegPad + 64;
    if (cs.cap < need) {
        cs.buf.reset(new uint8_t[need]);
        cs.cap = need;
    }
    cs.segs.clear();
    uint8_t* const o0 = cs.buf.get();
    uint8_t* o = o0;
    size_t begin = 0;
    uint8_t* const oend = o0 + cs.cap;
    for (;;) {
        s = hjd_internal::copy_until_ff(s, end, o, oend);
        const uint8_t* f = s < end ? s : nullptr;   // at an 0xFF (the scratch always has room)
        int marker = -1;
        if (f) {
            if (f + 1 < end && f[1] == 0x00) {   // stuffed FF
                *o++ = 0xFF;
                s = f + 2;
                continue;
            }
            const uint8_t* g = f;
            while (g < end && *g == 0xFF) ++g;   // marker prefix and fill bytes
            if (g < end && *g == 0x00) return false;
            if (g < end) marker = *g;
            s = g < end ? g + 1 : end;
        }
        const size_t seg_end = static_cast<size_t>(o - o0);
        memset(o, 0, kSegPad);
        o += kSegPad;
        cs.segs.push_back({begin, seg_end, marker});
        begin = static_cast<size_t>(o - o0);
        if (marker < 0xD0 || marker > 0xD7 || static_cast<int64_t>(cs.segs.size()) == max_segs) return true;
    }
}

struct FastReader {
    const uint8_t* p;
    const uint8_t* stop;   // the cursor's limit: the segment's end + kSegPad - 8
    uint64_t acc = 0;      // MSB-first; bits below the top nbits are zeros or the stream's next bits
    int nbits = 0;

    void seek(const CleanScan& cs, const CleanSeg& s)
    {
        p = cs.buf.get() + s.begin;
        stop = cs.buf.get() + s.end + (kSegPad - 8);
        acc = 0;
        nbits = 0;
    }
    __attribute__((always_inline)) void refill()
    {
        uint64_t v;
        memcpy(&v, p, 8);
        acc |= __builtin_bswap64(v) >> nbits;
        p += (63 - nbits) >> 3;
        p = p < stop ? p : stop;
        nbits |= 56;
    }
    // bits of the segment's data not taken yet; < 0: the decode took bits
    // past its data (exact in sign, see above)
    int64_t left() const { return 8 * (stop - static_cast<std::ptrdiff_t>(kSegPad - 8) - p) + nbits; }
    uint32_t peek(int n) const { return static_cast<uint32_t>(acc >> (64 - n)); }
    void skip(int n)
    {
        acc <<= n;
        nbits -= n;
    }
};

// decode_symbol without the refill (the step refilled: >= 56 bits)
__attribute__((always_inline)) inline int fast_symbol(FastReader& br, const HuffTable& t)
{
    const uint16_t e = t.fast[br.peek(kFastBits)];
    if (e) {
        br.skip(e >> 8);
        return e & 0xFF;
    }
    const uint32_t code16 = br.peek(16);
    for (int len = kFastBits + 1; len <= 16; ++len) {
        const int32_t c = static_cast<int32_t>(code16 >> (16 - len));
        if (c <= t.maxcode[len]) {
            br.skip(len);
            return t.vals[t.valptr[len] + c - t.mincode[len]];
        }
    }
    return -1;
}

__attribute__((always_inline)) inline int fast_extend(FastReader& br, int s)
{
    if (s == 0) return 0;
    const int v = static_cast<int>(br.peek(s));
    br.skip(s);
    return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v;
}

__attribute__((noinline, cold)) int report_error(int err, int64_t m, int64_t nmcu, int restarts)
{
    if (err == 1) return set_error(HJD_E_INVALID, "corrupt entropy data in MCU %lld", static_cast<long long>(m));
    if (err == 2)
        return set_error(HJD_E_INVALID, "expected RST%d before MCU %lld", restarts & 7, static_cast<long long>(m));
    if (err == 3) return report_incomplete(m - 1, nmcu);
    return HJD_OK;
}

// A file's block order and DC predictors (kept apart from FastDec, whose
// scalars then stay in registers: no dynamically indexed member).
struct BlockOrder {
    const HuffTable* dc[kMaxBlocksPerMcu];
    const HuffTable* ac[kMaxBlocksPerMcu];
    int comp[kMaxBlocksPerMcu], slot[kMaxBlocksPerMcu];
    int pred[3] = {0, 0, 0};
};

// decode_scan_bytewise restated as a one-unit step on the de-stuffed reader,
// with the same checks, errors and output.  Errors are recorded and reported
// (set_error) after the loop, so nothing on the step path calls out.  A block's DC
// difference is decoded when the block begins (after a refill), so a step is
// one AC unit of the current block's table.
struct FastDec {
    FastReader br;
    const CleanScan* cs = nullptr;
    BlockOrder* o = nullptr;
    const HuffTable* act = nullptr;   // the current block's AC table
    size_t seg = 0;
    int bpm = 0, bi = 0, k = 0;
    int64_t nmcu = 0, m = 0;
    int16_t* out = nullptr;
    int16_t* coefs = nullptr;
    int ri = 0, since = 0, restarts = 0;
    bool done = false;
    int err = 0;   // 1: corrupt entropy data in MCU m, 2: expected RSTn before MCU m, 3: data ended in MCU m-1

    __attribute__((always_inline)) void init(const CleanScan& c, BlockOrder& ord, const Frame& f,
                                             const hjd_jpeg_info& info, int16_t* co)
    {
        cs = &c;
        o = &ord;
        br.seek(c, c.segs[0]);
        const int nblk0 = f.ncomp == 1 ? 1 : f.comp[0].h * f.comp[0].v;   // as decode_scan_bytewise
        bpm = f.ncomp == 1 ? 1 : nblk0 + 2;
        int j = 0;
        for (int si = 0; si < f.ncomp; ++si) {
            const int cc = f.scan_order[si];
            const int nb = cc == 0 ? nblk0 : 1;
            const int base = cc == 0 ? 0 : cc == 1 ? nblk0 : nblk0 + 1;
            for (int b = 0; b < nb; ++b, ++j) {
                ord.dc[j] = &f.dc[f.comp[cc].td];
                ord.ac[j] = &f.ac[f.comp[cc].ta];
                ord.comp[j] = cc;
                ord.slot[j] = base + b;
            }
        }
        nmcu = static_cast<int64_t>(info.mcu_w) * info.mcu_h;
        ri = f.restart_interval;
        coefs = co;
        done = nmcu == 0;
        if (!done) begin_mcu();
    }
    // After the decode: the last segment's end check (the data ran out before
    // the last MCU's end) is made here, off the step path.
    __attribute__((always_inline)) int report() const
    {
        return report_error(err == 0 && br.left() < 0 ? 3 : err, m, nmcu, restarts);
    }
    __attribute__((always_inline)) void fail(int e)
    {
        err = e;
        done = true;
    }
    // zero the block and decode its DC difference (refilled: >= 56 bits, a DC
    // symbol takes at most 27, so >= 29 remain for the step schedule)
    __attribute__((always_inline)) void begin_block()
    {
        out = coefs + (m * bpm + o->slot[bi]) * 64;
        memset(out, 0, 64 * sizeof(int16_t));
        act = o->ac[bi];
        br.refill();
        int& p = o->pred[o->comp[bi]];
        const HuffTable& dc = *o->dc[bi];
        const int32_t fd = dc.fast_ac[br.peek(kFastBits)];
        if (fd) {
            br.skip(fd & 31);
            p += fd >> 16;
        } else {
            const int sz = fast_symbol(br, dc);
            if (sz < 0 || sz > 11) return fail(1);
            p += fast_extend(br, sz);
        }
        if (p < -32768 || p > 32767) return fail(1);
        out[0] = static_cast<int16_t>(p);
        k = 1;
    }
    __attribute__((always_inline)) void begin_mcu()   // src/decoder.cpp:288-314
    {
        if (ri > 0 && since == ri) {
            // the interval's data ran out (BitReader::overrun); the reference
            // reads the byte after the interval's last bits as the marker
            // (src/decoder.cpp:295-302), so a whole byte left is a mismatch
            const CleanSeg& s = cs->segs[seg];
            if (br.left() < 0) return fail(3);
            if (s.marker != 0xD0 + (restarts & 7) || seg + 1 >= cs->segs.size() || br.left() >= 8) return fail(2);
            br.seek(*cs, cs->segs[++seg]);
            ++restarts;
            since = 0;
            o->pred[0] = o->pred[1] = o->pred[2] = 0;
        }
        ++since;
        bi = 0;
        begin_block();
    }
    __attribute__((always_inline)) void end_block()
    {
        if (++bi < bpm) return begin_block();
        if (++m == nmcu) {
            done = true;   // report() checks the last segment's end
            return;
        }
        begin_mcu();
    }
    // One AC unit.  Needs kFastBits buffered bits; a one-lookup unit takes at
    // most kFastBits, a slow unit refills first (>= 56 bits) and takes at most
    // 31 (16-bit code + 15 extra bits), and a unit that ends the block leaves
    // >= 29 (begin_block).  So three steps per refill never run short:
    // 56 -> 45 -> 34 fast, or >= 25 after a refilled step -> >= 14.
    __attribute__((always_inline)) void step()
    {
        const uint32_t idx = br.peek(kFastBits);
        const uint32_t e2 = act->fast2[idx];
        const int p1 = k + static_cast<int>((e2 >> 6) & 15);
        const int p2 = p1 + static_cast<int>((e2 >> 10) & 15);
        if (e2 && p2 < 63) {   // up to two units in one lookup, not the block's last position
            br.skip(static_cast<int>(e2 & 31));
            out[p1] = static_cast<int16_t>(static_cast<int32_t>(e2 << 9) >> 23);
            out[p2] = static_cast<int16_t>(static_cast<int32_t>(e2) >> 23);
            k = p2 + 1;
            if (e2 & kPairEnd) end_block();
            return;
        }
        // one unit (near position 63, where a second unit may belong to the next block)
        const int32_t fe = act->fast_ac[idx];
        if (fe) {
            br.skip(fe & 31);
            if (fe & kFastEob) return end_block();
            k += (fe >> 5) & 15;
            if (k > 63) return fail(1);
            out[k++] = static_cast<int16_t>(fe >> 16);
            if (k == 64) end_block();
            return;
        }
        br.refill();
        const int rs = fast_symbol(br, *act);
        if (rs < 0) return fail(1);
        const int r = rs >> 4, sz = rs & 15;
        if (sz == 0) {
            if (r != 15) return end_block();   // EOB
            k += 16;                            // ZRL: to 64 ends the block, past it is corrupt (decode_block)
            if (k > 64) return fail(1);
            if (k == 64) end_block();
            return;
        }
        k += r;
        if (k > 63) return fail(1);
        out[k++] = static_cast<int16_t>(fast_extend(br, sz));
        if (k == 64) end_block();
    }
    // the rest of the file: three steps per refill
    __attribute__((always_inline)) void finish()
    {
        while (!done) {
            br.refill();
            step();
            if (done) break;
            step();
            if (done) break;
            step();
        }
    }
};

// The reader of single-scan decodes: 0 the de-stuffed reader where the scan
// admits it, 1 the byte-wise reader always (hjd_debug_host_reader: tests).
std::atomic<int> g_host_reader{0};

// Scratch of the de-stuffed reader, two per thread (the pair decode).  A
// buffer grows to the largest scan its thread has de-stuffed (a 4K q90 scan:
// a few MB) and stays for the next file; one past kScratchKeep (an outlier
// scan) is released after its decode, so a long-lived worker holds at most
// 2 x kScratchKeep.
constexpr size_t kScratchKeep = size_t{32} << 20;

CleanScan& clean_scratch(int i)
{
    thread_local CleanScan cs[2];
    return cs[i];
}

void trim_scratch(CleanScan& cs)
{
    if (cs.cap <= kScratchKeep) return;
    cs.buf.reset();
    cs.cap = 0;
    std::vector<CleanSeg>().swap(cs.segs);
}

int64_t scan_segments(const Frame& f, const hjd_jpeg_info& info)
{
    const int64_t nmcu = static_cast<int64_t>(info.mcu_w) * info.mcu_h;
    return f.restart_interval > 0 ? (nmcu + f.restart_interval - 1) / f.restart_interval : 1;
}

bool destuff_for(const uint8_t* d, size_t n, const Frame& f, const hjd_jpeg_info& info, CleanScan& cs)
{
    return g_host_reader.load(std::memory_order_relaxed) == 0 && f.scan_offset <= n &&
           destuff_scan(d + f.scan_offset, d + n, scan_segments(f, info), cs);
}

// One single-scan sequential file (src/decoder.cpp:262-358), de-stuffed into cs.
int decode_clean(const CleanScan& cs, const Frame& f, const hjd_jpeg_info& info, int16_t* coefs)
{
    BlockOrder oa;
    FastDec a;
    a.init(cs, oa, f, info, coefs);
    a.finish();
    return a.report();
}

// A file the de-stuffed reader rejected, decoded again by the byte-wise
// reader, whose checks run per MCU: its error names the MCU where the data
// ran out (or the first corrupt one), where the de-stuffed reader only
// notices at the interval's end.  Errors are rare; the re-run costs one decode.
__attribute__((noinline, cold)) int exact_error(const uint8_t* d, size_t n, const Frame& f,
                                                 const hjd_jpeg_info& info, int16_t* coefs, int rc)
{
    const int rb = decode_scan_bytewise(d, n, f, info, coefs);
    return rb != HJD_OK ? rb : rc;
}

int decode_scan(const uint8_t* d, size_t n, const Frame& f, const hjd_jpeg_info& info, int16_t* coefs)
{
    CleanScan& cs = clean_scratch(0);
    int rc;
    if (destuff_for(d, n, f, info, cs)) {
        rc = decode_clean(cs, f, info, coefs);
        if (rc != HJD_OK) rc = exact_error(d, n, f, info, coefs, rc);
    } else {
        rc = decode_scan_bytewise(d, n, f, info, coefs);
    }
    trim_scratch(cs);
    return rc;
}

// Two single-scan sequential files on one thread, their steps interleaved: a
// decode is one dependent chain (peek -> table load -> shift), so two files
// keep two chains in flight (+10 % per thread when introduced,
// profiles/r05i_host_huffman_two_stream_probe.txt).  rc[i] as decode_scan
// returns (errors recorded in the order they occurred); a file the de-stuffed
// reader declines is decoded alone, as decode_scan does.
void decode_scan_pair(const uint8_t* const d[2], const size_t n[2], const Frame* const f[2],
                      const hjd_jpeg_info* const info[2], int16_t* const coefs[2], int rc[2])
{
    CleanScan& c0 = clean_scratch(0);
    CleanScan& c1 = clean_scratch(1);
    const bool ok0 = destuff_for(d[0], n[0], *f[0], *info[0], c0);
    const bool ok1 = destuff_for(d[1], n[1], *f[1], *info[1], c1);
    if (!ok0 || !ok1) {
        for (int i = 0; i < 2; ++i) {
            if (i ? ok1 : ok0) {
                rc[i] = decode_clean(i ? c1 : c0, *f[i], *info[i], coefs[i]);
                if (rc[i] != HJD_OK) rc[i] = exact_error(d[i], n[i], *f[i], *info[i], coefs[i], rc[i]);
            } else {
                rc[i] = decode_scan_bytewise(d[i], n[i], *f[i], *info[i], coefs[i]);
            }
        }
        trim_scratch(c0);
        trim_scratch(c1);
        return;
    }
    BlockOrder oa, ob;
    FastDec a, b;
    a.init(c0, oa, *f[0], *info[0], coefs[0]);
    b.init(c1, ob, *f[1], *info[1], coefs[1]);
    while (!a.done && !b.done) {   // three interleaved step pairs per refill
        a.br.refill();
        b.br.refill();
        a.step();
        b.step();
        if (a.done | b.done) break;
        a.step();
        b.step();
        if (a.done | b.done) break;
        a.step();
        b.step();
    }
    const bool b_first = b.done && !a.done;
    a.finish();
    b.finish();
    if (b_first) {
        rc[1] = b.report();
        rc[0] = a.report();
    } else {
        rc[0] = a.report();
        rc[1] = b.report();
    }
    for (int i = 0; i < 2; ++i)
        if (rc[i] != HJD_OK) rc[i] = exact_error(d[i], n[i], *f[i], *info[i], coefs[i], rc[i]);
    trim_scratch(c0);
    trim_scratch(c1);
}

// ---- several scans per frame: sequential multi-scan and progressive -------
// (extensions; the reference decodes one interleaved sequential scan)

// Where block (by, bx) of frame component c lives in the MCU-major output, and
// the component's block grid in a non-interleaved scan (T.81 A.2.2: ceil of
// the component's own dimensions, not padded to whole MCUs; blocks outside it
// are never coded and stay zero).
struct CoefLayout {
    int mcu_w = 0, mcu_h = 0, bpm = 0;
    int hs[3] = {1, 1, 1}, vs[3] = {1, 1, 1}, base[3] = {0, 0, 0};
    int bw[3] = {0, 0, 0}, bh[3] = {0, 0, 0};

    CoefLayout(const Frame& f, const hjd_jpeg_info& info) : mcu_w(info.mcu_w), mcu_h(info.mcu_h)
    {
        if (f.ncomp == 1) {
            bpm = 1;
            bw[0] = (f.width + 7) / 8;
            bh[0] = (f.height + 7) / 8;
            return;
        }
        const int hmax = f.comp[0].h, vmax = f.comp[0].v;   // chroma is H1V1 in every admitted sampling
        for (int c = 0; c < 3; ++c) {
            hs[c] = f.comp[c].h;
            vs[c] = f.comp[c].v;
            const int cw = (f.width * hs[c] + hmax - 1) / hmax, ch = (f.height * vs[c] + vmax - 1) / vmax;
            bw[c] = (cw + 7) / 8;
            bh[c] = (ch + 7) / 8;
        }
        base[1] = hs[0] * vs[0];
        base[2] = base[1] + 1;
        bpm = base[2] + 1;
    }
    int16_t* at(int16_t* coefs, int c, int by, int bx) const
    {
        // sampling factors are 1, 2 or 4 in every admitted layout: shifts and masks
        const int lh = hs[c] >> 1, lv = vs[c] >> 1;   // log2 of 1, 2, 4
        const int64_t mcu = static_cast<int64_t>(by >> lv) * mcu_w + (bx >> lh);
        return coefs + (mcu * bpm + base[c] + ((by & (vs[c] - 1)) << lh) + (bx & (hs[c] - 1))) * 64;
    }
};

inline int get_bit(BitReader& br)
{
    if (br.nbits < 1) br.refill();
    const int b = static_cast<int>(br.peek(1));
    br.skip(1);
    return b;
}

inline int receive_bits(BitReader& br, int n)
{
    if (n == 0) return 0;
    if (br.nbits < n) br.refill();
    const int v = static_cast<int>(br.peek(n));
    br.skip(n);
    return v;
}

inline bool fits16(int v) { return v >= -32768 && v <= 32767; }

// Progressive decoding procedures (T.81 G.1.2.1-G.1.2.3).  Coefficients are
// kept in zigzag order, as the fused kernel takes them.
struct ProgState {
    int pred[3] = {0, 0, 0};
    int eobrun = 0;
};

inline bool dc_first(BitReader& br, const HuffTable& dc, int& pred, int al, int16_t* blk)
{
    const int s = decode_symbol(br, dc);
    if (s < 0 || s > 11) return false;
    pred += receive_extend(br, s);
    const int v = pred * (1 << al);
    if (!fits16(v)) return false;
    blk[0] = static_cast<int16_t>(v);
    return true;
}

inline bool ac_first(BitReader& br, const HuffTable& ac, const ScanSpec& sc, int& eobrun, int16_t* blk)
{
    if (eobrun > 0) {
        --eobrun;
        return true;
    }
    for (int k = sc.ss; k <= sc.se;) {
        if (br.nbits < 16) br.refill();
        const int32_t fe = ac.fast_ac[br.peek(kFastBits)];
        if (fe && !(fe & kFastEob)) {   // run + nonzero coefficient in one lookup (EOB0 takes the EOBRUN path)
            br.skip(fe & 31);
            k += (fe >> 5) & 15;
            if (k > sc.se) return false;
            const int v = (fe >> 16) * (1 << sc.al);
            if (!fits16(v)) return false;
            blk[k++] = static_cast<int16_t>(v);
            continue;
        }
        const int rs = decode_symbol(br, ac);
        if (rs < 0) return false;
        const int r = rs >> 4, s = rs & 15;
        if (s) {
            k += r;
            if (k > sc.se) return false;
            const int v = receive_extend(br, s) * (1 << sc.al);
            if (!fits16(v)) return false;
            blk[k++] = static_cast<int16_t>(v);
        } else if (r == 15) {
            k += 16;   // ZRL
        } else {       // EOBr: this block and (2^r - 1 + r bits) more end here
            eobrun = (1 << r) - 1 + receive_bits(br, r);
            break;
        }
    }
    return true;
}

// Correction bit of an already-nonzero coefficient (G.1.2.3).
inline void refine(BitReader& br, int16_t& coef, int p1)
{
    if (get_bit(br) && (coef & p1) == 0) coef = static_cast<int16_t>(coef >= 0 ? coef + p1 : coef - p1);
}

inline bool ac_refine(BitReader& br, const HuffTable& ac, const ScanSpec& sc, int& eobrun, int16_t* blk)
{
    const int p1 = 1 << sc.al;
    int k = sc.ss;
    if (eobrun == 0) {
        for (; k <= sc.se; ++k) {
            const int rs = decode_symbol(br, ac);
            if (rs < 0) return false;
            int r = rs >> 4;
            const int s = rs & 15;
            int val = 0;
            if (s) {
                if (s != 1) return false;   // a newly significant coefficient is +-1 << Al
                val = get_bit(br) ? p1 : -p1;
            } else if (r != 15) {
                eobrun = (1 << r) + receive_bits(br, r);
                break;                      // the EOB run starts with this block's remainder
            }
            // skip r still-zero coefficients (refining the nonzero ones passed
            // on the way), then place val on the next zero one
            for (; k <= sc.se; ++k) {
                int16_t& coef = blk[k];
                if (coef != 0)
                    refine(br, coef, p1);
                else if (--r < 0)
                    break;
            }
            if (val) {
                if (k > sc.se) return false;
                blk[k] = static_cast<int16_t>(val);
            }
        }
    }
    if (eobrun > 0) {   // inside an EOB run: only correction bits for nonzero coefficients
        for (; k <= sc.se; ++k)
            if (blk[k] != 0) refine(br, blk[k], p1);
        --eobrun;
    }
    return true;
}

// One scan of a multi-scan frame.  Returns HJD_OK and *end = the byte after
// the scan's entropy-coded segment (the next marker).
int decode_scan_any(const uint8_t* d, size_t n, const Frame& f, const CoefLayout& L, int16_t* coefs, size_t* end)
{
    const ScanSpec& sc = f.scan;
    BitReader br{d + sc.offset, d + n};
    ProgState st;
    const bool prog = f.process == 2;
    // interleaved scan: MCUs of the frame; non-interleaved: the component's blocks
    const int c0 = sc.comp[0];
    const int uw = sc.ns == 1 ? L.bw[c0] : L.mcu_w;
    const int64_t units = sc.ns == 1 ? static_cast<int64_t>(L.bw[c0]) * L.bh[c0]
                                     : static_cast<int64_t>(L.mcu_w) * L.mcu_h;
    auto block = [&](int c, int16_t* blk) -> bool {
        if (!prog) return decode_block(br, f.dc[f.comp[c].td], f.ac[f.comp[c].ta], st.pred[c], blk);
        if (sc.ss == 0) {
            if (sc.ah == 0) return dc_first(br, f.dc[f.comp[c].td], st.pred[c], sc.al, blk);
            if (get_bit(br)) blk[0] = static_cast<int16_t>(blk[0] | (1 << sc.al));
            return true;
        }
        return sc.ah == 0 ? ac_first(br, f.ac[f.comp[c].ta], sc, st.eobrun, blk)
                          : ac_refine(br, f.ac[f.comp[c].ta], sc, st.eobrun, blk);
    };
    int restarts = 0, since = 0;
    for (int64_t u = 0; u < units; ++u) {
        if (br.overrun()) return report_incomplete(u - 1, units);
        if (f.restart_interval > 0 && since == f.restart_interval) {
            if (!br.restart(restarts))
                return set_error(HJD_E_INVALID, "expected RST%d before MCU %lld", restarts & 7, static_cast<long long>(u));
            ++restarts;
            since = 0;
            st = ProgState();
        }
        ++since;
        const int uy = static_cast<int>(u / uw), ux = static_cast<int>(u % uw);
        bool ok = true;
        if (sc.ns == 1) {
            ok = block(c0, L.at(coefs, c0, uy, ux));
        } else {
            for (int si = 0; si < sc.ns && ok; ++si) {
                const int c = sc.comp[si];
                for (int yy = 0; yy < L.vs[c] && ok; ++yy)
                    for (int xx = 0; xx < L.hs[c] && ok; ++xx)
                        ok = block(c, L.at(coefs, c, uy * L.vs[c] + yy, ux * L.hs[c] + xx));
            }
        }
        if (!ok) return set_error(HJD_E_INVALID, "corrupt entropy data in MCU %lld", static_cast<long long>(u));
    }
    if (br.overrun()) return report_incomplete(units - 1, units);
    // next marker: the reader stops in front of one, or is short of it by the
    // bytes it has not needed yet (entropy data: 0xFF only as FF00 / RSTn)
    const uint8_t* q = br.p;
    while (q + 1 < d + n && !(q[0] == 0xFF && q[1] != 0x00 && (q[1] < 0xD0 || q[1] > 0xD7))) ++q;
    *end = static_cast<size_t>(q - d);
    return HJD_OK;
}

int decode_multiscan(const uint8_t* d, size_t n, Frame& f, hjd_jpeg_info* info, int16_t* coefs)
{
    memset(coefs, 0, static_cast<size_t>(info->nblocks) * 64 * sizeof(int16_t));
    const CoefLayout L(f, *info);
    bool latched[3] = {false, false, false};
    for (;;) {
        for (int i = 0; i < f.scan.ns; ++i) {   // quantisation tables latch at a component's first scan
            const int c = f.scan.comp[i];
            if (!latched[c]) {
                memcpy(info->qt[c], f.qt[f.comp[c].tq], sizeof(info->qt[c]));
                info->qt_precision[c] = f.qt_prec[f.comp[c].tq];
                latched[c] = true;
            }
        }
        size_t p = 0;
        int rc = decode_scan_any(d, n, f, L, coefs, &p);
        if (rc) return rc;
        bool eoi = false;
        rc = parse_segments(d, n, &p, f, true, &eoi);
        if (rc) return rc;
        if (eoi) break;
    }
    if (f.ncomp == 1) {   // gray: the Y table in all three slots, as fill_info()
        memcpy(info->qt[1], info->qt[0], sizeof(info->qt[0]));
        memcpy(info->qt[2], info->qt[0], sizeof(info->qt[0]));
        info->qt_precision[1] = info->qt_precision[2] = info->qt_precision[0];
    }
    return HJD_OK;
}

// Parse and check one file for decoding into `coefs`.
int prepare_one(const uint8_t* data, size_t size, hjd_jpeg_info* info, int16_t* coefs, int64_t capacity, Frame& f)
{
    if (!data || !info) return set_error(HJD_E_INVALID, "NULL argument");
    int rc = parse(data, size, f);
    if (rc) return rc;
    fill_info(f, info);
    if (!coefs) return set_error(HJD_E_INVALID, "coefs is NULL");
    if (capacity < info->nblocks)
        return set_error(HJD_E_INVALID, "capacity %lld < %lld blocks", static_cast<long long>(capacity),
                         static_cast<long long>(info->nblocks));
    return HJD_OK;
}

int decode_prepared(const uint8_t* data, size_t size, Frame& f, hjd_jpeg_info* info, int16_t* coefs)
{
    if (single_scan(f)) return decode_scan(data, size, f, *info, coefs);
    return decode_multiscan(data, size, f, info, coefs);
}

int decode_one(const uint8_t* data, size_t size, hjd_jpeg_info* info, int16_t* coefs, int64_t capacity)
{
    Frame f(0);
    const int rc = prepare_one(data, size, info, coefs, capacity, f);
    return rc ? rc : decode_prepared(data, size, f, info, coefs);
}

// Two files: interleaved when both are single-scan sequential files
// (decode_scan_pair), else one after the other; rc[i] as decode_one returns.
void decode_two(const uint8_t* const data[2], const size_t size[2], hjd_jpeg_info* const info[2],
                int16_t* const coefs[2], const int64_t capacity[2], int rc[2])
{
    Frame f[2] = {Frame(0), Frame(1)};
    for (int i = 0; i < 2; ++i) rc[i] = prepare_one(data[i], size[i], info[i], coefs[i], capacity[i], f[i]);
    if (rc[0] == HJD_OK && rc[1] == HJD_OK && single_scan(f[0]) && single_scan(f[1])) {
        const Frame* fp[2] = {&f[0], &f[1]};
        const hjd_jpeg_info* ip[2] = {info[0], info[1]};
        decode_scan_pair(data, size, fp, ip, coefs, rc);
        return;
    }
    for (int i = 0; i < 2; ++i)
        if (rc[i] == HJD_OK) rc[i] = decode_prepared(data[i], size[i], f[i], info[i], coefs[i]);
}

}  // namespace

namespace {

// The header of the scan parse_segments() stopped at (f.scan), with the
// frame's state (tables, DRI, quantisation) as of that scan.
void fill_scan_header(const Frame& f, hjd_internal::ScanHeader* h)
{
    const ScanSpec& sc = f.scan;
    hjd_jpeg_info info;
    fill_info(f, &info);
    const CoefLayout L(f, info);
    h->width = f.width;
    h->height = f.height;
    h->sampling = f.sampling;
    h->restart_interval = f.restart_interval;
    h->mcu_w = info.mcu_w;
    h->mcu_h = info.mcu_h;
    h->nblocks = info.nblocks;
    h->out_bpm = L.bpm;
    h->scan_offset = sc.offset;
    memcpy(h->qt, info.qt, sizeof(h->qt));
    h->extra_scans = f.ncomp - sc.ns;
    // bitstream block order of one MCU (src/decoder.cpp:308-344): scan components
    // in SOS order, H*V blocks each; output slot = Y blocks, then Cb, then Cr.
    // A one-component scan of a multi-component frame is non-interleaved: one
    // block per MCU, the component's blocks in raster order (T.81 A.2.2).
    h->layout = sc.ns == 1 && f.ncomp > 1 ? 1 : 0;
    int j = 0;
    for (int si = 0; si < sc.ns; ++si) {
        const int c = sc.comp[si];
        const int nb = h->layout ? 1 : L.hs[c] * L.vs[c];
        for (int b = 0; b < nb; ++b, ++j) {
            h->jcomp[j] = c;
            h->jdc[j] = f.comp[c].td;
            h->jac[j] = f.comp[c].ta;
            h->jslot[j] = L.base[c] + b;
        }
    }
    h->bpm = j;
    const int c0 = sc.comp[0];
    h->comp_bw = L.bw[c0];
    h->comp_bh = L.bh[c0];
    h->comp_lh = L.hs[c0] >> 1;   // sampling factors 1, 2 or 4
    h->comp_lv = L.vs[c0] >> 1;
    h->scan_blocks = h->layout ? static_cast<int64_t>(L.bw[c0]) * L.bh[c0]
                               : static_cast<int64_t>(info.mcu_w) * info.mcu_h * h->bpm;
    for (int cls = 0; cls < 2; ++cls)
        for (int id = 0; id < 4; ++id) {
            const HuffTable& t = cls ? f.ac[id] : f.dc[id];
            h->table_defined[cls][id] = t.defined;
            if (!t.defined) continue;
            memcpy(h->counts[cls][id], t.counts, 16);
            memcpy(h->symbols[cls][id], t.vals, static_cast<size_t>(t.nsym));
            h->nsym[cls][id] = t.nsym;
        }
}

// The byte after a scan's entropy-coded data: the first marker that is not
// RSTn (stuffed FF00 and fill bytes skipped), or the end of the data.
size_t scan_end(const uint8_t* d, size_t n, size_t p)
{
    while (p < n) {
        const uint8_t* f = static_cast<const uint8_t*>(memchr(d + p, 0xFF, n - p));
        if (!f) return n;
        p = static_cast<size_t>(f - d);
        if (p + 1 >= n) return n;
        const uint8_t b = d[p + 1];
        if (b == 0x00 || (b >= 0xD0 && b <= 0xD7)) p += 2;
        else if (b == 0xFF) p += 1;
        else return p;
    }
    return n;
}

}  // namespace

int hjd_internal::parse_scan_header(const uint8_t* data, size_t size, ScanHeader* h)
{
    if (!data || !h) return set_error(HJD_E_INVALID, "NULL argument");
    Frame f(2, false);
    int rc = parse(data, size, f);
    if (rc) return rc;
    if (f.process == 2)
        return set_error(HJD_E_INVALID, "progressive JPEG: the GPU entropy decoder takes sequential scans "
                         "(decode it with the host decoder, hjd_jpeg_decode_coefs / hjd_stream)");
    fill_scan_header(f, h);
    return HJD_OK;
}

int hjd_internal::parse_scan_headers(const uint8_t* data, size_t size, std::vector<ScanHeader>* hs)
{
    if (!data || !hs) return set_error(HJD_E_INVALID, "NULL argument");
    hs->clear();
    Frame f(2, false);
    int rc = parse(data, size, f);
    if (rc) return rc;
    if (f.process == 2)
        return set_error(HJD_E_INVALID, "progressive JPEG: the GPU entropy decoder takes sequential scans "
                         "(decode it with the host decoder, hjd_jpeg_decode_coefs / hjd_stream)");
    bool seen[3] = {false, false, false};
    for (;;) {
        for (int i = 0; i < f.scan.ns; ++i) {
            if (seen[f.scan.comp[i]])   // T.81 B.2.3: a sequential frame codes each component in one scan
                return set_error(HJD_E_INVALID, "component %d in two sequential scans", f.scan.comp[i]);
            seen[f.scan.comp[i]] = true;
        }
        hs->emplace_back();
        fill_scan_header(f, &hs->back());
        size_t p = scan_end(data, size, f.scan.offset);
        bool eoi = false;
        rc = parse_segments(data, size, &p, f, true, &eoi);
        if (rc) return rc;
        if (eoi) break;
    }
    for (int c = 0; c < f.ncomp; ++c)
        if (!seen[c]) return set_error(HJD_E_INVALID, "component %d is in no scan", c);
    return HJD_OK;
}

int hjd_internal::jpeg_decode_coefs_two(const uint8_t* const data[2], const size_t size[2], hjd_jpeg_info* const info[2],
                                        int16_t* const coefs[2], const int64_t capacity[2], int rc[2])
{
    decode_two(data, size, info, coefs, capacity, rc);
    return rc[0] != HJD_OK ? rc[0] : rc[1];
}

// ---- the process's CPU share (hjd_host_cpu_share) --------------------------
namespace {

std::string read_small_file(const std::string& path)
{
    FILE* f = fopen(path.c_str(), "r");
    if (!f) return {};
    char buf[4096];
    const size_t n = fread(buf, 1, sizeof(buf) - 1, f);
    fclose(f);
    buf[n] = 0;
    return buf;
}

// CPU quota of this process's cgroup, in CPUs rounded up (0: none).  The
// cgroup comes from /proc/self/cgroup: cgroup v2 ("0::<path>", cpu.max =
// "<quota> <period>" or "max ...") or v1 (a "cpu" controller line,
// cpu.cfs_quota_us / cpu.cfs_period_us, quota -1 = none), and every ancestor
// up to the mount root counts (a limit anywhere above applies too): the
// smallest quota wins.  `root` is "" for the real filesystem (tests pass a
// fake tree).
int cgroup_quota_cpus(const std::string& root)
{
    const std::string self = read_small_file(root + "/proc/self/cgroup");
    int best = 0;
    auto consider = [&](long long quota, long long period) {
        if (quota <= 0 || period <= 0) return;
        const int n = static_cast<int>((quota + period - 1) / period);
        if (n > 0 && (best == 0 || n < best)) best = n;
    };
    // walk a cgroup path and its ancestors under `mount`
    auto walk = [&](const std::string& mount, std::string path, bool v2) {
        for (;;) {
            const std::string dir = root + mount + (path == "/" ? "" : path);
            if (v2) {
                const std::string m = read_small_file(dir + "/cpu.max");
                char q[32] = {0};
                long long per = 0;
                if (!m.empty() && sscanf(m.c_str(), "%31s %lld", q, &per) == 2 && strcmp(q, "max") != 0)
                    consider(atoll(q), per);
            } else {
                const std::string q = read_small_file(dir + "/cpu.cfs_quota_us"), per = read_small_file(dir + "/cpu.cfs_period_us");
                if (!q.empty() && !per.empty()) consider(atoll(q.c_str()), atoll(per.c_str()));
            }
            if (path.empty() || path == "/") break;
            const size_t k = path.find_last_of('/');
            path = k == 0 || k == std::string::npos ? "/" : path.substr(0, k);
        }
    };
    size_t i = 0;
    while (i < self.size()) {
        size_t e = self.find('\n', i);
        if (e == std::string::npos) e = self.size();
        const std::string line = self.substr(i, e - i);
        i = e + 1;
        const size_t c1 = line.find(':'), c2 = c1 == std::string::npos ? c1 : line.find(':', c1 + 1);
        if (c2 == std::string::npos) continue;
        const std::string ctrl = line.substr(c1 + 1, c2 - c1 - 1), path = line.substr(c2 + 1);
        if (ctrl.empty()) {   // v2 unified hierarchy
            walk("/sys/fs/cgroup", path, true);
        } else if (("," + ctrl + ",").find(",cpu,") != std::string::npos) {   // v1 cpu controller
            walk("/sys/fs/cgroup/" + ctrl, path, false);
            walk("/sys/fs/cgroup/cpu", path, false);
        }
    }
    if (best == 0) {   // no /proc/self/cgroup (or nothing under it): the v2 and v1 mount roots
        walk("/sys/fs/cgroup", "/", true);
        walk("/sys/fs/cgroup/cpu", "/", false);
    }
    return best;
}

int cpu_share(const std::string& root)
{
    int n = 0;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = 1;
    const int q = cgroup_quota_cpus(root);
    return std::max(1, q > 0 ? std::min(n, q) : n);
}

}  // namespace

extern "C" {

int hjd_host_cpu_share(void)
{
    static const int share = cpu_share("");   // once per process
    return share;
}

int hjd_debug_cpu_share(const char* root) { return cpu_share(root ? root : ""); }

int hjd_jpeg_parse(const uint8_t* data, size_t size, hjd_jpeg_info* info)
{
    if (!data || !info) return set_error(HJD_E_INVALID, "NULL argument");
    Frame f(2, false);
    int rc = parse(data, size, f);
    if (rc) return rc;
    fill_info(f, info);
    return HJD_OK;
}

int hjd_debug_host_reader(int mode)
{
    if (mode < 0) return g_host_reader.load();
    if (mode > 1) return set_error(HJD_E_INVALID, "host reader mode %d (0 de-stuffed, 1 byte-wise)", mode);
    return g_host_reader.exchange(mode);
}

int hjd_jpeg_decode_coefs(const uint8_t* data, size_t size, hjd_jpeg_info* info, int16_t* coefs,
                          int64_t capacity_blocks)
{
    return decode_one(data, size, info, coefs, capacity_blocks);
}

int hjd_jpeg_decode_batch(const uint8_t* const* datas, const size_t* sizes, int n, int16_t* const* coefs,
                          int64_t capacity_blocks, int nthreads, int32_t* status)
{
    if (n < 0 || (n > 0 && (!datas || !sizes || !coefs))) return set_error(HJD_E_INVALID, "invalid arguments");
    if (nthreads <= 0) nthreads = hjd_host_cpu_share();
    // each thread takes two files at a time (decode_two: interleaved symbol steps)
    nthreads = std::min(nthreads, std::max((n + 1) / 2, 1));
    std::atomic<int> next{0}, failed{0};
    auto work = [&]() {
        hjd_jpeg_info info[2];
        for (int i = next.fetch_add(2); i < n; i = next.fetch_add(2)) {
            int rc[2] = {HJD_OK, HJD_OK};
            if (i + 1 < n) {
                const uint8_t* d[2] = {datas[i], datas[i + 1]};
                const size_t sz[2] = {sizes[i], sizes[i + 1]};
                hjd_jpeg_info* ip[2] = {&info[0], &info[1]};
                int16_t* const c[2] = {coefs[i], coefs[i + 1]};
                const int64_t cap[2] = {capacity_blocks, capacity_blocks};
                decode_two(d, sz, ip, c, cap, rc);
            } else {
                rc[0] = decode_one(datas[i], sizes[i], &info[0], coefs[i], capacity_blocks);
            }
            for (int j = 0; j < 2 && i + j < n; ++j) {
                if (status) status[i + j] = rc[j];
                if (rc[j]) failed++;
            }
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nthreads; ++t) pool.emplace_back(work);
    work();
    for (auto& t : pool) t.join();
    return failed ? set_error(HJD_E_INVALID, "%d of %d files failed to decode", failed.load(), n) : HJD_OK;
}

}  // extern "C"
