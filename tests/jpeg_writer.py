"""Test tooling: re-encode a baseline JPEG's quantised coefficients as a
sequential JPEG with a different scan structure (non-interleaved or partly
interleaved scans, any component order, optional DRI).  The tables (DQT,
DHT) and frame header are copied from the source file, so a decoder that
handles multi-scan files must return exactly the source's coefficients.
Plain Python (T.81 F.1.2 Huffman encoding); small images only."""
import numpy as np


def _segments(data: bytes):
    """(marker, payload) of every segment before the first SOS."""
    p, out = 2, []
    while True:
        assert data[p] == 0xFF
        m = data[p + 1]
        ln = (data[p + 2] << 8) | data[p + 3]
        if m == 0xDA:
            return out
        out.append((m, data[p + 4:p + 2 + ln]))
        p += 2 + ln


def _codes(counts, symbols):
    """symbol -> (code, length) of a canonical Huffman table (T.81 C.2)."""
    table, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(counts[ln - 1]):
            table[symbols[k]] = (code, ln)
            code += 1
            k += 1
        code <<= 1
    return table


class _Bits:
    def __init__(self):
        self.out = bytearray()
        self.acc = 0
        self.n = 0

    def put(self, v, n):
        for i in range(n - 1, -1, -1):
            self.acc = (self.acc << 1) | ((v >> i) & 1)
            self.n += 1
            if self.n == 8:
                self.out.append(self.acc)
                if self.acc == 0xFF:
                    self.out.append(0)
                self.acc = self.n = 0

    def flush(self):   # pad with 1-bits (F.1.2.3)
        if self.n:
            self.put((1 << (8 - self.n)) - 1, 8 - self.n)


def _category(v):
    a = abs(int(v))
    s = a.bit_length()
    return s, (v if v >= 0 else v + (1 << s) - 1) & ((1 << s) - 1)


def _encode_block(bw, blk, pred, dct, act):
    s, bits = _category(int(blk[0]) - pred)
    c, ln = dct[s]
    bw.put(c, ln)
    bw.put(bits, s)
    run = 0
    last = max([k for k in range(1, 64) if blk[k]] or [0])
    for k in range(1, last + 1):
        if blk[k] == 0:
            run += 1
            continue
        while run > 15:
            c, ln = act[0xF0]
            bw.put(c, ln)
            run -= 16
        s, bits = _category(int(blk[k]))
        c, ln = act[(run << 4) | s]
        bw.put(c, ln)
        bw.put(bits, s)
        run = 0
    if last < 63:
        c, ln = act[0x00]
        bw.put(c, ln)
    return int(blk[0])


def _dht_codes(segs):
    dht = {}
    for m, p in segs:
        if m != 0xC4:
            continue
        q = 0
        while q < len(p):
            tc, th = p[q] >> 4, p[q] & 15
            counts = list(p[q + 1:q + 17])
            n = sum(counts)
            dht[(tc, th)] = _codes(counts, list(p[q + 17:q + 17 + n]))
            q += 17 + n
    return dht


def _emit(header, comps, tabs, dht, w, h, coefs, scans, restart_interval):
    """SOI + header segments + DRI + the scans + EOI; returns (bytes, expect)."""
    nc = len(comps)
    # geometry (T.81 A.2): MCU-major layout of the coefficients
    hmax, vmax = max(c[1] for c in comps), max(c[2] for c in comps)
    if nc == 1:
        hs, vs, base, bpm = [1], [1], [0], 1
        mcu_w = (w + 7) // 8
        mcu_h = (h + 7) // 8
    else:
        hs, vs = [c[1] for c in comps], [c[2] for c in comps]
        base = [0, hs[0] * vs[0], hs[0] * vs[0] + 1]
        bpm = base[2] + 1
        mcu_w, mcu_h = -(-w // (8 * hmax)), -(-h // (8 * vmax))
    blocks = coefs.reshape(-1, bpm, 64)
    expect = np.zeros_like(blocks)

    def at(c, by, bx):
        return blocks[(by // vs[c]) * mcu_w + bx // hs[c], base[c] + (by % vs[c]) * hs[c] + bx % hs[c]]

    out = bytearray(b"\xff\xd8")
    for m, p in header:
        out += bytes([0xFF, m, (len(p) + 2) >> 8, (len(p) + 2) & 255]) + p
    if restart_interval:
        out += bytes([0xFF, 0xDD, 0, 4, restart_interval >> 8, restart_interval & 255])
    for sc in scans:
        out += bytes([0xFF, 0xDA, 0, 6 + 2 * len(sc), len(sc)])
        for c in sc:
            out += bytes([comps[c][0], (tabs[c][0] << 4) | tabs[c][1]])
        out += bytes([0, 63, 0])
        bw = _Bits()
        pred = [0] * nc
        if len(sc) == 1:
            c = sc[0]
            if nc == 1:
                bwc, bhc = mcu_w, mcu_h
            else:
                bwc = -(-(-(-w * hs[c] // hmax)) // 8)
                bhc = -(-(-(-h * vs[c] // vmax)) // 8)
            units = [[(c, by, bx)] for by in range(bhc) for bx in range(bwc)]
        else:
            units = [[(c, my * vs[c] + yy, mx * hs[c] + xx) for c in sc for yy in range(vs[c]) for xx in range(hs[c])]
                     for my in range(mcu_h) for mx in range(mcu_w)]
        for i, unit in enumerate(units):
            if restart_interval and i and i % restart_interval == 0:
                bw.flush()
                bw.out += bytes([0xFF, 0xD0 + ((i // restart_interval - 1) & 7)])
                pred = [0] * nc
            for c, by, bx in unit:
                blk = at(c, by, bx)
                pred[c] = _encode_block(bw, blk, pred[c], dht[(0, tabs[c][0])], dht[(1, tabs[c][1])])
                expect[(by // vs[c]) * mcu_w + bx // hs[c], base[c] + (by % vs[c]) * hs[c] + bx % hs[c]] = blk
        bw.flush()
        out += bw.out
    out += b"\xff\xd9"
    return bytes(out), expect.reshape(coefs.shape)


def rewrite_scans(data: bytes, coefs: np.ndarray, scans, restart_interval=0):
    """scans: list of tuples of frame component indices, e.g. [(0,), (1, 2)].
    coefs: the source's coefficients (MCU-major, zigzag) from the decoder under
    test's baseline path, which the tests pin against the reference.
    Returns (jpeg bytes, expected coefficients): a non-interleaved scan codes
    only the component's own block grid (T.81 A.2.2), so MCU-padding blocks
    outside it are expected as zeros (they lie wholly outside the image)."""
    segs = _segments(data)
    sof = next(p for m, p in segs if m in (0xC0, 0xC1))
    h, w, nc = (sof[1] << 8) | sof[2], (sof[3] << 8) | sof[4], sof[5]
    comps = [(sof[6 + 3 * c], sof[7 + 3 * c] >> 4, sof[7 + 3 * c] & 15) for c in range(nc)]
    dht = _dht_codes(segs)
    # table ids of each component: copy the source's first SOS
    p = 2
    while not (data[p] == 0xFF and data[p + 1] == 0xDA):
        p += 2 + ((data[p + 2] << 8) | data[p + 3])
    ns0 = data[p + 4]
    tabs = {}
    for i in range(ns0):
        cid, t = data[p + 5 + 2 * i], data[p + 6 + 2 * i]
        tabs[[c[0] for c in comps].index(cid)] = (t >> 4, t & 15)
    header = [(m, p) for m, p in segs if m != 0xDD]
    return _emit(header, comps, tabs, dht, w, h, coefs, scans, restart_interval)


def encode_frame(coefs: np.ndarray, width: int, height: int, factors, qt, huff_src: bytes, scans=None,
                 restart_interval=0) -> bytes:
    """A baseline JPEG of the given quantised coefficients (MCU-major, zigzag)
    with SOF sampling factors `factors` [(H, V) per component] -- e.g. the
    4:1:1 (H4V1) and 4:4:0 (H1V2) layouts Pillow cannot write.  qt: zigzag
    tables (Y; chroma).  The Huffman tables are copied from huff_src (a
    libjpeg file with the standard tables: DC/AC 0 for Y, 1 for chroma)."""
    nc = len(factors)
    comps = [(c + 1, hf, vf) for c, (hf, vf) in enumerate(factors)]
    header = []
    for t in range(min(nc, 2)):
        header.append((0xDB, bytes([t]) + bytes(int(v) for v in qt[t])))
    sof = bytes([8, height >> 8, height & 255, width >> 8, width & 255, nc])
    for c, (cid, hf, vf) in enumerate(comps):
        sof += bytes([cid, (hf << 4) | vf, 0 if c == 0 else 1])
    header.append((0xC0, sof))
    src = _segments(huff_src)
    header += [(m, p) for m, p in src if m == 0xC4]
    tabs = {c: (0, 0) if c == 0 else (1, 1) for c in range(nc)}
    if scans is None:
        scans = [tuple(range(nc))]
    return _emit(header, comps, tabs, _dht_codes(src), width, height, coefs, scans, restart_interval)[0]
