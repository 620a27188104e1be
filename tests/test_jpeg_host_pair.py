"""The host decoder's two-file interleaved decode (jpeg_host.cpp decode_two /
decode_scan_pair), used by hjd_jpeg_decode_batch and the host-Huffman stream
(hjd_stream workers take two jobs at a time): for every ordered pair of a
corpus of files -- every sampling, restart intervals, 16-bit tables, the
reference's sample, progressive and multi-scan files (which take the one-file
path) and damaged files -- the pair decode must return each file's status and
coefficients exactly as decoding that file alone does."""
import ctypes
import io
import os

import numpy as np
import pytest

import jpeg_writer as JW
import oracle_py as O
from test_jpeg_host import _pil_jpeg, _pil_smooth, decode

FACTORS = {0: [(1, 1)] * 3, 1: [(2, 2), (1, 1), (1, 1)], 3: [(2, 1), (1, 1), (1, 1)],
           5: [(4, 1), (1, 1), (1, 1)], 6: [(1, 2), (1, 1), (1, 1)]}


@pytest.fixture(scope="module")
def lib():
    from ocljpegdecoder_amd import _lib
    return _lib.load()


def _huff_src():
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, format="JPEG", quality=90)
    return b.getvalue()


def _damage(data: bytes, seed: int) -> bytes:
    """Flip a few bytes inside the entropy-coded segment (after the SOS header)."""
    rng = np.random.default_rng(seed)
    d = bytearray(data)
    sos = d.index(b"\xff\xda")
    start = sos + 2 + ((d[sos + 2] << 8) | d[sos + 3])
    for p in rng.integers(start, len(d) - 2, 3):
        d[p] ^= int(rng.integers(1, 256))
    return bytes(d)


def _corpus():
    files = [open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read() for n in O.golden_cases()]
    files += [_pil_smooth(40, 24, 90, "L")[0], _pil_smooth(333, 77, 90, "L", restart_marker_blocks=5)[0],
              _pil_smooth(333, 77, 90, "RGB", 1)[0], _pil_smooth(200, 40, 90, "RGB", 1, restart_marker_rows=1)[0],
              _pil_jpeg(64, 48, 50, 0), _pil_jpeg(130, 66, 95, 2, restart_marker_blocks=3),
              _pil_jpeg(96, 80, 85, 2, progressive=True)]
    src = _huff_src()
    for s in (5, 6, 3):
        for w, h, dri in ((97, 41, 0), (64, 16, 1)):
            coefs, qt = O.synthetic_coefs(w, h, s, seed=w + s)
            files.append(JW.encode_frame(coefs, w, h, FACTORS[s], qt, src, restart_interval=dri))
    coefs, qt = O.synthetic_coefs(80, 48, 1, seed=3)
    base = JW.encode_frame(coefs, 80, 48, FACTORS[1], qt, src)
    files.append(JW.rewrite_scans(base, coefs, [(0,), (1, 2)], 2)[0])        # sequential, two scans
    good = _pil_jpeg(120, 72, 90, 2)
    files += [_damage(good, k) for k in range(4)] + [good[: len(good) * 2 // 3]]
    return files


def _batch(lib, datas, cap, nthreads=1):
    u8p, i16p = ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int16)
    bufs = [(ctypes.c_uint8 * len(d)).from_buffer_copy(d) for d in datas]
    outs = [np.full((cap, 64), 0x5A5A, np.int16) for _ in datas]
    arr_d = (u8p * len(bufs))(*[ctypes.cast(b, u8p) for b in bufs])
    arr_s = (ctypes.c_size_t * len(datas))(*[len(d) for d in datas])
    arr_o = (i16p * len(outs))(*[o.ctypes.data_as(i16p) for o in outs])
    status = (ctypes.c_int32 * len(datas))()
    lib.hjd_jpeg_decode_batch(arr_d, arr_s, len(datas), arr_o, cap, nthreads, status)
    return list(status), outs


def test_pairs_equal_single_decodes(lib):
    files = _corpus()
    singles = [decode(lib, d) for d in files]
    assert sum(rc == 0 for rc, _, _ in singles) >= len(files) - 5    # the damaged ones may fail
    assert any(rc != 0 for rc, _, _ in singles)                        # ... and some do
    cap = max(i.nblocks for _, i, _ in singles)
    for a in range(len(files)):
        for b in range(len(files)):
            status, outs = _batch(lib, [files[a], files[b]], cap)      # one thread: files a, b as a pair
            for k, i in ((0, a), (1, b)):
                rc, info, coefs = singles[i]
                assert (status[k] == 0) == (rc == 0), (a, b, k, status[k], rc)
                if rc == 0:
                    np.testing.assert_array_equal(outs[k][: info.nblocks], coefs, err_msg=f"pair ({a},{b}) file {k}")


def test_odd_batch_and_many_threads(lib):
    """Batches of odd length (the last file alone) over several threads."""
    files = _corpus()[:13]
    singles = [decode(lib, d) for d in files]
    cap = max(i.nblocks for _, i, _ in singles)
    status, outs = _batch(lib, files, cap, nthreads=3)
    for k, (rc, info, coefs) in enumerate(singles):
        assert status[k] == rc == 0
        np.testing.assert_array_equal(outs[k][: info.nblocks], coefs)


def _fill_bytes(data: bytes, inside: bool) -> bytes:
    """Insert a fill byte (0xFF) in front of the first RST marker (legal: the
    readers skip it), or -- inside=True -- in front of the first stuffed FF00
    of the entropy data (FF FF 00: the byte-wise reader's own case)."""
    d = bytearray(data)
    sos = d.index(b"\xff\xda")
    start = sos + 2 + ((d[sos + 2] << 8) | d[sos + 3])
    pat = b"\xff\x00" if inside else bytes([0xFF, 0xD0])
    at = d.index(pat, start)
    d[at:at] = b"\xff"
    return bytes(d)


def _wrong_rst(data: bytes) -> bytes:
    d = bytearray(data)
    sos = d.index(b"\xff\xda")
    at = d.index(bytes([0xFF, 0xD1]), sos)
    d[at + 1] = 0xD3
    return bytes(d)


def test_readers_agree(lib):
    """The de-stuffed reader (the default for single-scan files) against the
    byte-wise reader (hjd_debug_host_reader(1)): the same status, error text
    and coefficients on the corpus, on fill bytes before a marker and inside
    the data, on a wrong RST number and on cut files."""
    rst = _pil_jpeg(130, 66, 95, 2, restart_marker_blocks=3)
    files = _corpus() + [_fill_bytes(rst, False), _fill_bytes(rst, True), _fill_bytes(_pil_jpeg(64, 48, 95, 0), True),
                         _wrong_rst(rst), rst[: len(rst) // 2], rst[: len(rst) // 2] + b"\xff"]
    assert lib.hjd_debug_host_reader(-1) == 0
    for i, d in enumerate(files):
        res = []
        for mode in (0, 1):
            assert lib.hjd_debug_host_reader(mode) in (0, 1)
            rc, info, coefs = decode(lib, d)
            res.append((rc, lib.hjd_last_error() if rc else b"", coefs))
        lib.hjd_debug_host_reader(0)
        (r0, e0, c0), (r1, e1, c1) = res
        assert r0 == r1 and e0 == e1, (i, r0, r1, e0, e1)
        if r0 == 0 and c0 is not None:
            np.testing.assert_array_equal(c0, c1, err_msg=f"file {i}")
    assert decode(lib, _fill_bytes(rst, False))[0] == 0          # a fill byte before RSTn is legal
    assert decode(lib, _wrong_rst(rst))[0] != 0
    assert lib.hjd_debug_host_reader(2) != 0 and lib.hjd_debug_host_reader(-1) == 0


def test_batch_into_given_outputs():
    """decode_coefs_batch(outs=...): caller buffers (larger than needed) get the
    same coefficients as fresh ones; a short buffer is refused before decoding."""
    import ocljpegdecoder_amd as hjd
    files = _corpus()[:6]
    fresh = hjd.decode_coefs_batch(files, nthreads=2)
    outs = [np.full((c.shape[0] + 7, 64), 0x5A5A, np.int16) for c in fresh]
    got = hjd.decode_coefs_batch(files, nthreads=2, outs=outs)
    assert all(g is o for g, o in zip(got, outs))
    for c, o in zip(fresh, outs):
        np.testing.assert_array_equal(o[: c.shape[0]], c)
    with pytest.raises(ValueError):
        hjd.decode_coefs_batch(files[:1], outs=[np.zeros((1, 64), np.int16)])
    with pytest.raises(ValueError):
        hjd.decode_coefs_batch(files[:2], outs=outs[:1])


def test_cpu_share_is_the_default_pool_size(lib):
    """hjd_host_cpu_share (the nthreads = 0 default of the host pools): the
    affinity mask capped by the cgroup's cpu.max quota -- the rule bench.py's
    host_cpu_share applies."""
    import bench
    share = lib.hjd_host_cpu_share()
    assert 1 <= share <= len(os.sched_getaffinity(0))
    assert share == bench.host_cpu_share()[0]
    status, outs = _batch(lib, _corpus()[:3], 4096, nthreads=0)   # default pool
    assert list(status) == [0, 0, 0]


def _edge_blocks(n, seed):
    """Quantised zigzag blocks aimed at the host decoder's lookup tables: the
    last coefficient at 63 (no EOB), coefficients at 61-63, zero runs of 14-47
    (ZRL), magnitudes at the 9-bit entry limit (255/256) and the AC maximum
    (1023), DC-only blocks and dense blocks."""
    rng = np.random.default_rng(seed)
    out = np.zeros((n, 64), np.int16)
    mags = np.array([1, 2, 3, 7, 31, 127, 255, 256, 511, 512, 1023])
    for i in range(n):
        kind = i % 8
        b = out[i]
        b[0] = rng.integers(-1000, 1000)
        if kind == 0:                      # DC only
            continue
        if kind == 1:                      # a coefficient at 63, no EOB
            b[63] = rng.choice([-1, 1, 5, -300])
            b[rng.integers(1, 40)] = rng.integers(-3, 4)
        elif kind == 2:                    # 61, 62, 63 (pairs near the end)
            b[61:64] = rng.choice(mags, 3) * rng.choice([-1, 1], 3)
        elif kind == 3:                    # zero runs of 14..47 (ZRL)
            k = 1 + int(rng.integers(14, 48))
            b[min(k, 63)] = rng.choice([-1, 2, 300])
            if k + 16 < 63:
                b[k + 16] = 1
        elif kind == 4:                    # entry limits and the AC maximum
            pos = np.sort(rng.choice(np.arange(1, 64), 6, replace=False))
            b[pos] = rng.choice(mags, 6) * rng.choice([-1, 1], 6)
        elif kind == 5:                    # dense, small values
            b[1:] = rng.integers(-3, 4, 63)
        elif kind == 6:                    # runs of exactly 15 and 16 before a coefficient
            b[16] = 2
            b[33] = -1
            b[63] = 1
        else:                              # random sparse
            pos = rng.choice(np.arange(1, 64), int(rng.integers(1, 12)), replace=False)
            b[pos] = rng.integers(-60, 61, pos.size)
    return out


@pytest.mark.parametrize("sampling,dri", [(1, 0), (1, 3), (0, 0), (3, 2)])
def test_edge_coefficients_round_trip(lib, sampling, dri):
    """Encode the edge blocks (tests/jpeg_writer.py, standard tables) and decode
    them: the default reader alone, in a pair, and the byte-wise reader all
    return exactly the encoded coefficients."""
    w, h = 96, 64
    nblk = O.frame_blocks(w, h, sampling)
    coefs = _edge_blocks(nblk, seed=sampling * 10 + dri)
    _, qt = O.synthetic_coefs(16, 16, sampling, seed=1)
    data = JW.encode_frame(coefs, w, h, FACTORS[sampling], qt, _huff_src(), restart_interval=dri)
    rc, info, got = decode(lib, data)
    assert rc == 0 and info.nblocks == nblk
    np.testing.assert_array_equal(got, coefs)
    other = _corpus()[0]
    cap = max(nblk, decode(lib, other)[1].nblocks)
    status, outs = _batch(lib, [data, other, data], cap)   # a pair, then a lone file
    assert list(status) == [0, 0, 0]
    np.testing.assert_array_equal(outs[0][:nblk], coefs)
    np.testing.assert_array_equal(outs[2][:nblk], coefs)
    lib.hjd_debug_host_reader(1)
    try:
        rc, _, got = decode(lib, data)
    finally:
        lib.hjd_debug_host_reader(0)
    assert rc == 0
    np.testing.assert_array_equal(got, coefs)


def test_small_thread_stack(lib):
    """The Huffman tables live in per-thread heap sets, not on the stack
    (ADVICE r05): the pair decode, the one-file decode and a header parse run
    on a thread with a 256 KiB stack (the r05 Frame alone was ~165 KB)."""
    import threading
    files = _corpus()[:4]
    singles = [decode(lib, d) for d in files]
    cap = max(i.nblocks for _, i, _ in singles)
    res = {}

    def body():
        try:
            res["pair"] = _batch(lib, files, cap, nthreads=1)   # the calling thread decodes the pairs
            res["one"] = decode(lib, files[0])
        except BaseException as e:   # noqa: BLE001 -- reported by the main thread
            res["error"] = e

    old = threading.stack_size(256 * 1024)
    try:
        t = threading.Thread(target=body)
        t.start()
        t.join()
    finally:
        threading.stack_size(old)
    assert "error" not in res, res.get("error")
    status, outs = res["pair"]
    for k, (rc, info, coefs) in enumerate(singles):
        assert status[k] == rc == 0
        np.testing.assert_array_equal(outs[k][: info.nblocks], coefs)
    np.testing.assert_array_equal(res["one"][2], singles[0][2])
