"""CPU tests of the host JPEG front end (include/hjd_host.h): the Huffman
decoder must reproduce the reference's coefficients exactly (the fixtures'
coefs_q16 are derived from the compiled reference's jpg.mcu_data)."""
import ctypes
import os

import numpy as np
import pytest

import oracle_py as O


@pytest.fixture(scope="module")
def lib():
    from ocljpegdecoder_amd import _lib
    return _lib.load()


def decode(lib, data: bytes):
    from ocljpegdecoder_amd._lib import HjdJpegInfo
    info = HjdJpegInfo()
    buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
    rc = lib.hjd_jpeg_parse(buf, len(data), ctypes.byref(info))
    if rc:
        return rc, info, None
    coefs = np.zeros((info.nblocks, 64), np.int16)
    rc = lib.hjd_jpeg_decode_coefs(buf, len(data), ctypes.byref(info),
                                   coefs.ctypes.data_as(ctypes.POINTER(ctypes.c_int16)), info.nblocks)
    return rc, info, coefs


@pytest.mark.parametrize("name", O.golden_cases())
def test_huffman_matches_reference(lib, name):
    data = open(os.path.join(O.GOLDEN, name + ".jpg"), "rb").read()
    c = O.load_case(name)
    rc, info, coefs = decode(lib, data)
    assert rc == 0, lib.hjd_last_error()
    assert (info.width, info.height, info.sampling) == (int(c["width"]), int(c["height"]), int(c["sampling"]))
    np.testing.assert_array_equal(np.array(info.qt), c["qt"])
    np.testing.assert_array_equal(coefs, c["coefs_q16"])
    # full host path + oracle pixel stage == the reference's BGRX (config 1)
    if name == "JPEG_example_JPG_RIP_050":
        px = O.decode_q16(coefs, np.array(info.qt), info.width, info.height, info.sampling)
        np.testing.assert_array_equal(px, c["bgrx"])


def test_batch_decode_threads(lib):
    names = O.golden_cases()
    datas = [open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read() for n in names] * 3
    bufs = [(ctypes.c_uint8 * len(d)).from_buffer_copy(d) for d in datas]
    cap = 4096
    outs = [np.zeros((cap, 64), np.int16) for _ in datas]
    u8p = ctypes.POINTER(ctypes.c_uint8)
    i16p = ctypes.POINTER(ctypes.c_int16)
    arr_d = (u8p * len(bufs))(*[ctypes.cast(b, u8p) for b in bufs])
    arr_s = (ctypes.c_size_t * len(datas))(*[len(d) for d in datas])
    arr_o = (i16p * len(outs))(*[o.ctypes.data_as(i16p) for o in outs])
    status = (ctypes.c_int32 * len(datas))()
    rc = lib.hjd_jpeg_decode_batch(arr_d, arr_s, len(datas), arr_o, cap, 4, status)
    assert rc == 0 and list(status) == [0] * len(datas)
    for i, n in enumerate(names * 3):
        ref = O.load_case(n)["coefs_q16"]
        np.testing.assert_array_equal(outs[i][: ref.shape[0]], ref)


def _pil_jpeg(w, h, quality, subsampling, **kw):
    import io
    from PIL import Image
    rng = np.random.default_rng(w * h)
    img = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", quality=quality, subsampling=subsampling, **kw)
    return b.getvalue()


def test_rejects_unsupported(lib):
    import io
    from PIL import Image
    img = Image.fromarray(np.zeros((16, 16, 3), np.uint8))
    b = io.BytesIO(); img.save(b, format="JPEG")
    data = bytearray(b.getvalue())
    data[data.index(b"\xff\xc0") + 1] = 0xC3               # lossless (SOF3); progressive: test_jpeg_multiscan.py
    assert decode(lib, bytes(data))[0] != 0
    # Y H3V1 (no such layout is supported): patch the luma sampling byte of a 4:2:2 file's SOF0
    b = io.BytesIO(); img.save(b, format="JPEG", subsampling=1)
    data = bytearray(b.getvalue())
    sof = data.index(b"\xff\xc0")
    assert data[sof + 11] == 0x21
    data[sof + 11] = 0x31
    assert decode(lib, bytes(data))[0] != 0
    assert decode(lib, b"\x00\x01garbage")[0] != 0
    good = _pil_jpeg(32, 32, 90, 2)
    assert decode(lib, good[: len(good) // 2])[0] != 0   # truncated: "data incomplete" (tests/test_truncation.py)


def _pil_smooth(w, h, quality, mode, subsampling=0, seed=0, **kw):
    """Gradient + mild noise image encoded by Pillow (mode "RGB" or "L")."""
    import io
    from PIL import Image
    rng = np.random.default_rng(seed)
    x = np.arange(w)[None, :]
    y = np.arange(h)[:, None]
    img = np.stack([x * 255 / w + 0 * y, y * 255 / h + 0 * x, (x + y) * 127 / (w + h) + 60], -1)
    img = np.clip(img + rng.normal(0, 6, img.shape), 0, 255).astype(np.uint8)
    im = Image.fromarray(img)
    if mode == "L":
        im = im.convert("L")
    b = io.BytesIO()
    im.save(b, format="JPEG", quality=quality, subsampling=subsampling, **kw)
    return b.getvalue(), b


@pytest.mark.parametrize("mode,sub,w,h,kw", [
    ("L", 0, 40, 24, {}),
    ("L", 0, 333, 77, {"restart_marker_blocks": 5}),
    ("RGB", 1, 48, 16, {}),
    ("RGB", 1, 333, 77, {}),
    ("RGB", 1, 200, 40, {"restart_marker_rows": 1}),
])
def test_extension_samplings_decode(lib, mode, sub, w, h, kw):
    """4:2:2 and gray (the reference rejects both, so
    there is no reference output to match).  Host Huffman + the oracle's
    restatement must agree with Pillow's own decode of the same file to within
    IDCT/upsampling differences (Pillow: libjpeg islow IDCT, fancy
    upsampling); a wrong entropy decode would be garbage, not +-1 noise."""
    import io
    from PIL import Image
    data, _ = _pil_smooth(w, h, 90, mode, sub, **kw)
    rc, info, coefs = decode(lib, data)
    assert rc == 0, lib.hjd_last_error()
    want_sampling = 4 if mode == "L" else 3
    assert (info.width, info.height, info.sampling) == (w, h, want_sampling)
    assert info.nblocks == O.frame_blocks(w, h, want_sampling)
    px = O.decode_q16(coefs, np.array(info.qt), w, h, want_sampling)
    bgr = px.view(np.uint8).reshape(h, w, 4)[..., :3].astype(np.int32)
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))[..., ::-1].astype(np.int32)
    d = np.abs(bgr - ref)
    # measured: gray max 1 (IDCT rounding), 4:2:2 max 4-6 (Pillow's filtered
    # chroma upsampling); one DC coefficient off by 20 already gives 8-14
    assert d.mean() < 1.5 and d.max() <= (1 if mode == "L" else 6), (d.mean(), d.max())
    if mode == "L":
        assert (bgr[..., 0] == bgr[..., 1]).all() and (bgr[..., 1] == bgr[..., 2]).all()


def test_16bit_dqt_and_restart_rows(lib):
    """16-bit DQT (q=100 keeps tables 8-bit in PIL, so write one by hand) and
    DRI by rows: decoded coefficients round-trip through the oracle to the
    same pixels as an independent decode of the 8-bit-table equivalent."""
    data = bytearray(_pil_jpeg(48, 40, 60, 2, restart_marker_rows=1))
    rc, info8, coefs8 = decode(lib, bytes(data))
    assert rc == 0, lib.hjd_last_error()
    # rewrite every 8-bit DQT table as 16-bit (same values)
    out, p = bytearray(data[:2]), 2
    while p < len(data):
        assert data[p] == 0xFF
        m = data[p + 1]
        if m == 0xDA:
            out += data[p:]
            break
        ln = (data[p + 2] << 8) | data[p + 3]
        seg = data[p + 4:p + 2 + ln]
        if m == 0xDB:
            new, q = bytearray(), 0
            while q < len(seg):
                tq = seg[q] & 15
                new.append(0x10 | tq)
                for v in seg[q + 1:q + 65]:
                    new += bytes([0, v])
                q += 65
            out += bytes([0xFF, 0xDB, (len(new) + 2) >> 8, (len(new) + 2) & 255]) + new
        else:
            out += data[p:p + 2 + ln]
        p += 2 + ln
    rc, info16, coefs16 = decode(lib, bytes(out))
    assert rc == 0, lib.hjd_last_error()
    assert list(info16.qt_precision) == [1, 1, 1]
    np.testing.assert_array_equal(np.array(info16.qt), np.array(info8.qt))
    np.testing.assert_array_equal(coefs16, coefs8)


def test_bmp_header_matches_reference_layout(hjd):
    """hjd_bmp_header == the reference's bmp_create() (src/decoder.cpp:372-394):
    packed BITMAPFILEHEADER (14 B) + BITMAPINFOHEADER (40 B), 32 bpp, BI_RGB,
    negative height (top-down)."""
    import struct
    for w, h in ((313, 234), (1, 1), (3840, 2160)):
        size = 54 + w * h * 4
        exp = struct.pack("<HIHHI", 0x4D42, size, 0, 0, 54) + struct.pack("<IiiHHIIiiII", 40, w, -h, 1, 32, 0, 0, 0, 0,
                                                                           0, 0)
        assert hjd.bmp_header(w, h) == exp
    px = np.arange(12, dtype=np.uint32).reshape(3, 4)
    assert hjd.bmp_bytes(px) == hjd.bmp_header(4, 3) + px.astype("<u4").tobytes()


def test_bmp_files_open_in_pillow(hjd):
    """Both sinks' BMP files (the reference's 32-bpp BGRX layout and the
    24-bpp BGR24 extension, rows padded to 4 bytes) decode in an independent
    BMP reader to the intended RGB pixels."""
    import io
    from PIL import Image
    rng = np.random.default_rng(9)
    for w, h in ((1, 1), (5, 3), (13, 7), (64, 2)):
        rgb = rng.integers(0, 256, (h, w, 3), dtype=np.uint8)
        bgrx = (rgb[..., 2].astype(np.uint32) | (rgb[..., 1].astype(np.uint32) << 8) |
                (rgb[..., 0].astype(np.uint32) << 16))
        pitch = hjd.default_pitch(w, hjd.OUT_BGR24)
        rows = np.zeros((h, pitch), np.uint8)
        rows[:, :3 * w] = rgb[..., ::-1].reshape(h, 3 * w)
        for data in (hjd.bmp_bytes(bgrx), hjd.bmp_bytes(rows, width=w)):
            im = Image.open(io.BytesIO(data))
            assert im.size == (w, h)
            np.testing.assert_array_equal(np.asarray(im.convert("RGB")), rgb)
        assert len(hjd.bmp_bytes(rows, width=w)) == 54 + pitch * h
