"""GPU: the sampling extensions of SURVEY.md s8(f) rank 4 -- 4:2:2 (Y H2V1)
and one-component (gray) frames -- through every entry point: the fused
kernel (both input formats), the host-Huffman JPEG path, the stream, and the
GPU entropy decoder.

4:1:1 (Y H4V1) and 4:4:0 (Y H1V2) follow the same rules (test_411_440_jpeg_paths;
CPU side: tests/test_samplings.py).

The reference rejects these samplings (src/decoder.cpp:58-69), so there is no
reference output: the HIP path is pinned bit-exactly to the oracle's
restatement (oracle/oracle.c put_mcu: the reference's IDCT and colour
arithmetic, nearest horizontal chroma replication, gray = the conversion with
U = V = 0), and the host Huffman decode of these files is pinned to Pillow's
decoder in tests/test_jpeg_host.py::test_extension_samplings_decode.
"""
import numpy as np
import pytest

import oracle_py as O
from test_entropy_emulation import _pil
from test_gpu_parity import _decode, to_u32

pytestmark = pytest.mark.gpu

YUV422, GRAY, YUV411, YUV440 = 3, 4, 5, 6
EXT = [YUV422, GRAY, YUV411, YUV440]


@pytest.mark.parametrize("s", EXT)
@pytest.mark.parametrize("w,h", [(1, 1), (8, 8), (16, 8), (17, 9), (191, 8), (193, 9), (383, 17), (385, 16),
                                 (1920, 40), (2049, 31), (95, 16), (97, 33), (255, 8), (257, 17)])
def test_random_frames_vs_oracle(hjd, ctx, s, w, h):
    coefs, qt = O.synthetic_coefs(w, h, s, seed=w * 31 + h + s)
    px, _ = _decode(hjd, ctx, coefs, qt, w, h, s)
    np.testing.assert_array_equal(px, O.decode_q16(coefs, qt, w, h, s))
    if s == GRAY:
        b = px.view(np.uint8).reshape(h, w, 4)
        assert (b[..., 0] == b[..., 1]).all() and (b[..., 1] == b[..., 2]).all() and (b[..., 3] == 0).all()


@pytest.mark.parametrize("s", EXT)
def test_i32_natural_input(hjd, ctx, s):
    w, h = 777, 45
    coefs, qt = O.synthetic_coefs(w, h, s, seed=5)
    nat = O.dequant_natural(coefs, qt, s)
    px, _ = _decode(hjd, ctx, nat, None, w, h, s, fmt=1)
    np.testing.assert_array_equal(px, O.decode_q16(coefs, qt, w, h, s))


@pytest.mark.parametrize("s", EXT)
def test_no_writes_outside_frame(hjd, ctx, s):
    w, h = 45, 37
    coefs, qt = O.synthetic_coefs(w, h, s, seed=3)
    guard, pitch = 4096, 64
    px, full = _decode(hjd, ctx, coefs, qt, w, h, s, pitch_px=pitch, guard=guard, fill=0x5A5A5A5A)
    np.testing.assert_array_equal(px, O.decode_q16(coefs, qt, w, h, s))
    mask = np.ones(full.shape, bool)
    body = mask[guard // 4: guard // 4 + pitch * h].reshape(h, pitch)
    body[:, :w] = False
    assert (full[mask] == 0x5A5A5A5A).all()


def _corner_frame(w, h, s, seed):
    """int32 natural blocks: chroma blocks DC-only at the colour corners
    (U,V) = (-200,200), (-100,100) and (0,0) (IDCT of DC d*8 is d), luma blocks
    with a DC sweep over [-256,255] and random small AC, so the rare flagged
    path of every sampling meets luma values inside and outside [188,201]."""
    rng = np.random.default_rng(seed)
    nblk = O.frame_blocks(w, h, s)
    comp = O.block_components(s, nblk)
    blocks = np.zeros((nblk, 64), np.int32)
    corners = [(-200, 200), (-100, 100), (0, 0), (-200, 200)]
    ny = int((comp == 0).sum())
    blocks[comp == 0, 0] = 8 * rng.integers(-256, 256, ny)
    blocks[comp == 0, 1:10] = rng.integers(-40, 41, (ny, 9))
    mcu = np.arange(nblk) // {0: 3, 1: 6, 3: 4, 4: 1, 5: 6, 6: 4}[s]
    for c in (1, 2):
        sel = comp == c
        blocks[sel, 0] = [8 * corners[m % 4][c - 1] for m in mcu[sel]]
    return blocks


@pytest.mark.parametrize("s", [0, 1, YUV422, YUV411, YUV440])
def test_colour_corners_through_the_kernel(hjd, ctx, s):
    """The kernel's wave-uniform corrected-G path (hjd_device.hpp g_fix) on
    every sampling with chroma, against the oracle's literal fp64 conversion."""
    w, h = 260, 50
    nat = _corner_frame(w, h, s, seed=s + 17)
    px, _ = _decode(hjd, ctx, nat, None, w, h, s, fmt=1)
    np.testing.assert_array_equal(px, O.decode_i32(nat, w, h, s))


JPEGS = [
    dict(w=640, h=480, q=90, sub=1),
    dict(w=333, h=77, q=85, sub=1, restart_marker_blocks=2),
    dict(w=1921, h=1081, q=92, sub=1),
    dict(w=640, h=480, q=90, sub=0, gray=True),
    dict(w=333, h=77, q=70, sub=0, gray=True, restart_marker_blocks=7),
    dict(w=1999, h=999, q=95, sub=0, gray=True),
]


def _jpegs():
    out = []
    for i, kw in enumerate(JPEGS):
        kw = dict(kw)
        out.append(_pil(kw.pop("w"), kw.pop("h"), kw.pop("q"), kw.pop("sub"), seed=300 + i, **kw))
    return out


def _expected(hjd, data):
    coefs, info = hjd.decode_coefs(data)
    return O.decode_q16(coefs, np.array(info.qt), info.width, info.height, info.sampling), info


def test_host_huffman_jpeg_path(hjd, ctx):
    for i, data in enumerate(_jpegs()):
        exp, info = _expected(hjd, data)
        assert info.sampling == (GRAY if JPEGS[i].get("gray") else YUV422)
        out = hjd.decode_jpeg(ctx, data)
        np.testing.assert_array_equal(to_u32(out), exp, err_msg=str(JPEGS[i]))


@pytest.mark.parametrize("sub_bits", [64, 2048])
def test_gpu_entropy_decoder(hjd, ctx, sub_bits):
    """GPU Huffman + fused kernel on a batch mixing all four samplings (one
    pixel launch per sampling class)."""
    import torch
    datas = _jpegs() + [_pil(500, 300, 90, 2, seed=1), _pil(300, 200, 90, 0, seed=2)]
    exps, infos = zip(*[_expected(hjd, d) for d in datas])
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), sum(i.nblocks for i in infos), sub_bits) as gd:
        gd.decode(datas, outs)
        status = gd.sync()
    for k, (o, e) in enumerate(zip(outs, exps)):
        np.testing.assert_array_equal(to_u32(o), e, err_msg=f"file {k} S={sub_bits}")
    assert all(s & ~1 == 0 for s in status)


def test_stream_paths(hjd, ctx):
    """Host-Huffman stream and GPU-entropy stream on the extension files."""
    import torch
    datas = _jpegs()
    exps, infos = zip(*[_expected(hjd, d) for d in datas])
    maxblk = max(i.nblocks for i in infos)
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    with hjd.JpegStream(ctx, maxblk, nslots=2, nthreads=2) as st:
        for d, o in zip(datas, outs):
            st.submit(d, o)
        st.sync()
    for o, e in zip(outs, exps):
        np.testing.assert_array_equal(to_u32(o), e)
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    with hjd.GpuJpegStream(ctx, max_frames=3, max_scan_bytes=sum(map(len, datas)),
                           max_blocks=sum(i.nblocks for i in infos)) as gs:
        for d, o in zip(datas, outs):
            gs.submit(d, o)
        gs.sync()
    for o, e in zip(outs, exps):
        np.testing.assert_array_equal(to_u32(o), e)


# ---- BGR24 output (SURVEY.md s8(f) rank 4 "RGB24 writer") -------------------
def _bgr24(bgrx):
    """(H, W) BGRX words -> (H, 3W) bytes B, G, R."""
    return np.ascontiguousarray(bgrx).view(np.uint8).reshape(bgrx.shape[0], bgrx.shape[1], 4)[..., :3].reshape(
        bgrx.shape[0], -1)


def _decode24(hjd, ctx, coefs, qt, w, h, s, pitch, guard=64, fmt=0):
    import torch
    buf = torch.full((guard * 2 + pitch * h,), 0xA5, dtype=torch.uint8, device="cuda")
    spec = hjd.FrameSpec(w, h, s, out_offset=guard, out_pitch=pitch, qt_index=(0, 1, 2), out_format=hjd.OUT_BGR24)
    plan = hjd.Plan(ctx, [spec], fmt, qtables=qt if fmt == 0 else None)
    plan.launch(torch.from_numpy(np.ascontiguousarray(coefs)).cuda(), buf)
    torch.cuda.synchronize()
    full = buf.cpu().numpy()
    rows = full[guard:guard + pitch * h].reshape(h, pitch)
    # nothing outside the W x 3 bytes of each row (pads, guard bands) is written
    mask = np.ones(full.shape, bool)
    mask[guard:guard + pitch * h].reshape(h, pitch)[:, :3 * w] = False
    assert (full[mask] == 0xA5).all()
    return rows[:, :3 * w]


@pytest.mark.parametrize("s", [0, 1] + EXT)
@pytest.mark.parametrize("w,h,pad", [(1, 1, 0), (17, 9, 0), (129, 33, 4), (385, 16, 0), (1920, 40, 0),
                                     (2049, 31, 12)])
def test_bgr24_vs_oracle(hjd, ctx, s, w, h, pad):
    coefs, qt = O.synthetic_coefs(w, h, s, seed=w + 7 * h + s)
    pitch = hjd.default_pitch(w, hjd.OUT_BGR24) + pad
    got = _decode24(hjd, ctx, coefs, qt, w, h, s, pitch)
    np.testing.assert_array_equal(got, _bgr24(O.decode_q16(coefs, qt, w, h, s)))


def test_bgr24_i32_input_and_golden(hjd, ctx):
    """BGR24 from the idct.h-compat input on the reference's golden files ==
    the reference's BGRX without the pad byte."""
    for name in O.golden_cases():
        c = O.load_case(name)
        w, h, s = int(c["width"]), int(c["height"]), int(c["sampling"])
        nat = O.dequant_natural(c["coefs_q16"], c["qt"], s)
        got = _decode24(hjd, ctx, nat, None, w, h, s, hjd.default_pitch(w, hjd.OUT_BGR24), fmt=1)
        np.testing.assert_array_equal(got, _bgr24(c["bgrx"]), err_msg=name)


def test_bgr24_jpeg_paths_and_d2h_sink(hjd, ctx):
    """decode_jpeg, GpuDecoder and the GPU-entropy stream's device and host
    (D2H) sinks in BGR24, on golden and extension files; the 24-bpp BMP of the
    result opens in Pillow with the same pixels."""
    import io
    import os
    import torch
    from PIL import Image
    datas = [open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read() for n in O.golden_cases()] + _jpegs()
    exps, infos = zip(*[_expected(hjd, d) for d in datas])
    pitches = [hjd.default_pitch(i.width, hjd.OUT_BGR24) for i in infos]
    for d, e, i, p in zip(datas, exps, infos, pitches):
        out = hjd.decode_jpeg(ctx, d, out_format=hjd.OUT_BGR24)
        assert tuple(out.shape) == (i.height, p)
        rows = out.cpu().numpy()
        np.testing.assert_array_equal(rows[:, :3 * i.width], _bgr24(e))
    im = Image.open(io.BytesIO(hjd.bmp_bytes(rows, width=infos[-1].width)))
    np.testing.assert_array_equal(np.asarray(im.convert("RGB"))[..., ::-1].reshape(rows.shape[0], -1),
                                  _bgr24(exps[-1]))
    outs = [torch.full((i.height, p), 0xA5, dtype=torch.uint8, device="cuda") for i, p in zip(infos, pitches)]
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), sum(i.nblocks for i in infos), 1024) as gd:
        gd.set_output_format(hjd.OUT_BGR24)
        gd.decode(datas, outs)
        gd.sync()
    for o, e, i in zip(outs, exps, infos):
        np.testing.assert_array_equal(o.cpu().numpy()[:, :3 * i.width], _bgr24(e))
    dev_outs = [torch.full((i.height, p), 0xA5, dtype=torch.uint8, device="cuda") for i, p in zip(infos, pitches)]
    host_outs = [torch.full((i.height, p), 0xA5, dtype=torch.uint8).pin_memory() for i, p in zip(infos, pitches)]
    with hjd.GpuJpegStream(ctx, max_frames=4, max_scan_bytes=sum(map(len, datas)),
                           max_blocks=sum(i.nblocks for i in infos), out_format=hjd.OUT_BGR24) as gs:
        for k, d in enumerate(datas):
            gs.submit(d, dev_outs[k] if k % 2 else host_outs[k])
        gs.sync()
        with pytest.raises(Exception):
            gs.submit(datas[0], dev_outs[0])
            gs.set_output_format(hjd.OUT_BGRX)   # refused while a batch is open
        gs.sync()
    for k, (e, i) in enumerate(zip(exps, infos)):
        got = (dev_outs[k].cpu() if k % 2 else host_outs[k]).numpy()
        np.testing.assert_array_equal(got[:, :3 * i.width], _bgr24(e), err_msg=f"frame {k}")


def test_bgr24_host_huffman_stream(hjd, ctx):
    """hjd_stream (host Huffman || H2D || kernel) in BGR24, golden + extension files."""
    import os
    import torch
    datas = [open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read() for n in O.golden_cases()] + _jpegs()
    exps, infos = zip(*[_expected(hjd, d) for d in datas])
    outs = [torch.full((i.height, hjd.default_pitch(i.width, hjd.OUT_BGR24)), 0xA5, dtype=torch.uint8, device="cuda")
            for i in infos]
    with hjd.JpegStream(ctx, max(i.nblocks for i in infos), nslots=3, nthreads=2, out_format=hjd.OUT_BGR24) as st:
        for d, o in zip(datas, outs):
            st.submit(d, o)
        st.sync()
    for o, e, i in zip(outs, exps, infos):
        np.testing.assert_array_equal(o.cpu().numpy()[:, :3 * i.width], _bgr24(e))


def _jw_jpegs():
    """4:1:1 and 4:4:0 files (Pillow cannot write them): tests/jpeg_writer.py
    from synthetic coefficients, with and without DRI, edge geometries."""
    import io
    from PIL import Image
    import jpeg_writer as JW
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, format="JPEG", quality=90)
    src = b.getvalue()
    fac = {YUV411: [(4, 1), (1, 1), (1, 1)], YUV440: [(1, 2), (1, 1), (1, 1)]}
    out = []
    for s in (YUV411, YUV440):
        for w, h, dri in ((640, 480, 0), (333, 77, 2), (1921, 1081, 0), (1, 1, 0)):
            coefs, qt = O.synthetic_coefs(w, h, s, seed=w + s)
            out.append(JW.encode_frame(coefs, w, h, fac[s], qt, src, restart_interval=dri))
    return out


def test_411_440_jpeg_paths(hjd, ctx):
    """decode_jpeg, the host-Huffman stream, the GPU entropy decoder (in a
    batch mixing all six samplings) and the GPU-entropy stream on 4:1:1 and
    4:4:0 files: bit-exact to the oracle on the host-decoded coefficients."""
    import torch
    datas = _jw_jpegs()
    mixed = datas + _jpegs() + [_pil(500, 300, 90, 2, seed=1), _pil(300, 200, 90, 0, seed=2)]
    exps, infos = zip(*[_expected(hjd, d) for d in mixed])
    assert {i.sampling for i in infos} == {0, 1, YUV422, GRAY, YUV411, YUV440}
    for d, e in zip(datas, exps):
        np.testing.assert_array_equal(to_u32(hjd.decode_jpeg(ctx, d)), e)
    for sub_bits in (64, 2048):
        outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
        with hjd.GpuDecoder(ctx, len(mixed), sum(map(len, mixed)), sum(i.nblocks for i in infos), sub_bits) as gd:
            gd.decode(mixed, outs)
            status = gd.sync()
        for k, (o, e) in enumerate(zip(outs, exps)):
            np.testing.assert_array_equal(to_u32(o), e, err_msg=f"file {k} S={sub_bits}")
        assert all(s & ~1 == 0 for s in status)
    n = len(datas)
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos[:n]]
    with hjd.JpegStream(ctx, max(i.nblocks for i in infos[:n]), nslots=2, nthreads=2) as st:
        for d, o in zip(datas, outs):
            st.submit(d, o)
        st.sync()
    for o, e in zip(outs, exps):
        np.testing.assert_array_equal(to_u32(o), e)
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos[:n]]
    with hjd.GpuJpegStream(ctx, max_frames=3, max_scan_bytes=sum(map(len, datas)),
                           max_blocks=sum(i.nblocks for i in infos[:n])) as gs:
        for d, o in zip(datas, outs):
            gs.submit(d, o)
        gs.sync()
    for o, e in zip(outs, exps):
        np.testing.assert_array_equal(to_u32(o), e)
