"""GPU: JPEG bytes -> pixels through the host front end and the stream
pipeline (host Huffman || pinned H2D || fused kernel).  Golden files are
checked against the reference's BGRX; other files against the oracle applied
to the host-decoded coefficients (the Huffman stage itself is pinned to the
reference in tests/test_jpeg_host.py)."""
import io
import os

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def _pil(w, h, q, sub, seed, **kw):
    from PIL import Image
    rng = np.random.default_rng(seed)
    x = np.linspace(0, 255, w)[None, :, None]
    y = np.linspace(0, 255, h)[:, None, None]
    img = np.clip(x * [1, 0, 0.5] + y * [0, 1, 0.5] + rng.normal(0, 20, (h, w, 3)), 0, 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", quality=q, subsampling=sub, **kw)
    return b.getvalue()


def test_decode_jpeg_golden(hjd, ctx):
    import torch
    for name in O.golden_cases():
        data = open(os.path.join(O.GOLDEN, name + ".jpg"), "rb").read()
        out = hjd.decode_jpeg(ctx, data)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), O.load_case(name)["bgrx"])


@pytest.mark.parametrize("nslots,nthreads", [(2, 1), (3, 4), (8, 16)])
def test_stream_many_images(hjd, ctx, nslots, nthreads):
    import torch
    files = []
    for name in O.golden_cases():
        files.append((open(os.path.join(O.GOLDEN, name + ".jpg"), "rb").read(), O.load_case(name)["bgrx"]))
    rng = np.random.default_rng(nslots * 7 + nthreads)
    for i in range(12):
        w, h = int(rng.integers(1, 700)), int(rng.integers(1, 300))
        sub = int(rng.choice([0, 2]))
        kw = {"restart_marker_blocks": int(rng.integers(1, 9))} if i % 3 == 0 else {}
        data = _pil(w, h, int(rng.integers(30, 100)), sub, seed=i, **kw)
        coefs, info = hjd.decode_coefs(data)
        files.append((data, O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)))
    files = files * 2
    max_blocks = max(hjd.parse(d).nblocks for d, _ in files)
    outs = [torch.full(e.shape, -1, dtype=torch.int32, device="cuda") for _, e in files]
    with hjd.JpegStream(ctx, max_blocks, nslots=nslots, nthreads=nthreads) as st:
        for (d, _), o in zip(files, outs):
            st.submit(d, o)
        stats = st.sync()
    assert stats["images"] == len(files) and stats["kernel_launches"] == len(files)
    for (d, e), o in zip(files, outs):
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), e)


def test_stream_reports_bad_file_and_continues(hjd, ctx):
    import torch
    good = open(os.path.join(O.GOLDEN, "syn420_96x64_q90.jpg"), "rb").read()
    exp = O.load_case("syn420_96x64_q90")["bgrx"]
    bad = good[:200]   # truncated
    outs = [torch.zeros((64, 96), dtype=torch.int32, device="cuda") for _ in range(3)]
    st = hjd.JpegStream(ctx, 1024, nslots=2, nthreads=2)
    st.submit(good, outs[0]); st.submit(bad, outs[1]); st.submit(good, outs[2])
    with pytest.raises(Exception):
        st.sync()
    np.testing.assert_array_equal(outs[0].cpu().numpy().view(np.uint32), exp)
    np.testing.assert_array_equal(outs[2].cpu().numpy().view(np.uint32), exp)
    st.submit(good, outs[1])      # the stream stays usable after an error
    st.sync()
    np.testing.assert_array_equal(outs[1].cpu().numpy().view(np.uint32), exp)
    st.close()


def test_stream_truncated_scan_reported(hjd, ctx):
    """A file whose scan is cut short (the reference's "data incomplete",
    src/decoder.cpp:310-313) fails in the host-Huffman stream with that error;
    its output stays untouched, the files around it decode exactly, and so do
    later submits.  Cuts: half the scan with an EOI appended, and 90 % without
    one, of a 4:2:0, a 4:4:4 and a restart-interval file."""
    import torch
    names = ["JPEG_example_JPG_RIP_050", "syn444_64x40_q90", "syn420_160x48_q95_dri"]
    goods, bads = [], []
    for n in names:
        data = open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read()
        so = hjd.parse(data).scan_offset
        goods.append((data, O.load_case(n)["bgrx"]))
        bads.append(data[: so + (len(data) - 2 - so) // 2] + b"\xff\xd9")
        bads.append(data[: so + (len(data) - 2 - so) * 9 // 10])
    max_blocks = max(hjd.parse(d).nblocks for d, _ in goods)
    order = []   # good, bad, good, bad, ...
    for i, b in enumerate(bads):
        order.append(("good", goods[i % len(goods)]))
        order.append(("bad", (b, goods[(i // 2) % len(goods)][1].shape)))
    order.append(("good", goods[0]))
    outs = []
    for kind, (d, e) in order:
        shape = e.shape if kind == "good" else e
        outs.append(torch.full(shape, 0x5A5A5A5A, dtype=torch.int32, device="cuda"))
    with hjd.JpegStream(ctx, max_blocks, nslots=3, nthreads=4) as st:
        for (kind, (d, _)), o in zip(order, outs):
            st.submit(d, o)
        with pytest.raises(hjd._lib.HjdError, match="incomplete"):
            st.sync()
        for (kind, (d, e)), o in zip(order, outs):
            got = o.cpu().numpy().view(np.uint32)
            if kind == "good":
                np.testing.assert_array_equal(got, e)
            else:
                assert (got == 0x5A5A5A5A).all()
        again = torch.zeros(goods[1][1].shape, dtype=torch.int32, device="cuda")
        st.submit(goods[1][0], again)
        st.sync()
        np.testing.assert_array_equal(again.cpu().numpy().view(np.uint32), goods[1][1])


def test_stream_error_names_the_first_failing_job(hjd, ctx):
    """Two truncated files decoded as one worker's pair: the stream reports
    the first one's error (its MCU count), not the second's."""
    import torch
    a = open(os.path.join(O.GOLDEN, "JPEG_example_JPG_RIP_050.jpg"), "rb").read()   # 300 MCUs
    b = open(os.path.join(O.GOLDEN, "syn444_64x40_q90.jpg"), "rb").read()           # 40 MCUs
    cut = [d[: hjd.parse(d).scan_offset + (len(d) - hjd.parse(d).scan_offset) // 2] + b"\xff\xd9" for d in (a, b)]
    outs = [torch.zeros((234, 313), dtype=torch.int32, device="cuda"), torch.zeros((40, 64), dtype=torch.int32,
                                                                                     device="cuda")]
    with hjd.JpegStream(ctx, 2048, nslots=4, nthreads=1) as st:
        for d, o in zip(cut, outs):
            st.submit(d, o)
        with pytest.raises(hjd._lib.HjdError, match="of 300"):
            st.sync()


def test_4k_jpeg_end_to_end(hjd, ctx):
    """Config 5's first pool file: its host coefficients hash to the
    reference's mcu_data (tests/scale_pins.py), its pixels are the oracle's."""
    import torch
    import scale_pins as SP
    data = SP.generate_one("bench_pool_4k420_q90", 0)
    coefs, info = hjd.decode_coefs(data)
    rec = SP.manifest_scale()["bench_pool_4k420_q90"]["files"][0]
    assert SP.check_coefs(rec, data, coefs, info.qt, info.sampling) == "pinned"
    out = hjd.decode_jpeg(ctx, data)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), O.decode_q16(coefs, info.qt, 3840, 2160, 1))


def test_progressive_and_multiscan_files(hjd, ctx):
    """Progressive (SOF2) and multi-scan sequential files go through the host
    decoder into the same fused kernel: decode_jpeg and the stream pipeline
    give exactly the pixels of the baseline file with the same coefficients
    (tests/test_jpeg_multiscan.py pins the coefficients)."""
    import torch
    import jpeg_writer as JW
    files = []
    for i, (w, h, sub, kw) in enumerate([(333, 177, 2, {}), (96, 64, 0, {"restart_marker_blocks": 3}),
                                         (200, 120, 1, {}), (1, 1, 2, {})]):
        base = _pil(w, h, 85, sub, seed=40 + i, **kw)
        prog = _pil(w, h, 85, sub, seed=40 + i, progressive=True, **kw)
        c0, i0 = hjd.decode_coefs(base)
        exp = O.decode_q16(c0, i0.qt, w, h, i0.sampling)
        files += [(base, exp), (prog, exp)]
        ms, _ = JW.rewrite_scans(base, c0, [(0,), (2,), (1,)], 4)
        files.append((ms, exp))
    for d, e in files:
        out = hjd.decode_jpeg(ctx, d)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), e)
    max_blocks = max(hjd.parse(d).nblocks for d, _ in files)
    outs = [torch.full(e.shape, -1, dtype=torch.int32, device="cuda") for _, e in files]
    with hjd.JpegStream(ctx, max_blocks, nslots=3, nthreads=4) as st:
        for (d, _), o in zip(files, outs):
            st.submit(d, o)
        st.sync()
    for (d, e), o in zip(files, outs):
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), e)
