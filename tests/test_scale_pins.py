"""The host Huffman decoder pinned to the compiled reference at config-5
scale: the reference's own mcu_data (src/decoder.cpp:
338-342) hashed for seeded 4K q90 4:2:0 (config 5's whole 64-file pool) and
4:4:4, FHD q50, 2049x1111 q30 and 1001x777 q100 optimised-table files
(tests/scale_pins.py, manifest.json "scale", written by
tests/golden/make_golden.py from oracle/_ref/libref.so).

And the reference's restart-marker read-boundary defect (src/decoder.cpp:
122-146, INTEGRATION.md "behaviour fixed"): a FHD q50 DRI-5 file whose RST7
0xFF is the last byte of the reference's 65th 2,048-byte read.  The reference
(and the drop-in, which keeps its front end) rejects it; this library's host
and GPU-algorithm decoders give the pinned coefficients.
"""
import os

import numpy as np
import pytest

import oracle_py as O
import scale_pins as SP


@pytest.fixture(scope="module")
def lib():
    from ocljpegdecoder_amd import _lib
    return _lib.load()


def _status(name, hjd):
    rec = SP.manifest_scale()[name]
    out = []
    for jpg, frec in zip(SP.generate(name), rec["files"]):
        coefs, info = hjd.decode_coefs(jpg)
        out.append(SP.check_coefs(frec, jpg, coefs, info.qt, info.sampling))
    return out


@pytest.mark.parametrize("name", [n for n in SP.SCALE_CASES if n != "bench_pool_4k420_q90"])
def test_scale_case_pinned(hjd, name):
    assert set(_status(name, hjd)) == {"pinned"}


def test_bench_pool_pinned(hjd):
    """All 64 files of config 5's pool (bench.encode_pool seed 7919)."""
    st = _status("bench_pool_4k420_q90", hjd)
    assert len(st) == 64 and set(st) == {"pinned"}, st


def test_pair_decode_and_bytewise_reader_pinned(lib, hjd):
    """The pair decode (hjd_jpeg_decode_batch: two files per thread) and the
    byte-wise reader give the pinned coefficients on 4K files too."""
    files = SP.generate("bench_pool_4k420_q90")[:4] + SP.generate("4k444_q90")
    recs = SP.manifest_scale()["bench_pool_4k420_q90"]["files"][:4] + SP.manifest_scale()["4k444_q90"]["files"]
    got = hjd.decode_coefs_batch(files, nthreads=2)
    infos = [hjd.parse(f) for f in files]
    for f, r, c, i in zip(files, recs, got, infos):
        assert SP.check_coefs(r, f, c[: i.nblocks], i.qt, i.sampling) == "pinned"
    lib.hjd_debug_host_reader(1)
    try:
        c, i = hjd.decode_coefs(files[-1])
    finally:
        lib.hjd_debug_host_reader(0)
    assert SP.check_coefs(recs[-1], files[-1], c, i.qt, i.sampling) == "pinned"


@pytest.mark.skipif(not O.ref_available(), reason="needs oracle/_ref/libref.so (make -C oracle)")
@pytest.mark.parametrize("name", ["fhd420_q50", "odd2049x1111_q30", "q100_opt_1001x777"])
def test_live_reference(hjd, name):
    """Live: the reference's mcu_data equals the host decoder's coefficients,
    dequantised to natural order (no hash in between)."""
    from test_truncation import _ref_decode
    jpg = SP.generate(name)[0]
    ok, cap = _ref_decode(jpg)
    assert ok
    coefs, info = hjd.decode_coefs(jpg)
    np.testing.assert_array_equal(O.dequant_natural(coefs, np.array(info.qt), info.sampling), cap)


def _dri_case(hjd):
    rec = SP.manifest_scale()["dri_read_boundary"]
    b = rec["base"]
    base = SP.encode_jpeg(SP.synthetic_rgb(b["w"], b["h"], b["seed"]), b["quality"], b["subsampling"])
    coefs, info = hjd.decode_coefs(base)
    pin = {"jpeg_sha256": rec["base_jpeg_sha256"], "coefs_q16_sha256": rec["coefs_q16_sha256"],
           "mcu_data_sha256": rec["mcu_data_sha256"]}
    assert SP.check_coefs(pin, base, coefs, info.qt, info.sampling) == "pinned"
    dri = SP.dri_file(base, coefs)
    assert SP.sha(dri) == rec["jpeg_sha256"]
    return rec, dri, coefs, info


def test_dri_read_boundary_host_decoders(lib, hjd):
    """Both host readers, the pair decode and the GPU entropy algorithm decode
    the DRI-5 file to the pinned coefficients; the RST the reference loses is
    where the fixture says (its 0xFF ends a 2,048-byte read)."""
    rec, dri, coefs, info = _dri_case(hjd)
    so = hjd.parse(dri).scan_offset
    ff = [i for i in range(so, len(dri) - 1) if dri[i] == 0xFF and 0xD0 <= dri[i + 1] <= 0xD7]
    assert (ff[807] - so + 1) % 2048 == 0 and dri[ff[807] + 1] == 0xD7
    for mode in (0, 1):
        lib.hjd_debug_host_reader(mode)
        try:
            got, gi = hjd.decode_coefs(dri)
        finally:
            lib.hjd_debug_host_reader(0)
        assert gi.restart_interval == 5
        np.testing.assert_array_equal(got, coefs)
    pair = hjd.decode_coefs_batch([dri, dri], nthreads=1)
    np.testing.assert_array_equal(pair[0], coefs)
    np.testing.assert_array_equal(pair[1], coefs)
    emu, status = hjd.emulate_entropy(dri, 256)
    assert status & ~1 == 0
    np.testing.assert_array_equal(emu, coefs)


@pytest.mark.skipif(not O.ref_available(), reason="needs oracle/_ref/libref.so (make -C oracle)")
def test_dri_read_boundary_reference_rejects(hjd):
    from test_truncation import _ref_decode
    rec, dri, _, _ = _dri_case(hjd)
    ok, _ = _ref_decode(dri)
    assert not ok
    assert "expected RST7 (interval = 5; 4040/8160 mcu)" in rec["reference_log"]


# ---- GPU ---------------------------------------------------------------------
@pytest.mark.gpu
def test_dri_read_boundary_on_gpu(hjd, ctx):
    """Host Huffman + fused kernel (decode_jpeg) and the GPU entropy decoder
    give the oracle's pixels of the pinned coefficients."""
    import torch
    rec, dri, coefs, info = _dri_case(hjd)
    exp = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
    out = hjd.decode_jpeg(ctx, dri)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
    o2 = torch.full((info.height, info.width), -1, dtype=torch.int32, device="cuda")
    with hjd.GpuDecoder(ctx, 1, len(dri), info.nblocks) as gd:
        gd.decode([dri], [o2])
        gd.sync()
    np.testing.assert_array_equal(o2.cpu().numpy().view(np.uint32), exp)


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(os.path.join(O.REPO, "oracle", "_ref", "ref_dropin")),
                    reason="oracle/_ref/ref_dropin not built")
def test_dri_read_boundary_dropin_keeps_reference_behaviour(hjd):
    """The drop-in is the reference's own front end (parser, read_more_data,
    Huffman) over libhjd.so's idct.h: on this file it fails exactly as the
    reference does, before any idct.h call decodes pixels."""
    import shutil
    import subprocess
    import tempfile
    rec, dri, _, _ = _dri_case(hjd)
    tmp = tempfile.mkdtemp(prefix="hjd_dropin_dri_")
    try:
        with open(os.path.join(tmp, "in.jpg"), "wb") as f:
            f.write(dri)
        r = subprocess.run([os.path.join(O.REPO, "oracle", "_ref", "ref_dropin"), "in.jpg"], cwd=tmp,
                           capture_output=True, text=True, timeout=120)
        assert "expected RST7 (interval = 5; 4040/8160 mcu)" in r.stdout, r.stdout[-2000:]
        assert not os.path.exists(os.path.join(tmp, "m:\\output.bmp"))
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
