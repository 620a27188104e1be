"""CPU tests of the host decoder's multi-scan extensions (include/hjd_host.h):
progressive JPEG (SOF2) and sequential files with several scans.  The
reference decodes one interleaved baseline scan only (src/decoder.cpp:308-344),
so these are pinned by construction rather than by reference output:

* progressive: libjpeg (via Pillow) quantises the same image identically
  whatever the scan script, so a progressive file's coefficients must equal
  those of the baseline file made with the same settings -- exactly;
* multi-scan sequential: tests/jpeg_writer.py re-encodes a baseline file's
  coefficients with the file's own tables as non-interleaved / partly
  interleaved scans, in any component order, with or without DRI.
The baseline path itself is pinned to the reference in test_jpeg_host.py."""
import io

import numpy as np
import pytest

import jpeg_writer as JW
import oracle_py as O


def _image(w, h, seed=1, noise=20):
    rng = np.random.default_rng(seed)
    x = np.arange(w)[None, :]
    y = np.arange(h)[:, None]
    a = np.stack([x * 255 / w + 0 * y, y * 255 / h + 0 * x, (x + y) * 127 / (w + h) + 60], -1)
    return np.clip(a + rng.normal(0, noise, a.shape), 0, 255).astype(np.uint8)


def _pair(w, h, sub, mode, quality=85, noise=20, **kw):
    """(baseline bytes, progressive bytes) of one image, same settings."""
    from PIL import Image
    im = Image.fromarray(_image(w, h, noise=noise))
    if mode == "L":
        im = im.convert("L")
    out = []
    for prog in (False, True):
        b = io.BytesIO()
        im.save(b, format="JPEG", quality=quality, subsampling=sub, progressive=prog, **kw)
        out.append(b.getvalue())
    return out


@pytest.mark.parametrize("w,h,sub,mode,quality,kw", [
    (64, 48, 2, "RGB", 85, {}),
    (333, 177, 2, "RGB", 85, {}),
    (333, 177, 0, "RGB", 95, {}),
    (333, 177, 1, "RGB", 75, {}),
    (333, 177, 0, "L", 85, {}),
    (1, 1, 2, "RGB", 90, {}),
    (200, 120, 2, "RGB", 85, {"restart_marker_blocks": 3}),
    (201, 97, 0, "L", 50, {"restart_marker_rows": 1}),
    (1024, 700, 2, "RGB", 30, {}),       # long EOB runs at low quality
])
def test_progressive_equals_baseline(hjd, w, h, sub, mode, quality, kw):
    base, prog = _pair(w, h, sub, mode, quality, **kw)
    assert b"\xff\xc2" in prog
    c0, i0 = hjd.decode_coefs(base)
    c1, i1 = hjd.decode_coefs(prog)
    assert i1.process == 2 and not i1.single_scan
    assert i0.process == 0 and i0.single_scan
    assert (i1.width, i1.height, i1.sampling, i1.nblocks) == (i0.width, i0.height, i0.sampling, i0.nblocks)
    np.testing.assert_array_equal(i1.qt, i0.qt)
    np.testing.assert_array_equal(c1, c0)


def test_progressive_pixels_match_pillow(hjd):
    """Independent decoder check: host progressive decode + the oracle's pixel
    stage against Pillow's decode of the same progressive file (IDCT and
    chroma-filter differences only, as in test_extension_samplings_decode)."""
    from PIL import Image
    _, prog = _pair(96, 64, 2, "RGB", 90, noise=5)
    c, i = hjd.decode_coefs(prog)
    px = O.decode_q16(c, i.qt, i.width, i.height, i.sampling)
    bgr = px.view(np.uint8).reshape(64, 96, 4)[..., :3].astype(np.int32)
    ref = np.asarray(Image.open(io.BytesIO(prog)).convert("RGB"))[..., ::-1].astype(np.int32)
    d = np.abs(bgr - ref)
    assert d.mean() < 2.0 and d.max() <= 16, (d.mean(), d.max())


@pytest.mark.parametrize("scans", [
    [(0,), (1,), (2,)],
    [(0,), (1, 2)],
    [(2,), (0,), (1,)],
    [(1, 2), (0,)],
    [(2, 1, 0)],                         # one interleaved scan, components out of frame order
])
@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("dri", [0, 5])
def test_multiscan_sequential(hjd, scans, sub, dri):
    from PIL import Image
    w, h = 133, 77
    b = io.BytesIO()
    Image.fromarray(_image(w, h)).save(b, format="JPEG", quality=85, subsampling=sub)
    base = b.getvalue()
    c0, i0 = hjd.decode_coefs(base)
    data, expect = JW.rewrite_scans(base, c0, scans, dri)
    c1, i1 = hjd.decode_coefs(data)
    assert i1.single_scan == (len(scans) == 1)
    assert i1.restart_interval == dri
    np.testing.assert_array_equal(c1, expect)
    # MCU-padding blocks a non-interleaved scan does not code lie outside the image
    np.testing.assert_array_equal(O.decode_q16(c1, i1.qt, w, h, i1.sampling),
                                  O.decode_q16(c0, i0.qt, w, h, i0.sampling))


def test_multiscan_gray_and_sof1(hjd):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(_image(77, 45)).convert("L").save(b, format="JPEG", quality=80)
    base = b.getvalue()
    c0, _ = hjd.decode_coefs(base)
    data, expect = JW.rewrite_scans(base, c0, [(0,)], 7)
    np.testing.assert_array_equal(hjd.decode_coefs(data)[0], expect)
    # SOF1 (extended sequential, 8-bit Huffman) decodes like SOF0
    ext = bytearray(base)
    ext[ext.index(b"\xff\xc0") + 1] = 0xC1
    c1, i1 = hjd.decode_coefs(bytes(ext))
    assert i1.process == 1
    np.testing.assert_array_equal(c1, c0)


def test_gpu_entropy_emulation_rejects_progressive(hjd):
    """The GPU entropy decoder takes sequential scans; a progressive file fails
    loudly there (and decodes on the host path)."""
    _, prog = _pair(32, 32, 2, "RGB")
    with pytest.raises(RuntimeError, match="progressive"):
        hjd.emulate_entropy(prog)


@pytest.mark.parametrize("scans", [
    [(0,), (1,), (2,)],
    [(0,), (1, 2)],
    [(2,), (0,), (1,)],
    [(1, 2), (0,)],
])
@pytest.mark.parametrize("sub", [0, 1, 2])
@pytest.mark.parametrize("dri", [0, 4])
@pytest.mark.parametrize("spec", ["0", "1"])
def test_gpu_entropy_emulation_multiscan(hjd, monkeypatch, scans, sub, dri, spec):
    """The GPU entropy algorithm (host emulation of the kernels) on sequential
    files with several scans: each scan is an entropy frame of its own
    (kLayoutMcu for interleaved scans, kLayoutRaster for one component) and
    all of them write the file's MCU-major coefficients -- exactly the host
    decoder's, padding blocks zero; round-based and speculative sync, short
    subsequences so that every scan spans several groups."""
    from PIL import Image
    monkeypatch.setenv("HJD_SYNC_SPEC", spec)
    w, h = 181, 97
    b = io.BytesIO()
    Image.fromarray(_image(w, h, seed=sub + 3)).save(b, format="JPEG", quality=90, subsampling=sub)
    base = b.getvalue()
    c0, _ = hjd.decode_coefs(base)
    data, expect = JW.rewrite_scans(base, c0, scans, dri)
    for sub_bits in (48, 0):
        c1, status = hjd.emulate_entropy(data, sub_bits)
        np.testing.assert_array_equal(c1, expect, err_msg=f"S={sub_bits}")
        assert status & ~1 == 0


def test_gpu_entropy_emulation_multiscan_damaged(hjd):
    """A damaged later scan is reported, never decoded silently as valid."""
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(_image(120, 80)).save(b, format="JPEG", quality=85, subsampling=2)
    base = b.getvalue()
    c0, _ = hjd.decode_coefs(base)
    data, expect = JW.rewrite_scans(base, c0, [(0,), (1,), (2,)], 0)
    last = data.rindex(b"\xff\xda")
    bad = bytearray(data)
    bad[last + 30:last + 50] = b"\x00" * 20
    try:
        c1, _ = hjd.emulate_entropy(bytes(bad))
    except RuntimeError:
        return                                  # reported as corrupt
    # accepted: then the host decoder accepts it too, with the same coefficients
    ref, _ = hjd.decode_coefs(bytes(bad))
    np.testing.assert_array_equal(c1, ref)


@pytest.mark.parametrize("marker", [0xC3, 0xC9, 0xCA])   # lossless, arithmetic
def test_rejects_other_processes(hjd, marker):
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(_image(16, 16)).save(b, format="JPEG")
    data = bytearray(b.getvalue())
    data[data.index(b"\xff\xc0") + 1] = marker
    with pytest.raises(RuntimeError):
        hjd.decode_coefs(bytes(data))


def test_bad_progressive_scan_header_rejected(hjd):
    _, prog = _pair(32, 32, 2, "RGB")
    data = bytearray(prog)
    sos = data.index(b"\xff\xda")                 # first scan: DC, Ss=Se=0
    ns = data[sos + 4]
    data[sos + 5 + 2 * ns + 1] = 5                # Se=5 in a DC scan: illegal
    with pytest.raises(RuntimeError, match="progressive scan"):
        hjd.decode_coefs(bytes(data))


def test_corrupt_progressive_never_crashes(hjd):
    """Random byte damage inside the scans: every decode returns (ok or an
    error), none reads or writes out of bounds (a crash fails the run)."""
    _, prog = _pair(160, 96, 2, "RGB", 80, restart_marker_blocks=4)
    rng = np.random.default_rng(5)
    first = prog.index(b"\xff\xda")
    errors = 0
    for _ in range(300):
        data = bytearray(prog)
        for _ in range(rng.integers(1, 6)):
            data[rng.integers(first, len(data))] = rng.integers(0, 256)
        if rng.integers(0, 4) == 0:
            data = data[: rng.integers(first, len(data))]
        try:
            hjd.decode_coefs(bytes(data))
        except RuntimeError:
            errors += 1
    assert errors > 0


def test_host_decoder_asan_fuzz():
    """The host decoder (baseline, progressive and multi-scan paths) built with
    AddressSanitizer + UBSan and fed 4,500 damaged files (tools/fuzz)."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run(["bash", os.path.join(root, "tools", "fuzz", "run.sh"), "300"], capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    assert "mutants decoded" in p.stdout
