"""GPU: sequential JPEGs with several scans through the device entropy decoder
(hjd_gdec / hjd_gstream; DESIGN.md s10 "Several scans").  An extension: the
reference decodes one interleaved baseline scan only (src/decoder.cpp:308-344),
so these are pinned by construction -- tests/jpeg_writer.py re-encodes a
baseline file's coefficients as non-interleaved / partly interleaved scans
with the file's own tables, and every path must return exactly those
coefficients (MCU-padding blocks no scan codes read as zeros, as the host
decoder's), and the oracle's pixels of them."""
import functools

import numpy as np
import pytest

import jpeg_writer as JW
import oracle_py as O
from test_entropy_emulation import _pil

pytestmark = pytest.mark.gpu

SPLITS = [[(0,), (1,), (2,)], [(0,), (1, 2)], [(2,), (0,), (1,)], [(1, 2), (0,)], [(2, 1, 0)]]


def _multiscan(w, h, sub, scans, dri, seed, q=85):
    base = _pil(w, h, q, sub, seed=seed)
    import ocljpegdecoder_amd as hjd
    c0, _ = hjd.decode_coefs(base)
    data, expect = JW.rewrite_scans(base, c0, scans, dri)
    return data, expect


@functools.lru_cache(maxsize=1)
def _cases():
    out = []
    for k, scans in enumerate(SPLITS):
        for sub in (0, 1, 2):
            dri = 0 if (k + sub) % 2 else 3 + k
            w, h = 97 + 61 * k, 43 + 29 * sub
            out.append(_multiscan(w, h, sub, scans, dri, seed=10 * k + sub))
    return tuple(out)


def _decode_coefs(hjd, ctx, datas, sub_bits=0, max_frames=None, pinned=False):
    import torch
    infos = [hjd.parse(d) for d in datas]
    total = sum(i.nblocks for i in infos)
    coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")   # padding blocks must be zeroed
    src = [hjd.pinned_bytes(d) for d in datas] if pinned else datas
    with hjd.GpuDecoder(ctx, max_frames or len(datas), sum(len(d) for d in datas), total, sub_bits) as gd:
        offs = gd.decode_coefs(src, coefs)
        status = gd.sync()
    host = coefs.cpu().numpy()
    return [host[o:o + i.nblocks] for o, i in zip(offs, infos)], status


@pytest.mark.parametrize("sub_bits", [64, 1024, 0])
def test_multiscan_coefficients(hjd, ctx, sub_bits):
    cases = list(_cases())
    # single-scan files in the same batch keep their own path
    singles = [_pil(160, 90, 90, 2, seed=77), _pil(33, 17, 90, 0, seed=78, restart_marker_blocks=1)]
    datas = [d for d, _ in cases] + singles
    expects = [e for _, e in cases] + [hjd.decode_coefs(d)[0] for d in singles]
    got, status = _decode_coefs(hjd, ctx, datas, sub_bits)
    for i, (g, e, s) in enumerate(zip(got, expects, status)):
        np.testing.assert_array_equal(g, e, err_msg=f"file {i} S={sub_bits}")
        assert s & ~1 == 0, (i, s)


def test_restart_every_block_fits_exact_capacity(hjd, ctx):
    """a non-interleaved scan with Ri = 1 (and a gray file with
    Ri = 1) has one restart interval per BLOCK; a decoder sized by the
    batch's exact block count (what hjd_gdec_create documents as enough) must
    take it."""
    data, expect = _multiscan(200, 120, 1, SPLITS[0], 1, seed=123)
    gray = _pil(96, 40, 90, 0, seed=124, gray=True, restart_marker_blocks=1)
    datas = [data, gray]
    expects = [expect, hjd.decode_coefs(gray)[0]]
    got, status = _decode_coefs(hjd, ctx, datas)
    for i, (g, e, st) in enumerate(zip(got, expects, status)):
        np.testing.assert_array_equal(g, e, err_msg=f"file {i}")
        assert st & ~1 == 0, (i, st)


def test_multiscan_pinned_inputs_take_host_destuff(hjd, ctx):
    """Pinned inputs normally reach the GPU raw; a multi-scan file's scans are
    found and destuffed on the host instead, in the same batch."""
    cases = list(_cases()[:6])
    singles = [_pil(300, 200, 90, 2, seed=91)]
    datas = [d for d, _ in cases] + singles
    expects = [e for _, e in cases] + [hjd.decode_coefs(singles[0])[0]]
    got, status = _decode_coefs(hjd, ctx, datas, pinned=True)
    for i, (g, e) in enumerate(zip(got, expects)):
        np.testing.assert_array_equal(g, e, err_msg=f"file {i}")


@pytest.mark.parametrize("scans", [SPLITS[0], SPLITS[3]])
def test_multiscan_latency_decoder(hjd, ctx, scans):
    """A one-frame decoder (speculative sync) on a larger
    multi-scan file: every scan is an entropy frame of its own."""
    d, e = _multiscan(640, 360, 2, scans, 0, seed=5, q=90)
    got, status = _decode_coefs(hjd, ctx, [d], max_frames=1)
    np.testing.assert_array_equal(got[0], e)
    assert status[0] & ~1 == 0


def test_multiscan_pixels_match_oracle(hjd, ctx):
    import torch
    cases = list(_cases()[::2])
    datas = [d for d, _ in cases]
    infos = [hjd.parse(d) for d in datas]
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), sum(i.nblocks for i in infos)) as gd:
        gd.decode(datas, outs)
        gd.sync()
    for (d, e), i, o in zip(cases, infos, outs):
        exp = O.decode_q16(e, i.qt, i.width, i.height, i.sampling)
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


def test_multiscan_gstream(hjd, ctx):
    """GPU-entropy stream with single- and multi-scan files interleaved,
    through rotating batches of 3."""
    import torch
    cases = list(_cases())
    singles = [(_pil(200 + 7 * k, 100, 90, k % 3, seed=200 + k), None) for k in range(5)]
    files = []
    for k in range(max(len(cases), len(singles))):
        if k < len(cases):
            files.append(cases[k])
        if k < len(singles):
            d = singles[k][0]
            files.append((d, hjd.decode_coefs(d)[0]))
    infos = [hjd.parse(d) for d, _ in files]
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    cap_bytes = 3 * max(len(d) for d, _ in files) + (1 << 16)
    cap_blocks = 3 * max(i.nblocks for i in infos)
    with hjd.GpuJpegStream(ctx, 3, cap_bytes, cap_blocks, nslots=2, nthreads=4) as st:
        for (d, _), o in zip(files, outs):
            st.submit(d, o)
        stats = st.sync()
    assert stats["images"] == len(files)
    for (d, e), i, o in zip(files, infos, outs):
        exp = O.decode_q16(e, i.qt, i.width, i.height, i.sampling)
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


def test_multiscan_corrupt_scan_reported(hjd, ctx):
    """Damage in a later scan is reported for its file (the scan's status is
    folded into the file's), not silently decoded."""
    import torch
    d, e = _multiscan(200, 120, 2, SPLITS[0], 0, seed=9)
    info = hjd.parse(d)
    b = bytearray(d)
    last_sos = bytes(b).rindex(b"\xff\xda")
    b[last_sos + 40: last_sos + 60] = b"\x00" * 20        # wipe part of the last scan's data
    bad = bytes(b)
    coefs = torch.zeros((2 * info.nblocks, 64), dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, 2, 2 * len(d), 2 * info.nblocks) as gd:
        offs = gd.decode_coefs([d, bad], coefs)
        status = gd.sync(raise_on_error=False)
    assert status[0] & ~1 == 0
    host = coefs.cpu().numpy()
    np.testing.assert_array_equal(host[offs[0]:offs[0] + info.nblocks], e)
    ref_ok = True
    try:
        ref, _ = hjd.decode_coefs(bad)
        ref_ok = np.array_equal(ref, host[offs[1]:offs[1] + info.nblocks])
    except Exception:
        ref_ok = False
    # either the host decoder also accepts the damaged file and both agree, or the GPU flags it
    assert ref_ok or status[1] & ~1 != 0
