"""Truncated and incomplete scans (the reference's "data incomplete" rejection,
src/decoder.cpp:310-313; load_jpg then stops before decode_mcu_data,
src/parser.cpp:384-388).

The host Huffman decoder -- both of its readers, alone and in the two-file
pair decode -- and the GPU entropy algorithm (its host emulation) must reject
a file whose scan ends before its last MCU, and decode exactly the
reference's coefficients when it accepts.  Cut points: every 2 % of the scan
plus the last 24 bytes one by one, with and without an appended EOI.

One documented divergence ("behaviour fixed"): the reference
checks for the end of its data before each component except the first, never
after the last one, so a file cut inside the LAST MCU's LAST component is
decoded there from whatever its bit buffer holds past the data (stale memory).
This library rejects such a file.  The live comparison accepts exactly that
case and checks it is that case: the error names the last MCU, and the
reference's output equals the uncut file's in every other block.
"""
import ctypes
import os
import shutil
import tempfile

import numpy as np
import pytest

import oracle_py as O
from test_jpeg_host import _pil_jpeg, decode
from test_jpeg_host_pair import _batch

FILES = ["JPEG_example_JPG_RIP_050", "syn444_64x40_q90", "syn420_160x48_q95_dri", "syn444_odd_41x23_q75",
         "syn420_80x80_q50_opt"]


@pytest.fixture(scope="module")
def lib():
    from ocljpegdecoder_amd import _lib
    return _lib.load()


def _golden(name):
    return open(os.path.join(O.GOLDEN, name + ".jpg"), "rb").read()


def cut_files(data: bytes, scan_offset: int):
    """(label, bytes) of every cut: each 2 % of the scan and the last 24 bytes
    before the EOI, each with and without an appended EOI."""
    end = len(data) - 2
    cuts = sorted({scan_offset + (end - scan_offset) * p // 100 for p in range(0, 100, 2)} |
                  set(range(max(scan_offset, end - 24), end)))
    for c in cuts:
        yield f"cut{c}", data[:c]
        yield f"cut{c}+EOI", data[:c] + b"\xff\xd9"


def host_status(lib, data: bytes):
    """(rc, error text, coefficients, info) from the de-stuffed reader and from
    the byte-wise reader."""
    out = []
    for mode in (0, 1):
        lib.hjd_debug_host_reader(mode)
        try:
            rc, info, coefs = decode(lib, data)
            out.append((rc, lib.hjd_last_error() if rc else b"", coefs, info))
        finally:
            lib.hjd_debug_host_reader(0)
    return out


def emulated_ok(hjd, data: bytes) -> bool:
    try:
        _, status = hjd.emulate_entropy(data, 256)
    except Exception:
        return False
    return not (status & ~1)


@pytest.mark.parametrize("name", FILES)
def test_cut_files_rejected_by_every_path(lib, hjd, name):
    """No reference needed: every cut is rejected by both host readers, by the
    pair decode and by the GPU entropy algorithm, with the same error text
    from the two readers; the uncut file decodes to the golden coefficients."""
    data = _golden(name)
    info = hjd.parse(data)
    ncut = 0
    for label, d in cut_files(data, info.scan_offset):
        (r0, e0, _, _), (r1, e1, _, _) = host_status(lib, d)
        assert r0 != 0 and r1 != 0, (label, r0, r1)
        assert e0 == e1, (label, e0, e1)
        assert b"incomplete" in e0 or b"corrupt" in e0 or b"expected RST" in e0, (label, e0)
        status, _ = _batch(lib, [d, d], max(info.nblocks, 1))
        assert status[0] != 0 and status[1] != 0, label
        assert not emulated_ok(hjd, d), label
        ncut += 1
    assert ncut >= 100
    rc, _, coefs = decode(lib, data)
    assert rc == 0
    np.testing.assert_array_equal(coefs, O.load_case(name)["coefs_q16"])


def test_truncated_4k_scale_file(lib, hjd):
    """A config-5 sized scan (3840x2160 4:2:0 q90, one restart-free scan) cut
    at 25/50/75/99 %: the pair decode and both readers reject it; the error
    names an MCU near the cut, not the end of the frame."""
    from test_jpeg_host import _pil_smooth
    data, _ = _pil_smooth(3840, 2160, 90, "RGB", 2, seed=5)
    info = hjd.parse(data)
    nmcu = ((3840 + 15) // 16) * ((2160 + 15) // 16)
    for frac in (0.25, 0.5, 0.75, 0.99):
        c = info.scan_offset + int((len(data) - 2 - info.scan_offset) * frac)
        d = data[:c] + b"\xff\xd9"
        res = host_status(lib, d)
        for rc, err, _, _ in res:
            assert rc != 0 and b"incomplete" in err, (frac, err)
            m = int(err.split(b"(MCU ")[1].split(b" ")[0])
            assert abs(m / nmcu - frac) < 0.1, (frac, m)
        status, _ = _batch(lib, [d, data], info.nblocks)
        assert status[0] != 0 and status[1] == 0


def test_vacuous_truncation_case_now_rejected(lib):
    """The case tests/test_jpeg_host.py once accepted either way: Pillow 32x32
    q90 cut at half its bytes."""
    good = _pil_jpeg(32, 32, 90, 2)
    assert decode(lib, good)[0] == 0
    assert decode(lib, good[: len(good) // 2])[0] != 0
    assert decode(lib, good[: len(good) // 2] + b"\xff\xd9")[0] != 0


def test_spare_byte_before_rst_rejected(lib, hjd):
    """The reference reads the byte after an interval's last bits as the RSTn
    marker (src/decoder.cpp:295-302): a whole extra byte in front of the
    marker is a mismatch there, and here (both readers, the GPU algorithm)."""
    data = bytearray(_golden("syn420_160x48_q95_dri"))
    at = data.index(b"\xff\xd0")
    bad = bytes(data[:at] + b"\x5a" + data[at:])
    for rc, err, _, _ in host_status(lib, bad):
        assert rc != 0 and b"expected RST0" in err, err
    assert not emulated_ok(hjd, bad)


# ---- live comparison with the compiled reference (this container only) ------
def _ref_decode(data: bytes):
    """Run the reference's load_jpg on `data` in a forked child (it may abort on
    a damaged file: vassert).  Returns (accepted, mcu_data or None)."""
    ref = O.ref()
    ref.ref_load_jpg.argtypes = [ctypes.c_char_p] * 3
    tmp = tempfile.mkdtemp(prefix="hjd_trunc_")
    try:
        path = os.path.join(tmp, "in.jpg")
        with open(path, "wb") as f:
            f.write(data)
        pid = os.fork()
        if pid == 0:   # child: the reference prints its log on stdout
            try:
                os.chdir(tmp)
                os.dup2(os.open(os.devnull, os.O_WRONLY), 1)
                ref.ref_load_jpg(path.encode(), b"cap.bin", None)
            finally:
                os._exit(0)
        _, st = os.waitpid(pid, 0)
        # load_jpg returns true whatever happened: the BMP is written only after
        # decode_huffman_data and decode_mcu_data both succeeded
        ok = st == 0 and os.path.exists(os.path.join(tmp, "m:\\output.bmp"))
        cap = np.fromfile(os.path.join(tmp, "cap.bin"), np.int32).reshape(-1, 64) if ok else None
        return ok, cap
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


@pytest.mark.skipif(not O.ref_available(), reason="needs oracle/_ref/libref.so (make -C oracle)")
@pytest.mark.parametrize("name", FILES)
def test_cut_sweep_matches_reference(lib, hjd, name):
    data = _golden(name)
    info = hjd.parse(data)
    full = O.dequant_natural(O.load_case(name)["coefs_q16"], O.load_case(name)["qt"], info.sampling)
    nmcu = info.mcu_w * info.mcu_h
    stats = {"both_reject": 0, "both_accept": 0, "last_component": 0}
    for label, d in list(cut_files(data, info.scan_offset)) + [("uncut", data), ("no-EOI", data[:-2])]:
        ref_ok, cap = _ref_decode(d)
        (rc, err, coefs, hinfo), _ = host_status(lib, d)
        if not ref_ok:
            assert rc != 0, label
            stats["both_reject"] += 1
        elif rc == 0:
            np.testing.assert_array_equal(O.dequant_natural(coefs, np.array(hinfo.qt), hinfo.sampling), cap,
                                          err_msg=label)
            stats["both_accept"] += 1
        else:
            # the documented case: the cut lies in the last component of the
            # last MCU, which the reference decodes from past its data
            assert f"(MCU {nmcu - 1} of {nmcu})".encode() in err, (label, err)
            np.testing.assert_array_equal(cap[:-1], full[:-1], err_msg=label)
            stats["last_component"] += 1
    assert stats["both_accept"] >= 2 and stats["both_reject"] >= 90, stats


def _with_com_after_scan(data: bytes) -> bytes:
    """A COM segment between the scan and EOI (legal: T.81 B.2.4.5 tables/misc.)."""
    assert data[-2:] == b"\xff\xd9"
    return data[:-2] + b"\xff\xfe\x00\x06test" + b"\xff\xd9"


@pytest.mark.parametrize("name", FILES)
def test_marker_after_scan_decodes(lib, hjd, name):
    """A marker segment after the scan ends the entropy data: both readers, the
    pair decode and the GPU entropy algorithm give the golden coefficients."""
    d = _with_com_after_scan(_golden(name))
    exp = O.load_case(name)["coefs_q16"]
    for rc, err, coefs, _ in host_status(lib, d):
        assert rc == 0, err
        np.testing.assert_array_equal(coefs, exp)
    status, outs = _batch(lib, [d, d], exp.shape[0])
    assert list(status) == [0, 0]
    np.testing.assert_array_equal(outs[1], exp)
    emu, st = hjd.emulate_entropy(d, 256)
    assert st & ~1 == 0
    np.testing.assert_array_equal(emu, exp)


@pytest.mark.skipif(not O.ref_available(), reason="needs oracle/_ref/libref.so (make -C oracle)")
def test_marker_after_scan_reference_defect():
    """The reference drops the data in front of an unknown marker within one
    of its 2,048-byte reads (read_more_data's default case returns without
    appending, src/decoder.cpp:147-148), so it rejects the sample with a COM
    segment after its scan: "data incomplete" (INTEGRATION.md s4)."""
    ok, _ = _ref_decode(_with_com_after_scan(_golden("JPEG_example_JPG_RIP_050")))
    assert not ok
    ok, _ = _ref_decode(_golden("JPEG_example_JPG_RIP_050"))
    assert ok
