"""AC run lengths at the end of a block (T.81 F.2.2.2): a run of zeros, a
ZRL (0xF0, sixteen zeros) or a coefficient that would pass index 63.

The reference skips the run and asserts `count + 1 <= 64` before storing
(src/decoder.cpp:241-256): a ZRL may bring the index to exactly 64 (the block
then ends without an EOB), one index further is a rejection, and so is a
coefficient at index 64.  The host decoder's two readers, the GPU entropy
algorithm (host emulation here, the device under -m gpu) and -- when built
-- the reference itself are run on hand-written 8x8 4:4:4 files."""
import io

import numpy as np
import pytest

import jpeg_writer as JW
import oracle_py as O


def _std_tables():
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, format="JPEG", quality=90)
    return b.getvalue()


def _file(y_symbols):
    """One 8x8 4:4:4 frame, quantisers all 1.  y_symbols: the luma block's AC
    part as (run/size symbol, value) pairs; DC 0 and chroma EOB-only."""
    src = JW._segments(_std_tables())
    dht = JW._dht_codes(src)
    out = bytearray(b"\xff\xd8")

    def seg(m, p):
        out.extend(bytes([0xFF, m, (len(p) + 2) >> 8, (len(p) + 2) & 255]) + p)

    seg(0xDB, bytes([0]) + bytes([1] * 64))
    seg(0xDB, bytes([1]) + bytes([1] * 64))
    seg(0xC0, bytes([8, 0, 8, 0, 8, 3, 1, 0x11, 0, 2, 0x11, 1, 3, 0x11, 1]))
    for m, p in src:
        if m == 0xC4:
            seg(m, p)
    seg(0xDA, bytes([3, 1, 0x00, 2, 0x11, 3, 0x11, 0, 63, 0]))
    bw = JW._Bits()
    for comp, syms in ((0, y_symbols), (1, [(0x00, 0)]), (1, [(0x00, 0)])):
        c, ln = dht[(0, comp)][0]
        bw.put(c, ln)
        for sym, v in syms:
            c, ln = dht[(1, comp)][sym]
            bw.put(c, ln)
            s, bits = JW._category(v)
            assert s == sym & 15
            bw.put(bits, s)
    bw.flush()
    out += bw.out + b"\xff\xd9"
    return bytes(out)


ZRL = (0xF0, 0)
CASES = {
    # name: (symbols, zigzag index of the coefficient 5, accepted)
    "zrl_to_64": ([ZRL, ZRL, (0xE3, 5), ZRL], 47, True),          # 1..32 zeros, 33..46, 47 = 5, 48..63 zeros
    "zrl_past_63": ([ZRL, ZRL, (0xF3, 5), ZRL], 48, False),       # the ZRL starts at 49: past 63
    "coef_at_63": ([ZRL, ZRL, ZRL, (0xE3, 5)], 63, True),         # no EOB needed after index 63
    "coef_past_63": ([ZRL, ZRL, ZRL, (0xF3, 5)], 64, False),      # 49 + 15 = 64
    "eob_after_63": ([ZRL, ZRL, ZRL, (0xE3, 5), (0x00, 0)], 63, None),
}


def _host(lib, data):
    from test_jpeg_host import decode
    out = []
    for mode in (0, 1):
        lib.hjd_debug_host_reader(mode)
        try:
            rc, _, coefs = decode(lib, data)
            out.append((rc, lib.hjd_last_error() if rc else b"", coefs))
        finally:
            lib.hjd_debug_host_reader(0)
    return out


@pytest.fixture(scope="module")
def lib():
    from ocljpegdecoder_amd import _lib
    return _lib.load()


@pytest.mark.parametrize("name", list(CASES))
def test_host_and_emulation(lib, hjd, name):
    syms, at, ok = CASES[name]
    data = _file(syms)
    exp = np.zeros((3, 64), np.int16)
    if at < 64:
        exp[0, at] = 5
    for rc, err, coefs in _host(lib, data):
        if ok:
            assert rc == 0, err
            np.testing.assert_array_equal(coefs, exp)
        elif ok is False:
            assert rc != 0 and b"corrupt" in err, err
    if ok:
        coefs, status = hjd.emulate_entropy(data, 256)
        assert not (status & ~1), status
        np.testing.assert_array_equal(coefs, exp)
    elif ok is False:
        with pytest.raises(Exception, match="corrupt"):
            hjd.emulate_entropy(data, 256)


def test_eob_after_index_63_is_a_next_block_symbol(lib):
    """After a coefficient at index 63 the block is complete; the EOB that
    follows is read as the next block's DC code (here: the Cb DC code for 0
    is '00' and the luma EOB is '1010'), so the rest of the scan shifts:
    rejected or decoded differently, never silently equal."""
    data = _file(CASES["eob_after_63"][0])
    exp = np.zeros((3, 64), np.int16)
    exp[0, 63] = 5
    for rc, _, coefs in _host(lib, data):
        assert rc != 0 or not np.array_equal(coefs, exp)


@pytest.mark.skipif(not O.ref_available(), reason="needs oracle/_ref/libref.so (make -C oracle)")
@pytest.mark.parametrize("name", [n for n in CASES if CASES[n][2] is not None])
def test_reference_agrees(lib, hjd, name):
    from test_truncation import _ref_decode
    syms, _, ok = CASES[name]
    data = _file(syms)
    ref_ok, cap = _ref_decode(data)
    assert ref_ok == ok
    if ok:
        (rc, _, coefs), _ = _host(lib, data)
        info = hjd.parse(data)
        np.testing.assert_array_equal(O.dequant_natural(coefs, np.array(info.qt), info.sampling), cap)


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(CASES))
def test_gpu_entropy(hjd, ctx, name):
    import torch
    syms, at, ok = CASES[name]
    data = _file(syms)
    coefs = torch.zeros((3, 64), dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, 1, len(data), 3, 256) as gd:
        gd.decode_coefs([data], coefs)
        status = gd.sync(raise_on_error=False)
    if ok:
        assert status[0] == 0
        exp = np.zeros((3, 64), np.int16)
        exp[0, at] = 5
        np.testing.assert_array_equal(coefs.cpu().numpy(), exp)
    elif ok is False:
        assert status[0] != 0
