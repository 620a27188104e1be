"""CPU tests of the 4:1:1 (Y H4V1) and 4:4:0 (Y H1V2) extensions, and of the
oracle's MCU assembly for every sampling.

The reference has no path for these layouts (src/decoder.cpp:58-69 rejects
them), so parity is pinned by construction:
* the oracle's put_mcu (oracle/oracle.c) against an independent numpy model
  that assembles component planes from the oracle's own IDCT blocks and
  replicates chroma by nearest neighbour (the reference's 4:2:0 rule,
  src/decoder.cpp:474-483, along the subsampled axes only);
* the host Huffman decoder and the GPU entropy algorithm (host emulation) on
  files written by tests/jpeg_writer.py from known coefficients: exact.
Pillow (libjpeg) decodes the same files as an independent decoder; with
flat chroma (no upsampling filter in play) it agrees to IDCT rounding."""
import io

import numpy as np
import pytest

import jpeg_writer as JW
import oracle_py as O

FACTORS = {0: [(1, 1)] * 3, 1: [(2, 2), (1, 1), (1, 1)], 3: [(2, 1), (1, 1), (1, 1)],
           5: [(4, 1), (1, 1), (1, 1)], 6: [(1, 2), (1, 1), (1, 1)], 4: [(1, 1)]}


def _huff_src():
    from PIL import Image
    b = io.BytesIO()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(b, format="JPEG", quality=90)
    return b.getvalue()


def _planes_model(coefs, qt, w, h, s):
    """Independent restatement of MCU assembly: planes from IDCT'd blocks."""
    pw, ph, bpm, nluma = O.GEOM[s]
    mw, mh = -(-w // pw), -(-h // ph)
    samples = O.idct_blocks(O.dequant_natural(coefs, qt, s)).reshape(mh, mw, bpm, 8, 8)
    hy, vy = (pw // 8, ph // 8)
    # luma plane: blocks of an MCU row-major (hy x vy)
    Y = samples[:, :, :nluma].reshape(mh, mw, vy, hy, 8, 8).transpose(0, 2, 4, 1, 3, 5).reshape(mh * ph, mw * pw)
    if bpm == 1:
        U = V = np.zeros_like(Y)
    else:
        def plane(k):
            return samples[:, :, k].transpose(0, 2, 1, 3).reshape(mh * 8, mw * 8)
        U, V = plane(nluma), plane(nluma + 1)
        U = np.repeat(np.repeat(U, vy, 0), hy, 1)
        V = np.repeat(np.repeat(V, vy, 0), hy, 1)
    return O.yuv_to_bgrx(Y[:h, :w], U[:h, :w], V[:h, :w])


@pytest.mark.parametrize("s", [0, 1, 3, 4, 5, 6])
@pytest.mark.parametrize("w,h", [(96, 64), (101, 37), (1, 1), (67, 129)])
def test_oracle_mcu_assembly_matches_plane_model(s, w, h):
    coefs, qt = O.synthetic_coefs(w, h, s, seed=w * h + s)
    np.testing.assert_array_equal(O.decode_q16(coefs, qt, w, h, s), _planes_model(coefs, qt, w, h, s))


@pytest.mark.parametrize("s", [5, 6])
@pytest.mark.parametrize("w,h,dri", [(96, 64, 0), (101, 37, 3), (1, 1, 0), (333, 177, 0), (64, 16, 1)])
def test_host_and_gpu_algorithm_decode_exact(hjd, s, w, h, dri):
    coefs, qt = O.synthetic_coefs(w, h, s, seed=w + 7 * s)
    data = JW.encode_frame(coefs, w, h, FACTORS[s], qt, _huff_src(), restart_interval=dri)
    c1, info = hjd.decode_coefs(data)
    assert info.sampling == s and info.nblocks == coefs.shape[0]
    np.testing.assert_array_equal(c1, coefs)
    np.testing.assert_array_equal(np.array(info.qt), qt)
    em, status = hjd.emulate_entropy(data, sub_bits=64)
    assert status & ~1 == 0          # bit 0: the repair path ran (allowed)
    np.testing.assert_array_equal(em, coefs)
    # multi-scan form of the same file (non-interleaved luma, interleaved chroma)
    ms, expect = JW.rewrite_scans(data, coefs, [(0,), (1, 2)], 2)
    np.testing.assert_array_equal(hjd.decode_coefs(ms)[0], expect)


@pytest.mark.parametrize("s", [5, 6])
def test_pillow_agrees_with_flat_chroma(hjd, s):
    from PIL import Image
    w, h = 96, 64
    coefs, qt = O.synthetic_coefs(w, h, s, seed=3)
    comp = O.block_components(s, coefs.shape[0])
    coefs[comp > 0] = 0
    coefs[comp == 1, 0] = 3
    coefs[comp == 2, 0] = -2
    data = JW.encode_frame(coefs, w, h, FACTORS[s], qt, _huff_src())
    px = O.decode_q16(coefs, qt, w, h, s)
    ref = np.asarray(Image.open(io.BytesIO(data)).convert("RGB"))[..., ::-1].astype(np.int32)
    d = np.abs(px.view(np.uint8).reshape(h, w, 4)[..., :3].astype(np.int32) - ref)
    # the same bound 4:2:2 shows on this content (IDCT rounding of clipped noise)
    assert d.mean() < 1.0 and d.max() <= 12, (d.mean(), d.max())


def test_geometry_tables_agree(hjd):
    for s in (0, 1, 3, 4, 5, 6):
        for w, h in ((1, 1), (33, 17), (3840, 2160)):
            assert hjd.frame_blocks(w, h, s) == O.frame_blocks(w, h, s)
            mw, mh, bpm, (pw, ph) = hjd.mcu_geometry(w, h, s)
            assert (pw, ph, bpm) == O.GEOM[s][:3]
