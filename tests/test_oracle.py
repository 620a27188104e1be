"""CPU tests: pin the oracle (oracle/oracle.c) to the reference.

Anchors, in order of strength:
  * oracle/_ref/libref.so -- the reference CPU path compiled from its own
    sources (only where /root/reference exists; skipped otherwise);
  * tests/golden/ -- fixtures produced by that compiled reference
    (tests/golden/make_golden.py), including the SURVEY.md s8(c) hashes of the
    reference's only sample, test/JPEG_example_JPG_RIP_050.jpg;
  * SURVEY.md s8(c) clamp-edge known answers.
"""
import hashlib

import numpy as np
import pytest

import oracle_py as O

SURVEY_SAMPLE = {
    "mcu_data_sha256": "c25806f5238c8ec7c2a4846cf6b67c5b567fd268599591392baf77e91023924e",
    "idct_sha256": "cfa0326de498c6fb4d0fafebe3033e4f35aba61179a9ba6cd5ec78386ccf50d1",
    "bgrx_sha256": "efb49cf99f2f6c583c546d6ef24c5d26ae339955c8bbe467341933aafa9b16e5",
}


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def test_manifest_carries_survey_hashes():
    case = O.manifest()["cases"]["JPEG_example_JPG_RIP_050"]
    for k, v in SURVEY_SAMPLE.items():
        assert case[k] == v, k
    assert (case["width"], case["height"], case["sampling"], case["blocks"]) == (313, 234, 1, 1800)


@pytest.mark.parametrize("name", O.golden_cases())
def test_oracle_matches_reference_fixture(name):
    c = O.load_case(name)
    rec = O.manifest()["cases"][name]
    w, h, s = int(c["width"]), int(c["height"]), int(c["sampling"])
    # dequant + zigzag reproduces the reference's jpg.mcu_data exactly
    nat = O.dequant_natural(c["coefs_q16"], c["qt"], s)
    assert sha(nat) == rec["mcu_data_sha256"]
    # IDCT of every block reproduces the reference's Fast_IDCT output
    assert sha(O.idct_blocks(nat)) == rec["idct_sha256"]
    # full pixel path, both input formats
    bgrx = O.decode_q16(c["coefs_q16"], c["qt"], w, h, s)
    assert sha(bgrx) == rec["bgrx_sha256"]
    np.testing.assert_array_equal(bgrx, c["bgrx"])
    np.testing.assert_array_equal(O.decode_i32(nat, w, h, s), c["bgrx"])


def test_oracle_idct_vectors():
    z = np.load(O.GOLDEN + "/idct_vectors.npz")
    np.testing.assert_array_equal(O.idct_blocks(z["inp"]), z["out"])


def test_clamp_edge_known_answers():
    """DC 2100 -> 255, -2100 -> -256, 2016 -> 252; the
    {b0=1000,b1=-900,b8=700} block's corners clamp to [90,255,-152,160]."""
    def one(dc):
        b = np.zeros(64, np.int32); b[0] = dc
        return O.idct_blocks(b)[0]
    assert (one(2100) == 255).all()
    assert (one(-2100) == -256).all()
    assert (one(2016) == 252).all()
    b = np.zeros(64, np.int32); b[0], b[1], b[8] = 1000, -900, 700
    out = O.idct_blocks(b)[0]
    assert [out[0], out[7], out[56], out[63]] == [90, 255, -152, 160]


def test_csc_sample_and_pixel_zero():
    z = np.load(O.GOLDEN + "/csc_sample.npz")
    np.testing.assert_array_equal(O.yuv_to_bgrx(z["y"], z["u"], z["v"]), z["out"])
    # pixel[0,0] of the sample image is B48 G75 R67
    c = O.load_case("JPEG_example_JPG_RIP_050")
    p = int(c["bgrx"][0, 0])
    assert (p & 255, (p >> 8) & 255, (p >> 16) & 255, p >> 24) == (48, 75, 67, 0)
    p = int(c["bgrx"][233, 312])
    assert (p & 255, (p >> 8) & 255, (p >> 16) & 255, p >> 24) == (36, 55, 64, 0)


def _grid_uv():
    u, v = np.meshgrid(np.arange(-256, 256, dtype=np.int32), np.arange(-256, 256, dtype=np.int32), indexing="ij")
    return u.ravel().copy(), v.ravel().copy()


def test_oracle_csc_exhaustive_hash():
    """Oracle colour conversion over all of [-256,255]^3 == the reference's."""
    u, v = _grid_uv()
    h = hashlib.sha256()
    for y in range(-256, 256):
        h.update(O.yuv_to_bgrx(np.full(u.shape, y, np.int32), u, v).tobytes())
    assert h.hexdigest() == O.manifest()["csc_exhaustive_sha256"]


# Constants of the device formulation (csrc/hjd_device.hpp colour block).
LEVEL = 128                      # luma leaves the IDCT as Ys = Y + 128
RK = 91881                       # floor(1.402 v) = (v * RK) >> 16
BK = 116130                      # floor(1.772 u) = (u * BK) >> 16, except u = -250 (one below; B saturates to 0 there)
GSCALE = 128
GKU, GKV = -17207 * GSCALE, -35707 * GSCALE
GMAGIC = 43980466                # ceil(2^48 / (50000 * GSCALE))
GCORNER_Q = -75


def integer_csc(y, u, v):
    """numpy model of the kernel's exact-integer colour formulation, op for op
    (csrc/hjd_device.hpp chroma_terms / pair_of / g_fix / pixels2): every
    chroma term is the high int16 of a 32-bit word."""
    y = y.astype(np.int64); u = u.astype(np.int64); v = v.astype(np.int64)
    ys = y + LEVEL
    r = (v * RK) >> 16
    b = (u * BK) >> 16
    hi = ((u * GKU + v * GKV) * GMAGIC) >> 32       # v_mul_hi_i32
    g = hi >> 16
    flagged = (hi & 0xFFFF) == 0xFFFF
    corner = (g == GCORNER_Q) & (ys >= 188 + LEVEL) & (ys <= 201 + LEVEL)
    g = g + (flagged & ~corner)
    r = np.clip(ys + r, 0, 255)
    g = np.clip(ys + g, 0, 255)
    b = np.clip(ys + b, 0, 255)
    return ((r << 16) | (g << 8) | b).astype(np.uint32)


def test_fixed_point_colour_terms():
    """The constants of the device formulation, exhaustively on their domains."""
    x = np.arange(-256, 256, dtype=np.int64)
    assert ((x * RK) >> 16 == np.floor_divide(701 * x, 500)).all()
    b = (x * BK) >> 16
    exact = np.floor_divide(443 * x, 250)
    assert (b[x != -250] == exact[x != -250]).all() and b[x == -250] == exact[x == -250] - 1
    # ... where Ys + B <= (255 + LEVEL) - 443 < 0: the blue channel saturates to 0 either way
    assert (255 + LEVEL) + exact[x == -250] < 0
    assert max(RK, BK, -GKU, -GKV) < 2 ** 23        # 24-bit signed multiplies
    assert GMAGIC < 2 ** 31 and GMAGIC == -(-(1 << 48) // (50000 * GSCALE))
    u, v = np.meshgrid(x, x, indexing="ij")
    mc = u * GKU + v * GKV
    assert np.abs(mc).max() < 2 ** 31                # fits the int32 mulhi operand
    hi = (mc * GMAGIC) >> 32
    q = hi >> 16
    exact = np.floor_divide(-(17207 * u + 35707 * v), 50000)
    flagged = (hi & 0xFFFF) == 0xFFFF
    # the mulhi is the floor everywhere except at the flagged points, where it
    # is one below; the flag marks exactly (U,V) = (-200,200) and (-100,100)
    assert (q[~flagged] == exact[~flagged]).all()
    assert (q[flagged] == exact[flagged] - 1).all()
    assert sorted(map(tuple, (np.argwhere(flagged) - 256).tolist())) == [(-200, 200), (-100, 100)]
    assert (hi & 0xFFFF)[~flagged].max() <= 0xFFFE


def test_integer_csc_formulation_is_exact():
    """The integer restatement equals the reference fp64 conversion on the whole
    domain (the device test then checks the device code against the same hash)."""
    u, v = _grid_uv()
    h = hashlib.sha256()
    for y in range(-256, 256):
        h.update(integer_csc(np.full(u.shape, y, np.int32), u, v).tobytes())
    assert h.hexdigest() == O.manifest()["csc_exhaustive_sha256"]


def test_special_chroma_pairs_enumerated():
    """G's chroma term is an exact integer only for these (U,V); only
    (-200,200) differs from the integer floor, for Y in [188,201]."""
    pairs = [(U, V) for U in range(-256, 256) for V in range(-256, 256)
             if (U, V) != (0, 0) and (17207 * U + 35707 * V) % 50000 == 0]
    assert pairs == [(-200, 200), (-100, 100), (100, -100), (200, -200)]
    for U, V in pairs:
        y = np.arange(-256, 256, dtype=np.int32)
        ref = O.yuv_to_bgrx(y, np.full_like(y, U), np.full_like(y, V))
        m = (17207 * U + 35707 * V) // 50000
        g_int = np.clip(y + 128 - m, 0, 255)
        bad = y[((ref >> 8) & 255) != g_int]
        if (U, V) == (-200, 200):
            assert bad.tolist() == list(range(188, 202))
        else:
            assert bad.size == 0


@pytest.mark.skipif(not O.ref_available(), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_vs_live_reference_random_blocks():
    """Random legal blocks: oracle IDCT == reference Fast_IDCT, live."""
    import ctypes
    rng = np.random.default_rng(99)
    coefs, qt = O.synthetic_coefs(64, 64, 1, seed=5, quality_scale=0.5)
    nat = O.dequant_natural(coefs, qt, 1)
    # random pixels -> float FDCT -> random quantisers: legal by construction
    # (arbitrary random coefficients can push the reference's iclp[] index out
    # of range, which is undefined behaviour in the reference)
    k = np.arange(8)
    m = np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16) * np.where(k == 0, 1 / np.sqrt(2), 1.0)[:, None] / 2
    pix = rng.integers(-128, 128, (2000, 8, 8)).astype(np.float64)
    F = np.einsum("ux,nxy,vy->nuv", m, pix, m).reshape(-1, 64)
    q = rng.integers(1, 40, (2000, 64))
    extra = (np.rint(F / q) * q).astype(np.int32)
    blocks = np.concatenate([nat, extra])
    ref_out = blocks.copy()
    O.ref().ref_fast_idct_n(ref_out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), ref_out.shape[0])
    np.testing.assert_array_equal(O.idct_blocks(blocks), ref_out)
