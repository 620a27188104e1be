"""GPU parity: the HIP path (through the C ABI) vs the reference fixtures and the
oracle.  Bit-exact everywhere (integer/byte work).  Run on the MI355X box:

    python -m pytest tests -m gpu -x -q
"""
import hashlib

import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu


def sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def to_u32(t):
    return t.cpu().numpy().view(np.uint32)


def _decode(hjd, ctx, coefs, qt, w, h, s, fmt=0, pitch_px=None, guard=0, fill=-1):
    """Run one frame through a Plan; returns (pixels HxW uint32, full buffer)."""
    import torch
    pitch_px = pitch_px or w
    nbytes = guard * 2 + pitch_px * 4 * h
    buf = torch.full((nbytes // 4,), fill, dtype=torch.int32, device="cuda")
    spec = hjd.FrameSpec(w, h, s, coef_offset=0, out_offset=guard, out_pitch=pitch_px * 4, qt_index=(0, 1, 2))
    plan = hjd.Plan(ctx, [spec], fmt, qtables=qt if fmt == 0 else None)
    dev = torch.from_numpy(np.ascontiguousarray(coefs)).cuda()
    before = dev.clone()
    plan.launch(dev, buf)
    torch.cuda.synchronize()
    assert torch.equal(dev, before), "kernel modified its input"
    full = to_u32(buf)
    px = full[guard // 4: guard // 4 + pitch_px * h].reshape(h, pitch_px)[:, :w]
    return px, full


@pytest.mark.parametrize("name", O.golden_cases())
def test_golden_q16(hjd, ctx, name):
    c = O.load_case(name)
    rec = O.manifest()["cases"][name]
    w, h, s = int(c["width"]), int(c["height"]), int(c["sampling"])
    px, _ = _decode(hjd, ctx, c["coefs_q16"], c["qt"], w, h, s)
    np.testing.assert_array_equal(px, c["bgrx"])
    assert sha(px) == rec["bgrx_sha256"]


@pytest.mark.parametrize("name", O.golden_cases())
def test_golden_i32_natural(hjd, ctx, name):
    """idct.h-compat input (jpg.mcu_data layout) gives the same pixels."""
    c = O.load_case(name)
    w, h, s = int(c["width"]), int(c["height"]), int(c["sampling"])
    nat = O.dequant_natural(c["coefs_q16"], c["qt"], s)
    assert sha(nat) == O.manifest()["cases"][name]["mcu_data_sha256"]
    px, _ = _decode(hjd, ctx, nat, None, w, h, s, fmt=1)
    np.testing.assert_array_equal(px, c["bgrx"])


def test_sample_jpeg_idct_stage_hash(hjd, ctx):
    """IDCT-only kernel reproduces the reference's post-IDCT blocks."""
    import torch
    c = O.load_case("JPEG_example_JPG_RIP_050")
    nat = O.dequant_natural(c["coefs_q16"], c["qt"], 1)
    d_in = torch.from_numpy(nat).cuda()
    d_out = torch.empty_like(d_in)
    ctx.idct_blocks(d_in, d_out, nat.shape[0])
    torch.cuda.synchronize()
    assert sha(d_out.cpu().numpy()) == "cfa0326de498c6fb4d0fafebe3033e4f35aba61179a9ba6cd5ec78386ccf50d1"


def test_idct_vectors(hjd, ctx):
    import torch
    z = np.load(O.GOLDEN + "/idct_vectors.npz")
    d_in = torch.from_numpy(z["inp"]).cuda()
    d_out = torch.empty_like(d_in)
    ctx.idct_blocks(d_in, d_out, z["inp"].shape[0])
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d_out.cpu().numpy(), z["out"])


@pytest.mark.parametrize("mode", [0, 1])
def test_csc_exhaustive(hjd, ctx, mode):
    """Device colour stage over all 2^27 (Y,U,V) == the reference's fp64
    conversion (hash recorded from the compiled reference).  mode 0 is the
    kernel's integer form, mode 1 the literal fp64 form."""
    import torch
    out = torch.empty(1 << 27, dtype=torch.int32, device="cuda")
    ctx.debug_csc_exhaustive(out, mode)
    torch.cuda.synchronize()
    assert sha(out.cpu().numpy()) == O.manifest()["csc_exhaustive_sha256"]


@pytest.mark.parametrize("w,h,s", [(1, 1, 1), (1, 1, 0), (8, 8, 0), (16, 16, 1), (17, 17, 1), (9, 15, 0),
                                   (127, 33, 1), (129, 40, 1), (255, 9, 0), (130, 17, 0), (640, 48, 1),
                                   (2048, 32, 0)])
def test_random_frames_vs_oracle(hjd, ctx, w, h, s):
    coefs, qt = O.synthetic_coefs(w, h, s, seed=w * 31 + h)
    px, _ = _decode(hjd, ctx, coefs, qt, w, h, s)
    np.testing.assert_array_equal(px, O.decode_q16(coefs, qt, w, h, s))


@pytest.mark.parametrize("s", [0, 1])
def test_no_writes_outside_frame(hjd, ctx, s):
    """Cropping: with a padded pitch and guard bands, only W x H words change."""
    w, h = 45, 37
    coefs, qt = O.synthetic_coefs(w, h, s, seed=3)
    guard, pitch = 4096, 64
    px, full = _decode(hjd, ctx, coefs, qt, w, h, s, pitch_px=pitch, guard=guard, fill=0x5A5A5A5A)
    np.testing.assert_array_equal(px, O.decode_q16(coefs, qt, w, h, s))
    mask = np.ones(full.shape, bool)
    body = mask[guard // 4: guard // 4 + pitch * h].reshape(h, pitch)
    body[:, :w] = False
    assert (full[mask] == 0x5A5A5A5A).all()


def test_batch_mixed_geometry(hjd, ctx):
    """One plan, many frames of different sizes and qtables, packed buffers."""
    import torch
    rng = np.random.default_rng(11)
    sizes = [(313, 234), (16, 16), (1920, 40), (33, 95), (64, 8), (200, 120), (1, 300)]
    for s in (0, 1):
        specs, all_coefs, qts, expect, off_blk, off_px = [], [], [], [], 0, 0
        for i, (w, h) in enumerate(sizes):
            coefs, qt = O.synthetic_coefs(w, h, s, seed=i, quality_scale=float(rng.uniform(0.3, 2.0)))
            qts.append(qt)
            specs.append(hjd.FrameSpec(w, h, s, coef_offset=off_blk, out_offset=off_px * 4,
                                       qt_index=(3 * i, 3 * i + 1, 3 * i + 2)))
            all_coefs.append(coefs)
            expect.append(O.decode_q16(coefs, qt, w, h, s))
            off_blk += coefs.shape[0]
            off_px += w * h
        plan = hjd.Plan(ctx, specs, 0, qtables=np.concatenate(qts))
        dev = torch.from_numpy(np.concatenate(all_coefs)).cuda()
        out = torch.zeros(off_px, dtype=torch.int32, device="cuda")
        plan.launch(dev, out)
        torch.cuda.synchronize()
        got = to_u32(out)
        pos = 0
        for (w, h), e in zip(sizes, expect):
            np.testing.assert_array_equal(got[pos:pos + w * h].reshape(h, w), e)
            pos += w * h


@pytest.mark.parametrize("s,grid", [(1, 1), (1, 3), (0, 7), (1, 0)])
def test_grid_sizes_and_repeat_launch(hjd, ctx, s, grid):
    """Persistent loop correctness for any grid size; relaunch is idempotent."""
    import torch
    w, h = 700, 70
    coefs, qt = O.synthetic_coefs(w, h, s, seed=grid)
    plan = hjd.Plan(ctx, [hjd.FrameSpec(w, h, s, qt_index=(0, 1, 2))], 0, qtables=qt)
    dev = torch.from_numpy(coefs).cuda()
    out = torch.zeros((h, w), dtype=torch.int32, device="cuda")
    exp = O.decode_q16(coefs, qt, w, h, s)
    for _ in range(2):
        plan.launch(dev, out, grid_blocks=grid)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(to_u32(out), exp)


def test_4k_frame_vs_oracle(hjd, ctx):
    """One full 3840x2160 4:2:0 frame (the bench unit) vs the oracle."""
    w, h, s = 3840, 2160, 1
    coefs, qt = O.synthetic_coefs(w, h, s, seed=2024)
    px, _ = _decode(hjd, ctx, coefs, qt, w, h, s)
    np.testing.assert_array_equal(px, O.decode_q16(coefs, qt, w, h, s))


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("s", [0, 1])
def test_extreme_legal_blocks(hjd, ctx, mode, s):
    """Clamp-edge blocks (DC +-2100, q=1 extremes, checkerboards) through the
    fused path, both kernels (1 persistent, 2 latency): every block of every
    MCU is one of the IDCT known-answer vectors."""
    import torch
    z = np.load(O.GOLDEN + "/idct_vectors.npz")
    bpm, mw = (6, 16) if s == 1 else (3, 8)
    n = (z["inp"].shape[0] // bpm) * bpm
    nat = np.ascontiguousarray(z["inp"][:n])
    w, h = mw * (n // bpm), mw
    plan = hjd.Plan(ctx, [hjd.FrameSpec(w, h, s, qt_index=(0, 1, 2))], 1)
    plan.set_kernel(mode)
    out = torch.full((h, w), -1, dtype=torch.int32, device="cuda")
    plan.launch(torch.from_numpy(nat).cuda(), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(to_u32(out), O.decode_i32(nat, w, h, s))


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("s", [0, 1])
def test_extreme_legal_blocks_q16(hjd, ctx, mode, s):
    """The same clamp-edge blocks in the hot int16 zigzag format (all-ones
    qtables), so the largest legal dequantised values go through the packed
    row pass (v_pk_mul_lo_u16 dequant + v_dot2_i32_i16 rotations)."""
    import torch
    z = np.load(O.GOLDEN + "/idct_vectors.npz")
    bpm, mw = (6, 16) if s == 1 else (3, 8)
    n = (z["inp"].shape[0] // bpm) * bpm
    nat = np.ascontiguousarray(z["inp"][:n])
    assert np.abs(nat).max() < 32768
    coefs = np.ascontiguousarray(nat[:, O.ZIGZAG].astype(np.int16))   # natural -> zigzag, q = 1
    qt = np.ones((3, 64), np.int32)
    w, h = mw * (n // bpm), mw
    plan = hjd.Plan(ctx, [hjd.FrameSpec(w, h, s, qt_index=(0, 1, 2))], 0, qtables=qt)
    plan.set_kernel(mode)
    out = torch.full((h, w), -1, dtype=torch.int32, device="cuda")
    plan.launch(torch.from_numpy(coefs).cuda(), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(to_u32(out), O.decode_i32(nat, w, h, s))
