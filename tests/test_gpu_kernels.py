"""GPU: the two fused kernels -- the persistent streaming kernel and the
latency kernel (one workgroup per task) -- give the oracle's pixels on every
sampling, input format, output format and edge geometry.  HJD_KERNEL_AUTO
sends small launches (single frames) to the latency kernel and batches to the
persistent one, so both are forced here explicitly."""
import numpy as np
import pytest

import oracle_py as O

pytestmark = pytest.mark.gpu

SIZES = [(1, 1), (17, 9), (129, 33), (385, 40), (1920, 1080)]


def _run(hjd, ctx, coefs, qt, w, h, s, mode, fmt=0, out_format=0, pad=0):
    import torch
    pitch = hjd.default_pitch(w, out_format) + pad
    guard = 256
    buf = torch.full((2 * guard + pitch * h,), 0x5A, dtype=torch.uint8, device="cuda")
    spec = hjd.FrameSpec(w, h, s, out_offset=guard, out_pitch=pitch, qt_index=(0, 1, 2), out_format=out_format)
    plan = hjd.Plan(ctx, [spec], fmt, qtables=qt if fmt == 0 else None)
    plan.set_kernel(mode)
    plan.launch(torch.from_numpy(np.ascontiguousarray(coefs)).cuda(), buf)
    torch.cuda.synchronize()
    full = buf.cpu().numpy()
    mask = np.ones(full.shape, bool)
    nbytes = hjd.OUT_BYTES[out_format] * w
    mask[guard:guard + pitch * h].reshape(h, pitch)[:, :nbytes] = False
    assert (full[mask] == 0x5A).all(), "write outside the frame"
    return full[guard:guard + pitch * h].reshape(h, pitch)[:, :nbytes]


def _expect(bgrx, out_format):
    b = np.ascontiguousarray(bgrx).view(np.uint8).reshape(bgrx.shape[0], bgrx.shape[1], 4)
    return b.reshape(bgrx.shape[0], -1) if out_format == 0 else b[..., :3].reshape(bgrx.shape[0], -1)


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("s", [0, 1, 3, 4, 5, 6])
def test_both_kernels_vs_oracle(hjd, ctx, mode, s):
    for (w, h) in SIZES:
        coefs, qt = O.synthetic_coefs(w, h, s, seed=w + h + s)
        exp = O.decode_q16(coefs, qt, w, h, s)
        for out_format in (0, 1):
            got = _run(hjd, ctx, coefs, qt, w, h, s, mode, out_format=out_format, pad=4 * (w % 3))
            np.testing.assert_array_equal(got, _expect(exp, out_format), err_msg=f"{w}x{h} s={s} fmt={out_format}")
        nat = O.dequant_natural(coefs, qt, s)
        got = _run(hjd, ctx, nat, None, w, h, s, mode, fmt=1)
        np.testing.assert_array_equal(got, _expect(exp, 0), err_msg=f"{w}x{h} s={s} i32")


@pytest.mark.parametrize("s", [0, 1, 3, 5, 6])
def test_latency_kernel_colour_corners(hjd, ctx, s):
    """The flagged-G path inside the latency kernel's split colour stage."""
    from test_gpu_extensions import _corner_frame
    w, h = 260, 50
    nat = _corner_frame(w, h, s, seed=s + 29)
    got = _run(hjd, ctx, nat, None, w, h, s, 2, fmt=1)
    np.testing.assert_array_equal(got, _expect(O.decode_i32(nat, w, h, s), 0))


def test_latency_kernel_multi_frame_plan(hjd, ctx):
    """Several frames of different sizes and qtables in one latency launch."""
    import torch
    sizes = [(313, 234), (16, 16), (1920, 40), (33, 95), (1, 300)]
    specs, coefs, qts, exps, off_blk, off_px = [], [], [], [], 0, 0
    for i, (w, h) in enumerate(sizes):
        c, q = O.synthetic_coefs(w, h, 1, seed=50 + i, quality_scale=0.5 + 0.3 * i)
        specs.append(hjd.FrameSpec(w, h, 1, coef_offset=off_blk, out_offset=off_px * 4,
                                   qt_index=(3 * i, 3 * i + 1, 3 * i + 2)))
        coefs.append(c); qts.append(q); exps.append(O.decode_q16(c, q, w, h, 1))
        off_blk += c.shape[0]; off_px += w * h
    plan = hjd.Plan(ctx, specs, 0, qtables=np.concatenate(qts))
    plan.set_kernel(hjd.KERNEL_LATENCY)
    out = torch.zeros(off_px, dtype=torch.int32, device="cuda")
    plan.launch(torch.from_numpy(np.concatenate(coefs)).cuda(), out)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    pos = 0
    for (w, h), e in zip(sizes, exps):
        np.testing.assert_array_equal(got[pos:pos + w * h].reshape(h, w), e)
        pos += w * h


def _q16_frame(w, h, s, seed):
    """16-bit-table frame: factors 256-1200, DC and one AC coefficient in
    {-1, 0, 1}; returns (coefs, qt, max |float IDCT output|)."""
    rng = np.random.default_rng(seed)
    nblk = O.frame_blocks(w, h, s)
    qt = rng.integers(256, 1201, (3, 64)).astype(np.int32)
    coefs = np.zeros((nblk, 64), np.int16)
    coefs[:, 0] = rng.integers(-1, 2, nblk)
    coefs[np.arange(nblk), rng.integers(1, 64, nblk)] = rng.integers(-1, 2, nblk)
    nat = O.dequant_natural(coefs, qt, s).astype(np.float64).reshape(-1, 8, 8)
    k = np.arange(8)
    c = np.where(k == 0, 1 / np.sqrt(2), 1.0)
    m = np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16) * c[:, None] / 2
    return coefs, qt, float(np.abs(np.einsum("ux,nuv,vy->nxy", m, nat, m)).max())


@pytest.mark.parametrize("mode", [1, 2])
@pytest.mark.parametrize("s", [0, 1, 3, 4, 5, 6])
def test_16bit_quantisation_tables(hjd, ctx, mode, s):
    """DQT precision 1 (16-bit entries, T.81 B.2.4.1): factors above 255
    through the 24-bit dequant multiply of both kernels, on blocks inside the
    reference's legal domain (column outputs within its iclp[-512, 511])."""
    w, h = 300, 70
    coefs, qt, peak = _q16_frame(w, h, s, seed=4000 + s)
    assert peak < 480, peak   # premise: legal domain, with margin for the integer IDCT's rounding
    got = _run(hjd, ctx, coefs, qt, w, h, s, mode)
    np.testing.assert_array_equal(got, _expect(O.decode_q16(coefs, qt, w, h, s), 0))


@pytest.mark.parametrize("d16", ["0", "probe"])
def test_444_gather_forms_vs_oracle(hjd, ctx, monkeypatch, d16):
    """4:4:4 persistent kernel with both coefficient-pair gathers: the
    ds_read_u16_d16_hi | ds_read_u16 form (hjd::kVarD16, taken where the
    hardware probe passed: MI355X as deployed) and the v_perm form (HJD_D16=0,
    and parts the probe did not pass)."""
    import torch
    if d16 == "0":
        monkeypatch.setenv("HJD_D16", "0")
    else:
        monkeypatch.delenv("HJD_D16", raising=False)
    arch = torch.cuda.get_device_properties(0).gcnArchName
    print("device", arch, "d16 gather selected", ctx.d16_gather()[1])
    assert ctx.d16_gather()[1] == (d16 != "0" and ctx.d16_gather()[0])
    for (w, h) in SIZES + [(3840, 64)]:
        coefs, qt = O.synthetic_coefs(w, h, 0, seed=7 * w + h)
        exp = O.decode_q16(coefs, qt, w, h, 0)
        for out_format in (0, 1):
            got = _run(hjd, ctx, coefs, qt, w, h, 0, 1, out_format=out_format)
            np.testing.assert_array_equal(got, _expect(exp, out_format), err_msg=f"{w}x{h} fmt={out_format}")


def test_d16_probe_selects_gather(hjd, ctx, monkeypatch):
    """Without an override the 4:4:4 gather form follows the one-wave hardware
    probe (hjd_probe.hip), not the device's ISA name; MI355X as deployed
    (sramecc+) zeroes the d16 load's low half, so the probe passes there."""
    import torch
    monkeypatch.delenv("HJD_D16", raising=False)
    zeroes, selected = ctx.d16_gather()
    arch = torch.cuda.get_device_properties(0).gcnArchName
    print("device", arch, "probe zeroes low half", zeroes, "d16 selected", selected)
    assert selected == zeroes
    if "sramecc+" in arch:
        assert zeroes, "sramecc+ part did not zero the d16 load's low half"


def test_d16_probe_failure_falls_back_to_perm_gather():
    """HJD_D16_PROBE=fail makes the probe report a half-preserving part: the
    runtime must then take the v_perm kernels, and 4:4:4 stays bit-exact.  A
    child process, because the probe result is cached per process."""
    import os
    import subprocess
    import sys
    code = r"""
import sys, numpy as np, torch
sys.path.insert(0, REPO); sys.path.insert(0, REPO + "/tests")
import ocljpegdecoder_amd as hjd, oracle_py as O
ctx = hjd.Context(0)
assert ctx.d16_gather() == (False, False), ctx.d16_gather()
w, h = 1920, 1080
coefs, qt = O.synthetic_coefs(w, h, 0, seed=5)
out, plan = hjd.decode_frame(ctx, torch.from_numpy(coefs).cuda(), qt, w, h, 0)
torch.cuda.synchronize()
assert np.array_equal(out.cpu().numpy().view(np.uint32), O.decode_q16(coefs, qt, w, h, 0))
print("fallback ok")
""".replace("REPO", repr(O.REPO))
    env = {k: v for k, v in os.environ.items() if k != "HJD_D16"}
    env["HJD_D16_PROBE"] = "fail"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "fallback ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


def test_d16_probe_hip_failure_is_not_sticky():
    """a probe whose HIP calls fail (HJD_D16_PROBE=hipfail: its
    allocation is one no device can satisfy -- a real hipErrorOutOfMemory)
    must clear that error, must not cache the failure, and the next 4:4:4
    launch must return HJD_OK with the oracle's pixels (v_perm kernels).  A
    child process: the probe result is per process."""
    import os
    import subprocess
    import sys
    code = r"""
import sys, numpy as np, torch
sys.path.insert(0, REPO); sys.path.insert(0, REPO + "/tests")
import ocljpegdecoder_amd as hjd, oracle_py as O
ctx = hjd.Context(0)                      # runs the probe: it fails inside HIP
assert ctx.d16_gather() == (False, False), ctx.d16_gather()
w, h = 1920, 1080
for s in (0, 1):
    coefs, qt = O.synthetic_coefs(w, h, s, seed=15 + s)
    plan = hjd.Plan(ctx, [hjd.FrameSpec(w, h, s, qt_index=(0, 1, 2))], hjd.IN_Q16_ZIGZAG, qtables=qt)
    plan.set_kernel(hjd.KERNEL_PERSISTENT)
    out = torch.zeros((h, w), dtype=torch.int32, device="cuda")
    plan.launch(torch.from_numpy(coefs).cuda(), out)   # raises if a stale HIP error surfaced
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy().view(np.uint32), O.decode_q16(coefs, qt, w, h, s)), s
print("hipfail ok")
""".replace("REPO", repr(O.REPO))
    env = {k: v for k, v in os.environ.items() if k != "HJD_D16"}
    env["HJD_D16_PROBE"] = "hipfail"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "hipfail ok" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("s", [0, 1])
def test_autotune_keeps_pixels(hjd, ctx, s):
    """hjd_plan_autotune times the launch shapes (tasks per wave x store
    policy) on the plan's own buffers and keeps the fastest: the chosen shape
    must be a candidate, the output left by the tuning launches and by a later
    default launch must both be the oracle's, and a plan small enough for the
    latency kernel is left unchanged."""
    import torch
    w, h, nf = 1920, 1080, 6
    coefs, qt = O.synthetic_coefs(w, h, s, seed=900 + s)
    exp = O.decode_q16(coefs, qt, w, h, s)
    nblk = coefs.shape[0]
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
             for i in range(nf)]
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
    assert plan.tasks > 1024
    d_coefs = torch.from_numpy(np.ascontiguousarray(np.tile(coefs, (nf, 1)))).cuda()
    out = torch.zeros((nf, h, w), dtype=torch.int32, device="cuda")
    hjd.autotune_cache_clear()
    tpw, var = plan.autotune(d_coefs, out)
    print("autotune chose", tpw, "tasks per wave, variant", var, plan.launch_shape())
    assert plan.launch_shape()["autotune_launches"] > 0 and not plan.launch_shape()["autotune_cached"]
    assert tpw in (1, 2, 4, 8, 16) and var in (0, 1)
    torch.cuda.synchronize()
    for i in range(nf):
        np.testing.assert_array_equal(out[i].cpu().numpy().view(np.uint32), exp, err_msg=f"tuning launch, frame {i}")
    out.zero_()
    plan.launch(d_coefs, out)
    torch.cuda.synchronize()
    for i in range(nf):
        np.testing.assert_array_equal(out[i].cpu().numpy().view(np.uint32), exp, err_msg=f"tuned launch, frame {i}")
    small = hjd.Plan(ctx, specs[:1], hjd.IN_Q16_ZIGZAG, qtables=qt)
    if small.tasks <= 1024:
        assert small.autotune(d_coefs, out) == (0, 0)
        assert small.launch_shape()["kernel"] == "latency"
    # a second plan of the same key takes the cached choice with no launch
    again = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
    assert again.autotune(d_coefs, out) == (tpw, var)
    shape = again.launch_shape()
    assert shape["autotune_launches"] == 0 and shape["autotune_cached"] == 1, shape
    assert shape["tasks_per_wave"] == plan.launch_shape()["tasks_per_wave"]
    assert shape["grid"] == plan.launch_shape()["grid"]
    # another batch geometry (half the frames) is another key: it tunes afresh
    half = hjd.Plan(ctx, specs[: nf // 2], hjd.IN_Q16_ZIGZAG, qtables=qt)
    if half.tasks > 1024:
        half.autotune(d_coefs, out)
        assert half.launch_shape()["autotune_cached"] == 0 and half.launch_shape()["autotune_launches"] > 0
    out.zero_()
    again.launch(d_coefs, out)
    torch.cuda.synchronize()
    for i in range(nf):
        np.testing.assert_array_equal(out[i].cpu().numpy().view(np.uint32), exp, err_msg=f"cached shape, frame {i}")


def _mixed_batch(hjd, s, guard=256):
    """Frames of different sizes (right and bottom edge strips), qtables and
    output pitches in one plan; returns (specs, coefs, qts, expected, bytes)."""
    sizes = [(1920, 1080), (313, 234), (3840, 64), (1000, 17), (1920, 1080), (257, 600)]
    specs, coefs, qts, exps, off_blk, off_b = [], [], [], [], 0, guard
    for i, (w, h) in enumerate(sizes):
        c, q = O.synthetic_coefs(w, h, s, seed=70 + i + 10 * s, quality_scale=0.6 + 0.2 * i)
        pitch = 4 * w + 16 * (i % 3)
        specs.append(hjd.FrameSpec(w, h, s, coef_offset=off_blk, out_offset=off_b, out_pitch=pitch,
                                   qt_index=(3 * i, 3 * i + 1, 3 * i + 2)))
        coefs.append(c); qts.append(q); exps.append((O.decode_q16(c, q, w, h, s), off_b, pitch, w, h))
        off_blk += c.shape[0]; off_b += pitch * h + guard
    return specs, np.concatenate(coefs), np.concatenate(qts), exps, off_b


def _check_mixed(buf, exps, what):
    full = buf.cpu().numpy()
    mask = np.ones(full.shape, bool)
    for e, off, pitch, w, h in exps:
        img = full[off:off + pitch * h].reshape(h, pitch)[:, :4 * w]
        np.testing.assert_array_equal(np.ascontiguousarray(img).view(np.uint32), e, err_msg=f"{w}x{h} {what}")
        mask[off:off + pitch * h].reshape(h, pitch)[:, :4 * w] = False
    assert (full[mask] == 0x5A).all(), f"write outside the frames ({what})"


@pytest.mark.parametrize("s", [0, 1])
def test_every_autotune_candidate_vs_oracle(hjd, ctx, s):
    """every launch shape hjd_plan_autotune can pick --
    1/2/4/8/16 tasks per wave x nt/plain stores, and the workgroup-interleaved
    order with each -- decodes a mixed batch bit-exactly, applied through
    hjd_plan_set_chunk x hjd_plan_set_variant; the shape the plan reports is
    the one asked for (set_chunk pins the chunk exactly, so chunks > 1 really
    run, across frame boundaries and edge strips)."""
    import torch
    specs, coefs, qts, exps, nbytes = _mixed_batch(hjd, s)
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qts)
    plan.set_kernel(hjd.KERNEL_PERSISTENT)
    d_coefs = torch.from_numpy(coefs).cuda()
    buf = torch.empty((nbytes,), dtype=torch.uint8, device="cuda")
    for chunk in (1, 2, 4, 8, 16):
        for variant in (0, 1, 2, 3):
            plan.set_chunk(chunk)
            plan.set_variant(variant)
            shape = plan.launch_shape()
            waves = -(-plan.tasks // chunk)
            assert shape["tasks_per_wave"] == chunk and shape["grid"] == -(-waves // 4), shape
            if variant & 2 == 0:
                assert shape["max_tasks_per_wave"] == -(-plan.tasks // (4 * shape["grid"])), shape
                assert chunk == 1 or shape["max_tasks_per_wave"] > 1, shape
            buf.fill_(0x5A)
            plan.launch(d_coefs, buf)
            torch.cuda.synchronize()
            _check_mixed(buf, exps, f"chunk {chunk} variant {variant}")


@pytest.mark.parametrize("s", [0, 1])
@pytest.mark.parametrize("chunk", [1, 3, 16])
def test_chunking_vs_oracle(hjd, ctx, s, chunk):
    """The persistent kernel's task chunks (hjd_plan_set_chunk) must each
    decode every frame of a mixed batch exactly once, bit-exact -- frames of
    different sizes (right and bottom edge strips), qtables and output pitches,
    output guard bands untouched, over repeated launches.  The chunk applied is
    the one asked for (no occupancy floor on a pinned chunk)."""
    import torch
    specs, coefs, qts, exps, nbytes = _mixed_batch(hjd, s)
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qts)
    plan.set_kernel(hjd.KERNEL_PERSISTENT)
    plan.set_chunk(chunk)
    assert plan.launch_shape()["tasks_per_wave"] == chunk
    assert plan.launch_shape()["max_tasks_per_wave"] >= min(chunk, 2) or chunk == 1
    d_coefs = torch.from_numpy(coefs).cuda()
    buf = torch.full((nbytes,), 0x5A, dtype=torch.uint8, device="cuda")
    for rep in range(3):
        plan.launch(d_coefs, buf)
    torch.cuda.synchronize()
    _check_mixed(buf, exps, f"chunk {chunk}")


def test_set_chunk_keeps_latency_kernel_for_small_auto_plans(hjd, ctx):
    """hjd_plan_set_chunk applies to persistent launches; a small
    HJD_KERNEL_AUTO plan keeps the latency kernel (as hjd_plan_autotune
    leaves it), with the oracle's pixels."""
    import torch
    w, h = 1920, 1080
    coefs, qt = O.synthetic_coefs(w, h, 1, seed=33)
    plan = hjd.Plan(ctx, [hjd.FrameSpec(w, h, 1, qt_index=(0, 1, 2))], hjd.IN_Q16_ZIGZAG, qtables=qt)
    assert plan.tasks <= 1024
    plan.set_chunk(4)
    assert plan.launch_shape()["kernel"] == "latency"
    out = torch.zeros((h, w), dtype=torch.int32, device="cuda")
    plan.launch(torch.from_numpy(coefs).cuda(), out)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), O.decode_q16(coefs, qt, w, h, 1))
    plan.set_kernel(hjd.KERNEL_PERSISTENT)
    assert plan.launch_shape()["kernel"] == "persistent" and plan.launch_shape()["tasks_per_wave"] == 4
