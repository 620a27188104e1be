"""GPU: the speculative sync of latency decoders (ent_spec_kernel,
ent_cand_kernel, ent_chain_kernel; DESIGN.md s10 "Single-image latency") on
the device.  Decoders sized for one or two frames use it by default; here
HJD_SYNC_SPEC=1 forces it on every decoder and stream, and every test of
test_gpu_entropy.py runs again (imported below): coefficients equal the host
decoder's, pixels the reference's and the oracle's, damaged files flagged.
The lead-in sweep at small S drives the chain kernel's repair path."""
import numpy as np
import pytest

import test_gpu_entropy as E
from test_gpu_entropy import *  # noqa: F401,F403  (re-run the whole module with the speculative sync)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _spec_sync(monkeypatch):
    monkeypatch.setenv("HJD_SYNC_SPEC", "1")
    yield


@pytest.mark.parametrize("lead", [0, 256, 1024])
@pytest.mark.parametrize("sub_bits", [64, 512])
def test_lead_in_sweep_on_device(hjd, ctx, monkeypatch, lead, sub_bits):
    monkeypatch.setenv("HJD_SPEC_LEAD", str(lead))
    datas = [E._pil(1920, 1080, 90, 2, seed=61), E._pil(640, 480, 95, 0, seed=62, restart_marker_blocks=3),
             E._pil(333, 77, 85, 1, seed=63)] + [d for _, d in E._golden_bytes()[:2]]
    got, status = E._coefs_gpu(hjd, ctx, datas, sub_bits)
    for d, g, s in zip(datas, got, status):
        ref, _ = hjd.decode_coefs(d)
        np.testing.assert_array_equal(g, ref)
        assert s & ~1 == 0


def test_single_image_default_is_speculative(hjd, ctx, monkeypatch):
    """A one-frame decoder takes the speculative sync without the override."""
    monkeypatch.delenv("HJD_SYNC_SPEC", raising=False)
    import torch
    d = E._pil(1920, 1080, 90, 2, seed=64)
    info = hjd.parse(d)
    out = torch.full((info.height, info.width), -1, dtype=torch.int32, device="cuda")
    with hjd.GpuDecoder(ctx, 1, len(d), info.nblocks) as gd:
        for _ in range(3):
            gd.decode([d], [out])
            assert gd.sync()[0] & ~1 == 0
    ref, info = hjd.decode_coefs(d)
    import oracle_py as O
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32),
                                  O.decode_q16(ref, info.qt, info.width, info.height, info.sampling))


def test_lead_ladder_after_a_repair(hjd, ctx, monkeypatch):
    """A latency decoder whose chain needed a repair (status bit 0) decodes the
    next frames with a longer lead-in (spec_lead_bits' ladder): this frame
    breaks at 512 bits and not at 1536 (pinned by the emulation,
    test_entropy_emulation_spec.py), so the first call reports a repair and
    the next ones none; every call's coefficients are exact."""
    monkeypatch.delenv("HJD_SYNC_SPEC", raising=False)
    monkeypatch.delenv("HJD_SPEC_LEAD", raising=False)
    import torch
    d = E._pil(1920, 1080, 90, 0, seed=5)
    ref, info = hjd.decode_coefs(d)
    coefs = torch.empty((info.nblocks, 64), dtype=torch.int16, device="cuda")
    bits = []
    with hjd.GpuDecoder(ctx, 1, len(d), info.nblocks) as gd:
        for _ in range(3):
            coefs.fill_(0x5A5A)
            gd.decode_coefs([d], coefs)
            bits.append(gd.sync()[0])
            np.testing.assert_array_equal(coefs.cpu().numpy(), ref)
    assert bits == [1, 0, 0]


@pytest.mark.parametrize("q,sub,seed", [(95, 2, 3), (97, 0, 3), (98, 2, 3), (100, 2, 8)])
def test_dense_single_images_take_the_round_based_tiers(hjd, ctx, monkeypatch, q, sub, seed):
    """Latency decoders leave the speculative sync for dense scans (> 200 bits
    per block) and run the round-based one at a longer S than their own
    (kDenseTiers: 1024, 2048, 8192 for these four FHD frames of 232, 301,
    322 and 436 bits per block).  Coefficients and pixels stay exact, the
    decoder reused across calls."""
    monkeypatch.delenv("HJD_SYNC_SPEC", raising=False)
    monkeypatch.delenv("HJD_SPEC_LEAD", raising=False)
    import torch
    import oracle_py as O
    d = E._pil(1920, 1080, q, sub, seed=seed)
    ref, info = hjd.decode_coefs(d)
    coefs = torch.empty((info.nblocks, 64), dtype=torch.int16, device="cuda")
    out = torch.full((info.height, info.width), -1, dtype=torch.int32, device="cuda")
    with hjd.GpuDecoder(ctx, 1, len(d), info.nblocks) as gd:
        for _ in range(2):
            coefs.fill_(0x5A5A)
            gd.decode_coefs([d], coefs)
            assert gd.sync()[0] & ~1 == 0
            np.testing.assert_array_equal(coefs.cpu().numpy(), ref)
        gd.decode([d], [out])
        gd.sync()
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32),
                                  O.decode_q16(ref, info.qt, info.width, info.height, info.sampling))


def test_early_pull_and_a_late_destuff_error(hjd, ctx, monkeypatch):
    """A lone large scan is pulled to the GPU in two parts, the first while the
    host still destuffs (gdec_early_pull).  A wrong RSTn near the end fails the
    host destuff after that first pull; the same decoder then decodes a good
    file exactly (the early pull of the failed call cannot leak into it)."""
    monkeypatch.delenv("HJD_SYNC_SPEC", raising=False)
    import torch
    import oracle_py as O
    good = E._pil(1920, 1080, 95, 2, seed=71, restart_marker_blocks=8)
    info = hjd.parse(good)
    assert len(good) - info.scan_offset >= 256 << 10   # the early pull's threshold
    at = good.rindex(b"\xff\xd0", 0, len(good) - 64)    # a late RST0
    bad = good[:at + 1] + bytes([0xD0 + (good[at + 1] - 0xD0 + 3) % 8]) + good[at + 2:]
    assert at > info.scan_offset + (len(good) - info.scan_offset) * 3 // 4
    out = torch.full((info.height, info.width), -1, dtype=torch.int32, device="cuda")
    ref, rinfo = hjd.decode_coefs(good)
    exp = O.decode_q16(ref, rinfo.qt, rinfo.width, rinfo.height, rinfo.sampling)
    with hjd.GpuDecoder(ctx, 1, len(good), info.nblocks) as gd:
        for _ in range(2):
            with pytest.raises(Exception, match="expected RST"):
                gd.decode([bad], [out])
            gd.decode([good], [out])
            assert gd.sync()[0] & ~1 == 0
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), exp)
