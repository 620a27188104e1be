"""GPU: Huffman decode on the device (hjd_gdec) through the C
ABI.  Coefficients must equal the host decoder's exactly (that decoder is
pinned to the reference's mcu_data in tests/test_jpeg_host.py); pixels must
equal the reference's BGRX on the golden files and the oracle elsewhere."""
import io
import os

import numpy as np
import pytest

import oracle_py as O
from test_entropy_emulation import _pil

pytestmark = pytest.mark.gpu


def _golden_bytes():
    return [(n, open(os.path.join(O.GOLDEN, n + ".jpg"), "rb").read()) for n in O.golden_cases()]


def _coefs_gpu(hjd, ctx, datas, sub_bits=0):
    import torch
    infos = [hjd.parse(d) for d in datas]
    total = sum(i.nblocks for i in infos)
    coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, len(datas), sum(len(d) for d in datas), total, sub_bits) as gd:
        offs = gd.decode_coefs(datas, coefs)
        status = gd.sync()
    host = coefs.cpu().numpy()
    return [host[o:o + i.nblocks] for o, i in zip(offs, infos)], status


@pytest.mark.parametrize("sub_bits", [32, 256, 1024, 8192])
def test_golden_coefficients(hjd, ctx, sub_bits):
    cases = _golden_bytes()
    got, status = _coefs_gpu(hjd, ctx, [d for _, d in cases], sub_bits)
    for (name, d), g, s in zip(cases, got, status):
        ref, _ = hjd.decode_coefs(d)
        np.testing.assert_array_equal(g, ref, err_msg=f"{name} S={sub_bits}")
        assert s & ~1 == 0


def test_golden_pixels_match_reference(hjd, ctx):
    import torch
    cases = _golden_bytes()
    datas = [d for _, d in cases]
    exp = [O.load_case(n)["bgrx"] for n, _ in cases]
    outs = [torch.full(e.shape, -1, dtype=torch.int32, device="cuda") for e in exp]
    infos = [hjd.parse(d) for d in datas]
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), sum(i.nblocks for i in infos)) as gd:
        gd.decode(datas, outs)
        gd.sync()
    for (n, _), o, e in zip(cases, outs, exp):
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), e, err_msg=n)


SYN = [
    dict(w=1920, h=1080, q=90, sub=2),
    dict(w=1280, h=720, q=90, sub=0),
    dict(w=1000, h=700, q=100, sub=0),
    dict(w=800, h=600, q=40, sub=2),
    dict(w=1024, h=768, q=90, sub=2, restart_marker_blocks=1),
    dict(w=1024, h=768, q=95, sub=0, restart_marker_blocks=5),
    dict(w=1024, h=768, q=90, sub=2, restart_marker_rows=1),
    dict(w=1024, h=768, q=75, sub=2, optimize=True),
    dict(w=1, h=1, q=90, sub=2),
    dict(w=33, h=17, q=90, sub=0, restart_marker_blocks=1),
]


@pytest.mark.parametrize("sub_bits", [64, 1024])
def test_mixed_batch_coefficients(hjd, ctx, sub_bits):
    datas = []
    for i, kw in enumerate(SYN):
        kw = dict(kw)
        datas.append(_pil(kw.pop("w"), kw.pop("h"), kw.pop("q"), kw.pop("sub"), seed=100 + i, **kw))
    got, status = _coefs_gpu(hjd, ctx, datas, sub_bits)
    for i, (d, g) in enumerate(zip(datas, got)):
        ref, _ = hjd.decode_coefs(d)
        np.testing.assert_array_equal(g, ref, err_msg=f"case {i} {SYN[i]} S={sub_bits}")
    assert all(s & ~1 == 0 for s in status)


def test_mixed_batch_pixels_match_oracle(hjd, ctx):
    import torch
    datas = []
    for i, kw in enumerate(SYN):
        kw = dict(kw)
        datas.append(_pil(kw.pop("w"), kw.pop("h"), kw.pop("q"), kw.pop("sub"), seed=200 + i, **kw))
    infos = [hjd.parse(d) for d in datas]
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), sum(i.nblocks for i in infos)) as gd:
        gd.decode(datas, outs)
        gd.sync()
    for d, o, info in zip(datas, outs, infos):
        coefs, _ = hjd.decode_coefs(d)
        exp = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


@pytest.mark.parametrize("sub_bits", [0, 8192])
def test_4k_frames(hjd, ctx, sub_bits):
    """Full-size 4K frames (BASELINE configs[4] input), both samplings; S = 8192
    is the stream's subsequence length."""
    datas = [_pil(3840, 2160, 90, 2, seed=7), _pil(3840, 2160, 90, 0, seed=8)]
    got, status = _coefs_gpu(hjd, ctx, datas, sub_bits)
    for d, g in zip(datas, got):
        ref, _ = hjd.decode_coefs(d)
        np.testing.assert_array_equal(g, ref)
    assert all(s & ~1 == 0 for s in status)   # bit 0: a chain repair ran (informational)


def test_repeated_calls_reuse_staging(hjd, ctx):
    """Back-to-back calls on one decoder (the second waits for the first's
    uploads); results stay exact."""
    import torch
    datas = [_pil(640, 480, 90, 2, seed=s) for s in range(4)]
    infos = [hjd.parse(d) for d in datas]
    outs = [[torch.empty((i.height, i.width), dtype=torch.int32, device="cuda") for i in infos] for _ in range(3)]
    with hjd.GpuDecoder(ctx, 4, sum(map(len, datas)), sum(i.nblocks for i in infos)) as gd:
        for k in range(3):
            gd.decode(datas, outs[k])
        gd.sync()
    for k in range(3):
        for d, o, info in zip(datas, outs[k], infos):
            coefs, _ = hjd.decode_coefs(d)
            exp = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
            np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


def test_corrupt_scan_reported(hjd, ctx):
    """A scan cut short decodes without faulting and is reported per frame."""
    import torch
    good = _pil(256, 128, 90, 2, seed=1)
    info = hjd.parse(good)
    cut = good[: info.scan_offset + 300] + b"\xff\xd9"
    coefs = torch.zeros((2 * info.nblocks, 64), dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, 2, 2 * len(good), 2 * info.nblocks) as gd:
        gd.decode_coefs([good, cut], coefs)
        status = gd.sync(raise_on_error=False)
        assert status[0] & ~1 == 0 and status[1] & ~1 != 0
        with pytest.raises(hjd._lib.HjdError):
            gd.decode_coefs([good, cut], coefs)
            gd.sync()


def test_capacity_errors(hjd, ctx):
    import torch
    d = _pil(256, 128, 90, 2, seed=2)
    info = hjd.parse(d)
    coefs = torch.zeros((info.nblocks, 64), dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, 1, len(d), info.nblocks) as gd:
        with pytest.raises(hjd._lib.HjdError):
            gd.decode_coefs([d, d], coefs)           # too many frames
    with hjd.GpuDecoder(ctx, 2, len(d) // 2, 2 * info.nblocks) as gd:
        with pytest.raises(hjd._lib.HjdError):
            gd.decode_coefs([d], coefs)              # too many scan bytes


@pytest.mark.parametrize("max_frames,nslots,nthreads", [(3, 2, 1), (5, 3, 4), (16, 4, 16), (32, 3, 8)])
def test_gstream_many_images(hjd, ctx, max_frames, nslots, nthreads):
    """GPU-entropy stream: many files of mixed geometry through rotating batches;
    pixels equal the reference's (golden) or the oracle on the host-decoded
    coefficients."""
    import torch
    files = []
    for name, d in _golden_bytes():
        files.append((d, O.load_case(name)["bgrx"]))
    rng = np.random.default_rng(max_frames * 13 + nslots)
    for i in range(14):
        w, h = int(rng.integers(1, 900)), int(rng.integers(1, 400))
        kw = {"restart_marker_blocks": int(rng.integers(1, 9))} if i % 3 == 0 else {}
        d = _pil(w, h, int(rng.integers(30, 100)), int(rng.choice([0, 2])), seed=i, **kw)
        coefs, info = hjd.decode_coefs(d)
        files.append((d, O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)))
    files = files * 2
    infos = [hjd.parse(d) for d, _ in files]
    cap_bytes = max(len(d) for d, _ in files) * max_frames + (1 << 16)
    cap_blocks = max(i.nblocks for i in infos) * max_frames
    outs = [torch.full(e.shape, -1, dtype=torch.int32, device="cuda") for _, e in files]
    with hjd.GpuJpegStream(ctx, max_frames, cap_bytes, cap_blocks, nslots=nslots, nthreads=nthreads) as st:
        for (d, _), o in zip(files, outs):
            st.submit(d, o)
        stats = st.sync()
        # the stream stays usable after a sync
        st.submit(files[0][0], outs[0])
        st.sync()
    assert stats["images"] == len(files)
    assert stats["batches"] >= -(-len(files) // max_frames)
    for (d, e), o in zip(files, outs):
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), e)


def test_gstream_bad_file_reported(hjd, ctx):
    import torch
    good = _pil(200, 100, 90, 2, seed=5)
    info = hjd.parse(good)
    cut = good[: info.scan_offset + 200] + b"\xff\xd9"
    outs = [torch.zeros((100, 200), dtype=torch.int32, device="cuda") for _ in range(3)]
    with hjd.GpuJpegStream(ctx, 4, 4 * len(good), 4 * info.nblocks, nslots=2, nthreads=2) as st:
        st.submit(good, outs[0])
        st.submit(cut, outs[1])
        st.submit(good, outs[2])
        with pytest.raises(hjd._lib.HjdError):
            st.sync()
        st.submit(good, outs[1])     # usable again
        st.sync()
    coefs, _ = hjd.decode_coefs(good)
    exp = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
    for o in outs:
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


def test_gstream_host_outputs(hjd, ctx):
    """D2H sink: pixels copied back into host memory (numpy and pinned torch),
    mixed with device outputs in the same batches."""
    import torch
    datas = [_pil(int(w), int(h), 90, sub, seed=300 + i, **kw) for i, (w, h, sub, kw) in enumerate(
        [(640, 480, 2, {}), (333, 177, 0, {}), (1024, 768, 2, {"restart_marker_blocks": 2}), (17, 9, 0, {})] * 3)]
    infos = [hjd.parse(d) for d in datas]
    outs = []
    for i, info in enumerate(infos):
        if i % 3 == 0:
            outs.append(np.full((info.height, info.width), -1, dtype=np.int32))
        elif i % 3 == 1:
            outs.append(torch.full((info.height, info.width), -1, dtype=torch.int32).pin_memory())
        else:
            outs.append(torch.full((info.height, info.width), -1, dtype=torch.int32, device="cuda"))
    cap_b = max(len(d) for d in datas) * 4 + (1 << 16)
    with hjd.GpuJpegStream(ctx, 4, cap_b, 4 * max(i.nblocks for i in infos), nslots=2, nthreads=4) as st:
        for d, o in zip(datas, outs):
            st.submit(d, o)
        st.sync()
    for d, o, info in zip(datas, outs, infos):
        coefs, _ = hjd.decode_coefs(d)
        exp = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
        got = o if isinstance(o, np.ndarray) else o.cpu().numpy()
        np.testing.assert_array_equal(got.view(np.uint32), exp)


def test_calls_on_different_streams_are_ordered(hjd, ctx):
    """Back-to-back calls on two streams reuse the decoder's device buffers;
    the second must not overwrite them under the first."""
    import torch
    datas = [_pil(1280, 720, 90, 2, seed=s) for s in range(3)]
    infos = [hjd.parse(d) for d in datas]
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    outs = [[torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos] for _ in range(4)]
    with hjd.GpuDecoder(ctx, 3, sum(map(len, datas)), sum(i.nblocks for i in infos)) as gd:
        for k in range(4):
            gd.decode(datas, outs[k], s1 if k % 2 == 0 else s2)
        gd.sync()
    torch.cuda.synchronize()
    for d, info, *os_ in zip(datas, infos, *outs):
        coefs, _ = hjd.decode_coefs(d)
        exp = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
        for o in os_:
            np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


def test_gstream_concurrent_submitters(hjd, ctx):
    """Several host threads submitting to one GPU-entropy stream."""
    import threading

    import torch
    datas = [_pil(320 + 16 * i, 200, 90, 2 if i % 2 else 0, seed=400 + i) for i in range(8)]
    infos = [hjd.parse(d) for d in datas]
    jobs = [(datas[i % 8], infos[i % 8]) for i in range(48)]
    outs = [torch.full((inf.height, inf.width), -1, dtype=torch.int32, device="cuda") for _, inf in jobs]
    cap_b = max(map(len, datas)) * 3 + (1 << 16)
    with hjd.GpuJpegStream(ctx, 3, cap_b, 3 * max(i.nblocks for i in infos), nslots=2, nthreads=4) as st:
        def worker(k):
            for i in range(k, len(jobs), 4):
                st.submit(jobs[i][0], outs[i])
        ts = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        st.sync()
    for (d, info), o in zip(jobs, outs):
        coefs, _ = hjd.decode_coefs(d)
        exp = O.decode_q16(coefs, info.qt, info.width, info.height, info.sampling)
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


@pytest.mark.parametrize("sub_bits", [32, 96, 1024])
def test_random_sweep_on_device(hjd, ctx, sub_bits):
    """The device kernels on seeded random files of all four samplings, with
    and without restart intervals, pure noise included (the host mirror of
    the same logic is swept in test_entropy_emulation.py): coefficients equal
    the host decoder's, batches of 40."""
    from PIL import Image
    rng = np.random.default_rng(77 + sub_bits)
    datas = []
    while len(datas) < 160:
        w, h = int(rng.integers(8, 300)), int(rng.integers(8, 200))
        kw = {}
        r = int(rng.integers(0, 3))
        if r == 1:
            kw["restart_marker_blocks"] = int(rng.integers(1, 6))
        elif r == 2:
            kw["restart_marker_rows"] = 1
        img = (rng.integers(0, 256, (h, w, 3), dtype=np.uint8) if rng.integers(0, 3) == 0 else
               np.clip(rng.normal(128, rng.uniform(0, 60), (h, w, 3)), 0, 255).astype(np.uint8))
        im = Image.fromarray(img)
        if rng.integers(0, 5) == 0:
            im = im.convert("L")
        b = io.BytesIO()
        try:
            im.save(b, format="JPEG", quality=int(rng.integers(20, 101)), subsampling=int(rng.choice([0, 1, 2])), **kw)
        except OSError:
            continue
        datas.append(b.getvalue())
    for k in range(0, len(datas), 40):
        chunk = datas[k:k + 40]
        got, status = _coefs_gpu(hjd, ctx, chunk, sub_bits)
        for i, (d, g) in enumerate(zip(chunk, got)):
            ref, _ = hjd.decode_coefs(d)
            np.testing.assert_array_equal(g, ref, err_msg=f"file {k + i} S={sub_bits}")
        assert all(s & ~1 == 0 for s in status)


def test_progressive_rejected_loudly(hjd, ctx):
    """The device decoder takes one interleaved sequential scan; a progressive
    file is refused with a message naming the host path (no silent fallback)."""
    import torch
    prog = _pil(64, 48, 90, 2, seed=3, progressive=True)
    info = hjd.parse(prog)
    assert info.process == 2 and not info.single_scan
    coefs = torch.zeros((info.nblocks, 64), dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, 1, len(prog), info.nblocks) as gd:
        with pytest.raises(hjd._lib.HjdError, match="host decoder"):
            gd.decode_coefs([prog], coefs)


def _mutants(seeds, n, seed):
    """Damaged copies of sequential JPEGs (byte flips, 0xFF / RSTn insertions,
    truncation) that still parse as sequential files (one scan or several)."""
    import ocljpegdecoder_amd as hjd
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < n:
        d = bytearray(seeds[int(rng.integers(len(seeds)))])
        for _ in range(int(rng.integers(1, 9))):
            at = int(rng.integers(len(d)))
            kind = int(rng.integers(4))
            if kind == 0:
                d[at] = 0xFF
            elif kind == 1 and at + 1 < len(d):
                d[at], d[at + 1] = 0xFF, 0xD0 + int(rng.integers(8))
            else:
                d[at] = int(rng.integers(256))
        if rng.integers(4) == 0:
            d = d[: int(rng.integers(1, len(d) + 1))]
        try:
            info = hjd.parse(bytes(d))
        except Exception:
            continue
        if info.process != 2 and 0 < info.nblocks <= 4096:
            out.append(bytes(d))
    return out


@pytest.mark.parametrize("multiscan", [False, True])
@pytest.mark.parametrize("pinned", [False, True])
def test_damaged_files_on_device(hjd, ctx, pinned, multiscan):
    """Damaged JPEGs through the device decoder (host destuff for pageable
    bytes, the device destuff kernels for pinned ones) in batches of 8: no
    fault, no write outside the batch's coefficient blocks (guard blocks keep
    their sentinel), and every frame reported clean decodes to exactly the
    host decoder's coefficients (the host emulation of the same code is
    ASan-fuzzed on the CPU, tests/test_entropy_emulation.py)."""
    import torch
    seeds = [_pil(256, 128, 90, 2, seed=31), _pil(160, 96, 95, 0, seed=32, restart_marker_blocks=5),
             _pil(200, 100, 75, 1, seed=33)]
    if multiscan:   # the same images as sequential files with several scans
        import jpeg_writer as JW
        splits = [[(0,), (1,), (2,)], [(1, 2), (0,)], [(2,), (0, 1)]]
        seeds = [JW.rewrite_scans(d, hjd.decode_coefs(d)[0], splits[k], 4 if k == 1 else 0)[0]
                 for k, d in enumerate(seeds)]
    muts = _mutants(seeds, 96, seed=5 + int(pinned) + 2 * int(multiscan))
    guard = 64
    checked = flagged = staged_out = 0
    # every batch also holds two undamaged files, which must come out clean and
    # exact next to their damaged neighbours
    batches = [[seeds[k % 3], seeds[(k + 1) % 3]] + muts[b0:b0 + 6] for k, b0 in enumerate(range(0, len(muts), 6))]
    while batches:
        datas = batches.pop(0)
        infos = [hjd.parse(d) for d in datas]
        total = sum(i.nblocks for i in infos)
        coefs = torch.full((total + guard, 64), 0x5A5A, dtype=torch.int16, device="cuda")
        inputs = [hjd.pinned_bytes(d) for d in datas] if pinned else datas
        with hjd.GpuDecoder(ctx, len(datas), sum(len(d) for d in datas), total, 64) as gd:
            try:
                offs = gd.decode_coefs(inputs, coefs)
            except hjd._lib.HjdError:
                # rejected while staging (e.g. RSTn out of order on the host
                # destuff path): the whole call fails; retry its frames alone
                if len(datas) > 1:
                    batches += [[d] for d in datas]
                else:
                    staged_out += 1
                continue
            status = gd.sync(raise_on_error=False)
        host = coefs.cpu().numpy()
        assert (host[total:] == 0x5A5A).all(), "write past the batch's blocks"
        for d, o, info, st in zip(datas, offs, infos, status):
            if st & ~1:
                assert d not in seeds, "an undamaged file was flagged"
                flagged += 1
                continue
            try:
                ref, _ = hjd.decode_coefs(d)
            except Exception:
                continue
            np.testing.assert_array_equal(host[o:o + info.nblocks], ref)
            checked += 1
    assert flagged + staged_out > 0 and checked >= 2 * 16, (flagged, staged_out, checked)


@pytest.mark.parametrize("sub_bits", [32, 1024])
def test_edge_coefficients_on_device(hjd, ctx, sub_bits):
    """The host decoder's edge blocks (tests/test_jpeg_host_pair.py: a last
    coefficient at 63, ZRL runs, magnitudes 255/256/1023, DC-only and dense
    blocks; with and without restart markers) through the GPU Huffman decode:
    a batch (round-based sync) and one file per decoder (speculative sync)
    return exactly the encoded coefficients."""
    import jpeg_writer as JW
    from test_jpeg_host_pair import FACTORS, _edge_blocks, _huff_src
    datas, expect = [], []
    for sampling, dri in ((1, 0), (1, 3), (0, 0), (3, 2)):
        w, h = 96, 64
        c = _edge_blocks(O.frame_blocks(w, h, sampling), seed=100 + sampling * 10 + dri)
        _, qt = O.synthetic_coefs(16, 16, sampling, seed=1)
        datas.append(JW.encode_frame(c, w, h, FACTORS[sampling], qt, _huff_src(), restart_interval=dri))
        expect.append(c)
    got, status = _coefs_gpu(hjd, ctx, datas, sub_bits)
    for i, (g, e, s) in enumerate(zip(got, expect, status)):
        assert s & ~1 == 0, (i, s)
        np.testing.assert_array_equal(g, e, err_msg=f"batch file {i} S={sub_bits}")
    for i, (d, e) in enumerate(zip(datas, expect)):
        (g,), (s,) = _coefs_gpu(hjd, ctx, [d], sub_bits)
        assert s & ~1 == 0, (i, s)
        np.testing.assert_array_equal(g, e, err_msg=f"lone file {i} S={sub_bits}")
