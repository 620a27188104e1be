"""GPU destuff ("Destuff on the GPU"): scan bytes that reach the
device raw -- from pinned caller memory, or forced with HJD_DESTUFF=device --
are destuffed by destuff_{count,scan,write}_kernel instead of the host's
destuff() (which restates the reference's read_more_data byte handling,
src/decoder.cpp:94-159, and its RST handling, :288-307).

1. The kernels alone against the host routine on adversarial byte strings
   (stuffing, fill bytes, RSTn in and out of order, truncation at FF, scan end
   markers) around the 64-byte thread and 16-KiB tile boundaries.
2. Whole decodes: every test of test_gpu_entropy.py again with
   HJD_DESTUFF=device (imported below, so they run in this module too), and
   pinned-memory inputs through GpuDecoder and GpuJpegStream, whose host scan
   bytes must be zero.
"""
import ctypes

import numpy as np
import pytest

import oracle_py as O
import test_gpu_entropy as E
from test_gpu_entropy import *  # noqa: F401,F403  (re-run the whole module with device destuff)

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _device_destuff(monkeypatch):
    monkeypatch.setenv("HJD_DESTUFF", "device")
    yield


def _u8p(a):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))


def _host(hjd, scan):
    lib = hjd._lib.load()
    out = np.zeros(len(scan) + 64, np.uint8)
    seg = np.zeros(len(scan) + 2, np.uint32)
    nseg, nb = ctypes.c_int(0), ctypes.c_int64(0)
    rc = lib.hjd_debug_destuff_host(_u8p(scan), len(scan), _u8p(out), out.size,
                                    seg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), seg.size,
                                    ctypes.byref(nseg), ctypes.byref(nb))
    if rc != 0:
        return None
    return out[:nb.value].copy(), seg[:nseg.value].copy()


def _gpu(hjd, ctx, scan, nseg):
    lib = hjd._lib.load()
    out = np.zeros(((len(scan) + 64 + 15) // 16) * 16, np.uint8)
    seg = np.zeros(nseg, np.uint32)
    nb, st = ctypes.c_int64(0), ctypes.c_uint32(0)
    hjd._lib.check(lib.hjd_debug_destuff_gpu(ctx.handle, _u8p(scan), len(scan), nseg, _u8p(out), out.size,
                                             seg.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(nb),
                                             ctypes.byref(st)), "hjd_debug_destuff_gpu")
    return out, nb.value, seg, st.value


def _adversarial(rng, n, p_ff=0.02, rst=True):
    """Random scan bytes with FF pairs of every kind sprinkled in."""
    a = rng.integers(0, 255, n, dtype=np.uint8)            # 0..254: no FF by chance
    pos = np.sort(rng.choice(n - 1, size=max(1, int(n * p_ff)), replace=False))
    nrst = 0
    for p in pos:
        if a[p - 1] == 0xFF if p > 0 else False:
            continue
        kind = rng.random()
        a[p] = 0xFF
        if kind < 0.55:
            a[p + 1] = 0x00                                 # stuffed FF
        elif kind < 0.75:
            a[p + 1] = 0xFF                                 # fill byte (next FF starts a pair)
            if p + 2 < n:
                a[p + 2] = 0x00
        elif rst:
            a[p + 1] = 0xD0 + (nrst & 7)                    # restart marker, in order
            nrst += 1
        else:
            a[p + 1] = 0x00
    return a


def _check(hjd, ctx, scan, nseg_expect=None):
    h = _host(hjd, scan)
    if h is None:                                           # host rejects (RSTn out of order)
        nseg = nseg_expect or 1
        _, _, _, st = _gpu(hjd, ctx, scan, nseg)
        assert st & 2, "GPU accepted a scan the host rejects"
        return "rejected"
    data, seg = h
    nseg = nseg_expect or len(seg)
    out, nb, gseg, st = _gpu(hjd, ctx, scan, nseg)
    if len(seg) != nseg or len(data) == 0:
        assert st & 2, "GPU accepted a wrong restart count / empty scan"
        return "count"
    assert st == 0, st
    assert nb == len(data)
    np.testing.assert_array_equal(out[:nb], data)
    assert (out[nb:nb + 64] == 0xFF).all(), "read-ahead pad"
    np.testing.assert_array_equal(gseg, seg)
    return "ok"


@pytest.mark.parametrize("n", [1, 2, 63, 64, 65, 127, 16383, 16384, 16385, 3 * 16384 + 17, 200_003])
def test_destuff_kernels_vs_host_random(hjd, ctx, n):
    rng = np.random.default_rng(n)
    seen = set()
    for trial in range(6):
        scan = _adversarial(rng, max(n, 2), p_ff=[0.0, 0.001, 0.01, 0.05, 0.2, 0.4][trial])[:n].copy()
        seen.add(_check(hjd, ctx, scan))
    assert "ok" in seen or n < 3          # a 1-2 byte string with an FF pair is an empty scan


def test_destuff_kernels_edges(hjd, ctx):
    cases = {
        "ff_at_end": bytes([1, 2, 3, 0xFF]),
        "stuffed_at_end": bytes([1, 0xFF, 0x00]),
        "fill_then_eoi": bytes([7, 0xFF, 0xFF, 0xFF, 0xD9, 5, 5]),
        "fill_then_rst": bytes([7, 0xFF, 0xFF, 0xD0, 8, 0xFF, 0x00]),
        "ff_ff_00": bytes([0xFF, 0xFF, 0x00, 9]),
        "eoi_first": bytes([0xFF, 0xD9, 1, 2]),
        "rst_out_of_order": bytes([1, 0xFF, 0xD1, 2]),
        "rst_wraps": bytes(sum(([i, 0xFF, 0xD0 + (i & 7)] for i in range(19)), []) + [42]),
        "rst_then_eoi": bytes([1, 0xFF, 0xD0, 2, 0xFF, 0xD9]),
        "sof_marker_ends": bytes([1, 2, 0xFF, 0xC0, 0xFF, 0xD0]),
    }
    for name, b in cases.items():
        scan = np.frombuffer(b, np.uint8).copy()
        _check(hjd, ctx, scan)
    # restart count mismatch: host finds 1 interval, the header promised 3
    r = _check(hjd, ctx, np.frombuffer(bytes([1, 2, 3]), np.uint8).copy(), nseg_expect=3)
    assert r == "count"


def test_destuff_marker_across_boundaries(hjd, ctx):
    """FF as the last byte of a thread's 64 / a tile's 16384 bytes, its second
    byte in the next thread / tile."""
    for cut in (63, 127, 16383, 2 * 16384 - 1):
        for second in (0x00, 0xFF, 0xD0, 0xD9):
            scan = np.full(cut + 70, 0x11, np.uint8)
            scan[cut] = 0xFF
            scan[cut + 1] = second
            if second == 0xFF:
                scan[cut + 2] = 0x00
            _check(hjd, ctx, scan)


def _pil_files():
    out = []
    for i, kw in enumerate(E.SYN[:3] + E.SYN[4:6]):        # plain, 4:4:4, q100, DRI by blocks
        kw = dict(kw)
        out.append(E._pil(kw.pop("w"), kw.pop("h"), kw.pop("q"), kw.pop("sub"), seed=300 + i, **kw))
    return out + [d for _, d in E._golden_bytes()]


def test_pinned_inputs_gpu_decoder(hjd, ctx, monkeypatch):
    """HJD_DESTUFF=auto (the default): pinned bytes take the device path."""
    import torch
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    datas = _pil_files()
    pinned = [hjd.pinned_bytes(d) for d in datas]
    infos = [hjd.parse(d) for d in datas]
    total = sum(i.nblocks for i in infos)
    coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), total) as gd:
        offs = gd.decode_coefs(pinned, coefs)
        status = gd.sync()
    host = coefs.cpu().numpy()
    for d, o, i, s in zip(datas, offs, infos, status):
        ref, _ = hjd.decode_coefs(d)
        np.testing.assert_array_equal(host[o:o + i.nblocks], ref)
        assert s & ~1 == 0


def test_pinned_scans_in_separate_registrations(hjd, ctx, monkeypatch):
    """Two scans in separately page-locked ranges that lie less than 64 KiB
    apart: the decoder mirrors their distance and tries one DMA over both,
    which crosses the unregistered page between them and is rejected; it then
    copies the scans one by one (torch's pinned blocks can lie this close)."""
    import mmap
    import torch
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    datas = _pil_files()[:2]
    page = mmap.PAGESIZE
    n1 = -(-len(datas[0]) // page) * page
    n2 = -(-len(datas[1]) // page) * page
    mm = mmap.mmap(-1, n1 + page + n2)
    arr = np.frombuffer(mm, np.uint8)
    o1 = n1 - len(datas[0])                      # file 1 ends where region 1 ends
    o2 = n1 + page                               # file 2 starts region 2, one page later
    arr[o1:o1 + len(datas[0])] = np.frombuffer(datas[0], np.uint8)
    arr[o2:o2 + len(datas[1])] = np.frombuffer(datas[1], np.uint8)
    lib = hjd._lib.load()
    base = arr.ctypes.data
    hjd._lib.check(lib.hjd_host_register(ctypes.c_void_p(base), n1), "register 1")
    hjd._lib.check(lib.hjd_host_register(ctypes.c_void_p(base + o2), n2), "register 2")
    views = None
    try:
        views = [torch.from_numpy(arr[o1:o1 + len(datas[0])]), torch.from_numpy(arr[o2:o2 + len(datas[1])])]
        infos = [hjd.parse(d) for d in datas]
        total = sum(i.nblocks for i in infos)
        coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")
        # raw-area capacity for the mirrored layout: both scans plus the page between
        with hjd.GpuDecoder(ctx, 2, n1 + page + n2 + (1 << 16), total) as gd:
            offs = gd.decode_coefs(views, coefs)
            status = gd.sync()
        host = coefs.cpu().numpy()
        for d, o, i, s in zip(datas, offs, infos, status):
            ref, _ = hjd.decode_coefs(d)
            np.testing.assert_array_equal(host[o:o + i.nblocks], ref)
            assert s & ~1 == 0
    finally:
        lib.hjd_host_unregister(ctypes.c_void_p(base + o2))
        lib.hjd_host_unregister(ctypes.c_void_p(base))
        views = None   # the mapping goes with its last reference


def _registered_layout(hjd, datas, gaps, first=5):
    """The files in one anonymous mapping, file i+1 starting gaps[i] bytes after
    file i ends; files sharing a page are page-locked together, the others in
    registrations of their own (hjd_host_register), so the gaps between the
    registrations are unregistered pages.  Returns (views, cleanup)."""
    import mmap
    import torch
    page = mmap.PAGESIZE
    pos, starts = first, []
    for d, g in zip(datas, list(gaps) + [0]):
        starts.append(pos)
        pos += len(d) + int(g)
    size = -(-(pos + page) // page) * page
    mm = mmap.mmap(-1, size)
    arr = np.frombuffer(mm, np.uint8)
    for s, d in zip(starts, datas):
        arr[s:s + len(d)] = np.frombuffer(d, np.uint8)
    groups = []                                     # [first page, last page] per registration
    for s, d in zip(starts, datas):
        p0, p1 = s // page, (s + len(d) - 1) // page
        if groups and p0 <= groups[-1][1]:
            groups[-1][1] = max(groups[-1][1], p1)
        else:
            groups.append([p0, p1])
    lib = hjd._lib.load()
    base = arr.ctypes.data
    done = []
    for p0, p1 in groups:
        hjd._lib.check(lib.hjd_host_register(ctypes.c_void_p(base + p0 * page), (p1 - p0 + 1) * page), "register")
        done.append(base + p0 * page)
    views = [torch.from_numpy(arr[s:s + len(d)]) for s, d in zip(starts, datas)]

    def cleanup():
        for p in done:
            lib.hjd_host_unregister(ctypes.c_void_p(p))
    return views, cleanup, len(groups)


@pytest.mark.parametrize("policy", ["auto", "device"])
def test_pinned_separate_registrations_exact_capacity(hjd, ctx, monkeypatch, policy):
    """scans in separately page-locked regions at gaps of
    1 B to 60 KiB, decoder capacity exactly the sum of the file sizes (the
    documented sizing): every frame decodes bit-exactly on the device path
    (no host destuff), whatever the gaps cost the mirrored DMA layout."""
    import torch
    monkeypatch.setenv("HJD_DESTUFF", policy)
    base = _pil_files()
    datas = (base * 3)[:14]
    gaps = [1, 3, 40, 4096 + 5, 61440, 2 * 4096 + 1, 16, 20000, 60 * 1024, 7, 100, 8191, 2]
    views, cleanup, nreg = _registered_layout(hjd, datas, gaps)
    try:
        assert nreg >= 6
        infos = [hjd.parse(d) for d in datas]
        total = sum(i.nblocks for i in infos)
        coefs = torch.full((total + 64, 64), 0x5A5A, dtype=torch.int16, device="cuda")
        with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), total) as gd:
            for _ in range(2):
                coefs.fill_(0x5A5A)
                offs = gd.decode_coefs(views, coefs)
                assert gd.last_bytes()["host_scan_bytes"] == 0
                status = gd.sync()
                host = coefs.cpu().numpy()
                for d, o, i, s in zip(datas, offs, infos, status):
                    ref, _ = hjd.decode_coefs(d)
                    np.testing.assert_array_equal(host[o:o + i.nblocks], ref)
                    assert s & ~1 == 0
                assert (host[total:] == 0x5A5A).all()
    finally:
        views = None
        cleanup()


def test_pinned_capacity_by_entropy_bytes_falls_back_to_host(hjd, ctx, monkeypatch):
    """sized by entropy-coded bytes (the older sizing), pinned
    frames whose raw scans would not fit are destuffed on the host in auto
    mode instead of failing the batch; HJD_DESTUFF=device reports it."""
    import torch
    datas = _pil_files()
    ent = 0
    for d in datas:
        scan = np.frombuffer(d[hjd.parse(d).scan_offset:], np.uint8).copy()
        ent += len(_host(hjd, scan)[0])
    pinned = [hjd.pinned_bytes(d) for d in datas]
    infos = [hjd.parse(d) for d in datas]
    total = sum(i.nblocks for i in infos)
    coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    with hjd.GpuDecoder(ctx, len(datas), ent, total) as gd:
        offs = gd.decode_coefs(pinned, coefs)
        assert gd.last_bytes()["host_scan_bytes"] > 0
        status = gd.sync()
        host = coefs.cpu().numpy()
        for d, o, i, s in zip(datas, offs, infos, status):
            ref, _ = hjd.decode_coefs(d)
            np.testing.assert_array_equal(host[o:o + i.nblocks], ref)
            assert s & ~1 == 0
        monkeypatch.setenv("HJD_DESTUFF", "device")
        with pytest.raises(hjd._lib.HjdError):
            gd.decode_coefs(pinned, coefs)


def test_pinned_capacity_by_raw_scan_bytes_stays_on_device(hjd, ctx, monkeypatch):
    """sized by the files' entropy-coded bytes as they lie in
    the file (stuffing and markers included: size - scan_offset), every pinned
    frame's raw scan fits, so none may fall back to the host destuff -- the
    placement must not reserve whole file sizes for the frames still to come."""
    import torch
    datas = _pil_files()
    raw = sum(len(d) - hjd.parse(d).scan_offset for d in datas)
    pinned = [hjd.pinned_bytes(d) for d in datas]
    infos = [hjd.parse(d) for d in datas]
    total = sum(i.nblocks for i in infos)
    coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    with hjd.GpuDecoder(ctx, len(datas), raw, total) as gd:
        offs = gd.decode_coefs(pinned, coefs)
        assert gd.last_bytes()["host_scan_bytes"] == 0
        status = gd.sync()
        host = coefs.cpu().numpy()
        for d, o, i, s in zip(datas, offs, infos, status):
            ref, _ = hjd.decode_coefs(d)
            np.testing.assert_array_equal(host[o:o + i.nblocks], ref)
            assert s & ~1 == 0


def test_pinned_input_reusable_on_return(hjd, ctx, monkeypatch):
    """hjd_gdec_decode* may return before the kernels run, but
    not before the DMA has read the caller's pinned bytes; overwriting them
    right after the call must not change the result."""
    import torch
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    datas = [E._pil(2048, 1536, 95, 0, seed=41), E._pil(1920, 1080, 90, 2, seed=42)] + _pil_files()[:2]
    infos = [hjd.parse(d) for d in datas]
    total = sum(i.nblocks for i in infos)
    coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)), total) as gd:
        for rep in range(3):
            pinned = [hjd.pinned_bytes(d) for d in datas]
            offs = gd.decode_coefs(pinned, coefs)
            for p in pinned:
                p.fill_(0xFF)                  # the caller reuses its buffers at once
            status = gd.sync()
            host = coefs.cpu().numpy()
            for d, o, i, s in zip(datas, offs, infos, status):
                ref, _ = hjd.decode_coefs(d)
                np.testing.assert_array_equal(host[o:o + i.nblocks], ref)
                assert s & ~1 == 0


@pytest.mark.parametrize("policy", ["auto", "device"])
def test_small_last_scan_tight_decoder(hjd, ctx, monkeypatch, policy):
    """the destuff kernels walk a frame's whole last 16-KiB
    tile; a small scan that ends a tightly sized raw area must decode (lanes
    past the scan's end load nothing)."""
    import torch
    monkeypatch.setenv("HJD_DESTUFF", policy)
    for d in [E._pil(1, 1, 90, 2, seed=3), E._pil(33, 17, 90, 0, seed=4), E._pil(64, 64, 50, 2, seed=5)]:
        info = hjd.parse(d)
        p = hjd.pinned_bytes(d)
        coefs = torch.full((info.nblocks, 64), 0x5A5A, dtype=torch.int16, device="cuda")
        with hjd.GpuDecoder(ctx, 1, len(d), info.nblocks) as gd:
            gd.decode_coefs([p], coefs)
            assert gd.last_bytes()["host_scan_bytes"] == 0
            assert gd.sync()[0] & ~1 == 0
        ref, _ = hjd.decode_coefs(d)
        np.testing.assert_array_equal(coefs.cpu().numpy(), ref)


def test_pinned_inputs_stream_no_host_scan_bytes(hjd, ctx, monkeypatch):
    import torch
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    datas = _pil_files()
    infos = [hjd.parse(d) for d in datas]
    pinned = [hjd.pinned_bytes(d) for d in datas]
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    with hjd.GpuJpegStream(ctx, 4, 4 * max(map(len, datas)) + (1 << 16), 4 * max(i.nblocks for i in infos),
                           nslots=3, nthreads=2) as st:
        for p, o in zip(pinned, outs):
            st.submit(p, o)
        s1 = st.sync()
        assert s1["host_scan_bytes"] == 0, s1
        for d, o in zip(datas, outs):                       # pageable bytes: destuffed on the host
            st.submit(d, o)
        s2 = st.sync()
        assert s2["host_scan_bytes"] > 0
    for d, o, i in zip(datas, outs, infos):
        ref, info = hjd.decode_coefs(d)
        exp = O.decode_q16(ref, info.qt, info.width, info.height, info.sampling)
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)


def _arena(hjd, datas, seed):
    """JPEG files back to back in ONE pinned buffer, at odd offsets (as a loader
    reading files into a pinned ring would leave them): views into it."""
    import torch
    rng = np.random.default_rng(seed)
    gaps = rng.integers(0, 40, len(datas))
    total = int(sum(len(d) for d in datas) + gaps.sum() + 64)
    arena = torch.zeros(total, dtype=torch.uint8).pin_memory()
    views, pos = [], int(rng.integers(1, 16))
    for d, g in zip(datas, gaps):
        arena[pos:pos + len(d)] = torch.frombuffer(bytearray(d), dtype=torch.uint8)
        views.append(arena[pos:pos + len(d)])
        pos += len(d) + int(g)
    return arena, views


def test_pinned_arena_runs_gpu_decoder(hjd, ctx, monkeypatch):
    """Adjacent files in one pinned arena: their scans are placed at the same
    distance in the raw area (unaligned starts) and move in one DMA per run."""
    import torch
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    datas = _pil_files()
    arena, views = _arena(hjd, datas, seed=5)
    infos = [hjd.parse(d) for d in datas]
    total = sum(i.nblocks for i in infos)
    coefs = torch.full((total, 64), 0x5A5A, dtype=torch.int16, device="cuda")
    with hjd.GpuDecoder(ctx, len(datas), sum(map(len, datas)) + 4096, total) as gd:
        for _ in range(2):
            offs = gd.decode_coefs(views, coefs)
            status = gd.sync()
            host = coefs.cpu().numpy()
            for d, o, i, s in zip(datas, offs, infos, status):
                ref, _ = hjd.decode_coefs(d)
                np.testing.assert_array_equal(host[o:o + i.nblocks], ref)
                assert s & ~1 == 0
    del arena


def test_pinned_arena_stream(hjd, ctx, monkeypatch):
    import torch
    monkeypatch.setenv("HJD_DESTUFF", "auto")
    datas = _pil_files() * 3
    arena, views = _arena(hjd, datas, seed=9)
    infos = [hjd.parse(d) for d in datas]
    outs = [torch.full((i.height, i.width), -1, dtype=torch.int32, device="cuda") for i in infos]
    with hjd.GpuJpegStream(ctx, 5, 5 * max(map(len, datas)) + (1 << 16), 5 * max(i.nblocks for i in infos),
                           nslots=3, nthreads=3) as st:
        for v, o in zip(views, outs):
            st.submit(v, o)
        stats = st.sync()
    assert stats["host_scan_bytes"] == 0
    for d, o, i in zip(datas, outs, infos):
        ref, info = hjd.decode_coefs(d)
        exp = O.decode_q16(ref, info.qt, info.width, info.height, info.sampling)
        np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), exp)
    del arena
