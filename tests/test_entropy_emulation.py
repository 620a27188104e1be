"""CPU: the GPU entropy-decode algorithm (self-synchronising parallel decode,
DESIGN.md s10), run on the host through the test hook
hjd_debug_entropy_emulate with the same state machine the kernels use
(csrc/hjd_entropy.hpp), must reproduce the host Huffman decoder's
coefficients exactly -- and those are pinned to the reference's own
mcu_data (tests/test_jpeg_host.py).  Subsequence sizes from 32 bits up force
every boundary case: entries inside codes, inside padding, exactly on restart
boundaries, and chains that only meet in the sequential fallback."""
import io
import os

import numpy as np
import pytest

import oracle_py as O


def _pil(w, h, q, sub, seed, noise=20.0, gray=False, **kw):
    from PIL import Image
    rng = np.random.default_rng(seed)
    x = np.linspace(0, 255, w)[None, :, None]
    y = np.linspace(0, 255, h)[:, None, None]
    img = np.clip(x * [1, 0, 0.5] + y * [0, 1, 0.5] + rng.normal(0, noise, (h, w, 3)), 0, 255).astype(np.uint8)
    im = Image.fromarray(img)
    if gray:
        im = im.convert("L")
    b = io.BytesIO()
    im.save(b, format="JPEG", quality=q, subsampling=sub, **kw)
    return b.getvalue()


@pytest.mark.parametrize("sub_bits", [32, 64, 100, 1024, 4096, 8192, 16384])
def test_golden_files(hjd, sub_bits):
    for name in O.golden_cases():
        data = open(os.path.join(O.GOLDEN, name + ".jpg"), "rb").read()
        ref, _ = hjd.decode_coefs(data)
        got, status = hjd.emulate_entropy(data, sub_bits)
        np.testing.assert_array_equal(got, ref, err_msg=f"{name} S={sub_bits}")
        assert status & ~1 == 0


def test_reference_sample_mcu_hash(hjd):
    """The emulated decode of the reference's sample, dequantised, hashes to
    the reference's mcu_data."""
    import hashlib
    data = open(os.path.join(O.GOLDEN, "JPEG_example_JPG_RIP_050.jpg"), "rb").read()
    info = hjd.parse(data)
    coefs, _ = hjd.emulate_entropy(data, 256)
    nat = O.dequant_natural(coefs, info.qt, info.sampling)
    assert hashlib.sha256(nat.astype("<i4").tobytes()).hexdigest() == (
        "c25806f5238c8ec7c2a4846cf6b67c5b567fd268599591392baf77e91023924e")


CASES = [
    ("640x480 q90 4:2:0", dict(w=640, h=480, q=90, sub=2)),
    ("640x480 q90 4:4:4", dict(w=640, h=480, q=90, sub=0)),
    ("600x400 q100 4:4:4", dict(w=600, h=400, q=100, sub=0)),
    ("640x480 q40 4:2:0", dict(w=640, h=480, q=40, sub=2)),
    ("640x480 DRI 1 MCU", dict(w=640, h=480, q=90, sub=2, restart_marker_blocks=1)),
    ("640x480 DRI 3 MCUs", dict(w=640, h=480, q=95, sub=0, restart_marker_blocks=3)),
    ("640x480 DRI 1 row", dict(w=640, h=480, q=90, sub=0, restart_marker_rows=1)),
    ("640x480 optimized", dict(w=640, h=480, q=75, sub=2, optimize=True)),
    ("1x1", dict(w=1, h=1, q=90, sub=2)),
    ("17x9 DRI 1", dict(w=17, h=9, q=90, sub=0, restart_marker_blocks=1)),
    # extensions: 4:2:2 and one-component scans
    ("640x480 q90 4:2:2", dict(w=640, h=480, q=90, sub=1)),
    ("333x77 4:2:2 DRI 2", dict(w=333, h=77, q=85, sub=1, restart_marker_blocks=2)),
    ("640x480 q90 gray", dict(w=640, h=480, q=90, sub=0, gray=True)),
    ("333x77 gray DRI 7", dict(w=333, h=77, q=70, sub=0, gray=True, restart_marker_blocks=7)),
    ("9x17 gray", dict(w=9, h=17, q=95, sub=0, gray=True)),
]


@pytest.mark.parametrize("name,kw", CASES, ids=[c[0] for c in CASES])
@pytest.mark.parametrize("sub_bits", [32, 160, 1024, 2048])
def test_synthetic(hjd, name, kw, sub_bits):
    kw = dict(kw)
    data = _pil(kw.pop("w"), kw.pop("h"), kw.pop("q"), kw.pop("sub"), seed=len(name) * 31 + sub_bits, **kw)
    ref, _ = hjd.decode_coefs(data)
    got, status = hjd.emulate_entropy(data, sub_bits)
    np.testing.assert_array_equal(got, ref)
    assert status & ~1 == 0


def test_random_sweep(hjd):
    """Seeded random files x subsequence sizes, including pure-noise content
    (the worst case for self-synchronisation), all four samplings.  This sweep
    found the stale-segment-index convergence bug (csrc/hjd_entropy.hpp
    same_state): a 158x82 4:2:2 file with a 2-MCU restart interval at S=32,
    where a wrong chain crossed a restart pad as data and met the true
    (pos, z, j) with the previous segment's index."""
    from PIL import Image
    rng = np.random.default_rng(2024)
    done = 0
    while done < 150:
        w, h = int(rng.integers(8, 200)), int(rng.integers(8, 160))
        kw = {}
        r = int(rng.integers(0, 3))
        if r == 1:
            kw["restart_marker_blocks"] = int(rng.integers(1, 9))
        elif r == 2:
            kw["restart_marker_rows"] = 1
        img = (rng.integers(0, 256, (h, w, 3), dtype=np.uint8) if rng.integers(0, 3) == 0 else
               np.clip(rng.normal(128, rng.uniform(0, 60), (h, w, 3)), 0, 255).astype(np.uint8))
        b = io.BytesIO()
        im = Image.fromarray(img)
        if rng.integers(0, 6) == 0:
            im = im.convert("L")
        try:
            im.save(b, format="JPEG", quality=int(rng.integers(20, 101)), subsampling=int(rng.choice([0, 1, 2])), **kw)
        except OSError:
            continue
        data = b.getvalue()
        sub_bits = int(rng.choice([32, 33, 64, 127, 256, 1000, 1024]))
        ref, _ = hjd.decode_coefs(data)
        got, status = hjd.emulate_entropy(data, sub_bits)
        np.testing.assert_array_equal(got, ref, err_msg=f"{w}x{h} {kw} S={sub_bits}")
        done += 1


def test_corrupt_inputs_rejected(hjd):
    data = _pil(64, 48, 90, 2, seed=3, restart_marker_blocks=2)
    # wrong RST sequence number
    i = data.index(b"\xff\xd1")
    bad = data[:i] + b"\xff\xd3" + data[i + 2:]
    with pytest.raises(hjd._lib.HjdError):
        hjd.emulate_entropy(bad)
    # scan cut short: fewer blocks than the frame needs
    info = hjd.parse(data)
    cut = data[: info.scan_offset + 40] + b"\xff\xd9"
    with pytest.raises(hjd._lib.HjdError):
        hjd.emulate_entropy(cut)


def test_emulation_asan_fuzz():
    """The GPU entropy decoder's algorithm (host build of the same destuff,
    sync/link/repair and write code) under AddressSanitizer + UBSan, fed
    damaged single-scan JPEGs of several sizes at random S
    (tools/fuzz/run_entropy.sh): no read past a frame's padded bit string, no
    write past its blocks, corrupt data flagged rather than decoded."""
    import os
    import shutil
    import subprocess
    if shutil.which("g++") is None or not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("no toolchain")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run(["bash", os.path.join(root, "tools", "fuzz", "run_entropy.sh"), "150"], capture_output=True,
                       text=True, timeout=900)
    assert p.returncode == 0, (p.stdout + p.stderr)[-3000:]
    assert "entropy mutants" in p.stdout


def test_damaged_files_match_host_decoder(hjd):
    """Differential check on damaged files (byte flips, 0xFF / RSTn insertions,
    truncation): whenever the GPU algorithm (host emulation) reports a frame
    clean, its coefficients equal the host decoder's.  Found two semantic gaps,
    now closed: a restart interval that decodes to a different MCU count than
    DRI is corrupt (write path checks each interval's first block), and FF FF
    is a fill byte before the pair, as in the reference's read_more_data."""
    from test_gpu_entropy import _mutants
    seeds = [_pil(256, 128, 90, 2, seed=31), _pil(160, 96, 95, 0, seed=32, restart_marker_blocks=5),
             _pil(200, 100, 75, 1, seed=33), _pil(120, 88, 85, 2, seed=34, restart_marker_blocks=3)]
    clean = 0
    for rnd in range(3):
        for i, d in enumerate(_mutants(seeds, 200, seed=100 + rnd)):
            try:
                got, status = hjd.emulate_entropy(d, [32, 64, 256, 1024][i % 4])
            except Exception:
                continue
            if status & ~1:
                continue
            try:
                ref, _ = hjd.decode_coefs(d)
            except Exception:
                continue
            np.testing.assert_array_equal(got, ref, err_msg=f"round {rnd} mutant {i}")
            clean += 1
    assert clean > 20


@pytest.mark.parametrize("case", ["golden", "fhd_q90", "q100_444", "dri1", "q40", "optimized", "multiscan_first"])
def test_sync_step_decode_equals_unit_decode(hjd, case):
    """The sync kernels' run (AC step tables, several units per lookup, both
    lookups computed by every lane and selected) gives exactly the exit state
    and statistics of the unit-by-unit decode, from guessed entries at every
    block-in-MCU phase and a few bit offsets, and from true unit boundaries
    (hjd_debug_entropy_sync_check)."""
    import ctypes
    import oracle_py as O
    if case == "golden":
        data = open(os.path.join(O.GOLDEN, "JPEG_example_JPG_RIP_050.jpg"), "rb").read()
    elif case == "multiscan_first":
        import jpeg_writer as JW
        base = _pil(200, 120, 90, 2, seed=4)
        data = JW.rewrite_scans(base, hjd.decode_coefs(base)[0], [(1, 2), (0,)], 3)[0]
    else:
        kw = {"fhd_q90": dict(w=640, h=360, q=90, sub=2), "q100_444": dict(w=320, h=200, q=100, sub=0),
              "dri1": dict(w=300, h=180, q=90, sub=2, restart_marker_blocks=1),
              "q40": dict(w=400, h=300, q=40, sub=2), "optimized": dict(w=400, h=240, q=85, sub=1, optimize=True)}[case]
        kw = dict(kw)
        data = _pil(kw.pop("w"), kw.pop("h"), kw.pop("q"), kw.pop("sub"), seed=11, **kw)
    lib = hjd._lib.load()
    runs, bad = ctypes.c_int64(0), ctypes.c_int64(0)
    buf = (ctypes.c_uint8 * len(data)).from_buffer_copy(data)
    for S in (64, 512, 2048):
        assert lib.hjd_debug_entropy_sync_check(buf, len(data), S, ctypes.byref(runs), ctypes.byref(bad)) == 0
        assert runs.value > 0 and bad.value == 0, (case, S, runs.value, bad.value)
