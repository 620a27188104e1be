"""The drop-in boundary: libhjd.so replaces src/oclDCT8x8.cpp (+ OpenCL) behind
the reference's src/idct.h (include/idct.h has the same declarations).

CPU: every idct.h symbol is exported with the reference's mangled name, and
     every symbol the reference's own callers (decoder.cpp, main.cpp) leave
     undefined resolves in libhjd.so.
GPU: oracle/_ref/ref_dropin -- the reference's main.cpp + decoder.cpp (GPU
     build, no USE_CPU_ONLY) + parser/bitstream/huffman, linked against
     libhjd.so -- decodes the reference's sample JPEG on the MI355X and writes
     the BMP whose pixels are bit-identical to the reference CPU path.
"""
import ctypes
import hashlib
import os
import shutil
import subprocess
import tempfile

import numpy as np
import pytest

import oracle_py as O

REPO = O.REPO
LIB = os.path.join(REPO, "ocljpegdecoder_amd", "lib", "libhjd.so")
DROPIN = os.path.join(REPO, "oracle", "_ref", "ref_dropin")

# src/idct.h:4-18 with C++ (Itanium) mangling, as `nm` shows them for the
# reference objects.
IDCT_H_SYMBOLS = [
    "_Z20Initialize_Fast_IDCTv", "_Z9Fast_IDCTPi", "_Z7idctrowPi", "_Z7idctcolPi",
    "_Z22Initialize_OpenCL_IDCTv", "_Z13clidct_createv", "_Z22clidct_allocate_memoryimmii",
    "_Z30clidct_transfer_data_to_devicePA64_Kiii", "_Z12clidct_build10ColorSpace", "_Z10clidct_run10ColorSpace",
    "_Z32clidct_retrieve_data_from_devicePA64_i", "_Z33clidct_retrieve_image_from_devicePvmm",
    "_Z26clidct_wait_for_completionv", "_Z15clidct_clean_upv",
]


def nm_defined(path):
    out = subprocess.run(["nm", "-D", "--defined-only", path], capture_output=True, text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_exports_idct_h_symbols():
    syms = nm_defined(LIB)
    missing = [s for s in IDCT_H_SYMBOLS if s not in syms]
    assert not missing, missing


def test_exports_every_c_abi_symbol():
    """Every function declared in include/hjd.h and include/hjd_host.h is exported."""
    import re
    syms = nm_defined(LIB)
    for h in ("hjd.h", "hjd_host.h"):
        text = open(os.path.join(REPO, "include", h)).read()
        decls = set(re.findall(r"^\s*(?:int|int64_t|const char\*)\s+(hjd_\w+)\s*\(", text, re.M))
        assert decls, h
        missing = sorted(d for d in decls if d not in syms)
        assert not missing, (h, missing)


@pytest.mark.skipif(not os.path.exists(os.path.join(REPO, "oracle", "_ref", "gpu_decoder.o")),
                    reason="reference objects not built here (no /root/reference)")
def test_reference_callers_resolve_in_libhjd():
    """Undefined symbols of the reference's idct.h callers == what libhjd provides."""
    ref = os.path.join(REPO, "oracle", "_ref")
    needed = set()
    for o in ("gpu_decoder.o", "gpu_main.o"):
        out = subprocess.run(["nm", "-u", os.path.join(ref, o)], capture_output=True, text=True, check=True).stdout
        needed |= {l.split()[-1] for l in out.splitlines() if "clidct" in l or "IDCT" in l or "idct" in l}
    assert needed, "no idct.h references found"
    assert needed <= set(IDCT_H_SYMBOLS), needed - set(IDCT_H_SYMBOLS)
    assert needed <= nm_defined(LIB)


def test_cpu_entry_points_match_reference_vectors():
    """Fast_IDCT / idctrow / idctcol (the USE_CPU_ONLY API) are bit-exact."""
    lib = ctypes.CDLL(LIB)
    fast = getattr(lib, "_Z9Fast_IDCTPi")
    fast.argtypes = [ctypes.POINTER(ctypes.c_int32)]
    getattr(lib, "_Z20Initialize_Fast_IDCTv")()
    z = np.load(O.GOLDEN + "/idct_vectors.npz")
    blocks = z["inp"].copy()
    for b in blocks:
        fast(b.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    np.testing.assert_array_equal(blocks, z["out"])


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built")
@pytest.mark.parametrize("name", ["JPEG_example_JPG_RIP_050", "syn444_odd_41x23_q75", "syn420_160x48_q95_dri"])
def test_reference_program_on_mi355x(name):
    """The reference's own host program, GPU build, linked to libhjd.so."""
    rec = O.manifest()["cases"][name]
    tmp = tempfile.mkdtemp(prefix="hjd_dropin_")
    try:
        jpg = os.path.join(tmp, "in.jpg")
        shutil.copy(os.path.join(O.GOLDEN, name + ".jpg"), jpg)
        r = subprocess.run([DROPIN, jpg], cwd=tmp, capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
        assert "HIP device selected" in r.stdout
        bmp = open(os.path.join(tmp, "m:\\output.bmp"), "rb").read()
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    w, h = rec["width"], rec["height"]
    assert len(bmp) == 54 + w * h * 4          # GPU path writes exactly H rows
    import ocljpegdecoder_amd as hjd
    assert bmp[:54] == hjd.bmp_header(w, h)    # our BMP sink writes the reference's header
    px = bmp[54:]
    assert hashlib.sha256(px).hexdigest() == rec["bgrx_sha256"]


def _fnv1a(b: bytes) -> int:
    h = 1469598103934665603
    for c in np.frombuffer(b, np.uint8).tolist():
        h = ((h ^ c) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


@pytest.mark.gpu
@pytest.mark.skipif(not os.path.exists(DROPIN), reason="oracle/_ref/ref_dropin not built")
def test_reference_program_many_images_one_process():
    """The reference program decodes several files per process (src/main.cpp:31-39)
    and runs the whole idct.h lifecycle per image (src/decoder.cpp:202-216,
    :518-521).  The shim keeps context, stream, buffers and plans across images:
    the first image allocates, a smaller image of a new geometry only builds a
    plan, the first geometry again allocates and builds nothing -- and every
    image's retrieved pixels are the reference's (FNV-1a of the BGRX rows)."""
    names = ["JPEG_example_JPG_RIP_050", "syn444_odd_41x23_q75", "JPEG_example_JPG_RIP_050", "syn420_160x48_q95_dri"]
    tmp = tempfile.mkdtemp(prefix="hjd_dropin_multi_")
    try:
        files = []
        for i, n in enumerate(names):
            files.append(os.path.join(tmp, f"{i}.jpg"))
            shutil.copy(os.path.join(O.GOLDEN, n + ".jpg"), files[-1])
        env = dict(os.environ, HJD_COMPAT_STATS="1")
        r = subprocess.run([DROPIN, *files], cwd=tmp, capture_output=True, text=True, timeout=120, env=env)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    stats = [dict(kv.split("=", 1) for kv in l.split()[1:]) for l in r.stderr.splitlines()
             if l.startswith("[hjd-compat]")]
    assert [int(s["image"]) for s in stats] == [1, 2, 3, 4], r.stderr[-2000:]
    allocs = [int(s["allocs"]) for s in stats]
    plans = [int(s["plans_built"]) for s in stats]
    assert allocs[0] >= 2 and allocs[1:] == [0, 0, 0], allocs     # growth only: image 1 is the largest
    assert plans == [1, 1, 0, 1], plans                              # plan cache hit for the repeated geometry
    for n, s in zip(names, stats):
        c = O.load_case(n)
        assert int(s["fnv"], 16) == _fnv1a(np.ascontiguousarray(c["bgrx"]).tobytes()), n
