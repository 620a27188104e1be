"""ctypes access to the CPU oracle (oracle/liboracle.so) and, when built, the
reference itself (oracle/_ref/libref.so).  TEST INFRASTRUCTURE ONLY: used by
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker.
"""
from __future__ import annotations

import ctypes
import glob
import json
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_LIB = os.path.join(ORACLE_DIR, "liboracle.so")
REF_LIB = os.path.join(ORACLE_DIR, "_ref", "libref.so")
GOLDEN = os.path.join(REPO, "tests", "golden")

i16p = ctypes.POINTER(ctypes.c_int16)
i32p = ctypes.POINTER(ctypes.c_int32)
u32p = ctypes.POINTER(ctypes.c_uint32)

_oracle = None
_ref = None


def _p(a, t):
    return a.ctypes.data_as(t)


def oracle():
    global _oracle
    if _oracle is None:
        if not os.path.exists(ORACLE_LIB):
            subprocess.run(["make", "-s", "-C", ORACLE_DIR, "oracle"], check=True)
        lib = ctypes.CDLL(ORACLE_LIB)
        lib.oracle_fast_idct.argtypes = [i32p]
        lib.oracle_dequant_block.argtypes = [i16p, i32p, i32p]
        lib.oracle_yuv_to_bgrx.argtypes = [ctypes.c_int32] * 3
        lib.oracle_yuv_to_bgrx.restype = ctypes.c_uint32
        lib.oracle_yuv_to_bgrx_n.argtypes = [i32p, i32p, i32p, u32p, ctypes.c_int64]
        lib.oracle_decode_frame_q16.argtypes = [i16p, i32p, i32p, i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                                u32p, ctypes.c_int]
        lib.oracle_decode_frame_i32.argtypes = [i32p, ctypes.c_int, ctypes.c_int, ctypes.c_int, u32p, ctypes.c_int]
        lib.oracle_idct_blocks.argtypes = [i32p, i32p, ctypes.c_int64]
        lib.oracle_decode_batch_q16_mt.argtypes = [i16p, ctypes.c_int64, ctypes.c_int, i32p, i32p, i32p,
                                                   ctypes.c_int, ctypes.c_int, ctypes.c_int, u32p, ctypes.c_int64,
                                                   ctypes.c_int, ctypes.c_int]
        _oracle = lib
    return _oracle


def ref_available() -> bool:
    return os.path.exists(REF_LIB)


def ref():
    """The reference CPU path compiled from /root/reference/src (may be absent)."""
    global _ref
    if _ref is None:
        lib = ctypes.CDLL(REF_LIB)
        lib.ref_init()
        lib.ref_fast_idct_n.argtypes = [i32p, ctypes.c_int64]
        lib.ref_yuv_to_rgb32_n.argtypes = [i32p, i32p, i32p, u32p, ctypes.c_int64]
        _ref = lib
    return _ref


# --- oracle wrappers ---------------------------------------------------------
def idct_blocks(blocks: np.ndarray) -> np.ndarray:
    b = np.ascontiguousarray(blocks, dtype=np.int32).reshape(-1, 64)
    out = np.empty_like(b)
    oracle().oracle_idct_blocks(_p(b, i32p), _p(out, i32p), b.shape[0])
    return out


def yuv_to_bgrx(y, u, v) -> np.ndarray:
    y, u, v = (np.ascontiguousarray(a, dtype=np.int32) for a in (y, u, v))
    out = np.empty(y.shape, dtype=np.uint32)
    oracle().oracle_yuv_to_bgrx_n(_p(y, i32p), _p(u, i32p), _p(v, i32p), _p(out, u32p), y.size)
    return out


def decode_q16(coefs: np.ndarray, qt: np.ndarray, width: int, height: int, sampling: int) -> np.ndarray:
    c = np.ascontiguousarray(coefs, dtype=np.int16)
    q = np.ascontiguousarray(qt, dtype=np.int32).reshape(3, 64)
    out = np.zeros((height, width), dtype=np.uint32)
    rc = oracle().oracle_decode_frame_q16(_p(c, i16p), _p(q[0], i32p), _p(q[1], i32p), _p(q[2], i32p), width,
                                          height, sampling, _p(out, u32p), width)
    assert rc == 0
    return out


def decode_i32(mcu_data: np.ndarray, width: int, height: int, sampling: int) -> np.ndarray:
    m = np.ascontiguousarray(mcu_data, dtype=np.int32)
    out = np.zeros((height, width), dtype=np.uint32)
    rc = oracle().oracle_decode_frame_i32(_p(m, i32p), width, height, sampling, _p(out, u32p), width)
    assert rc == 0
    return out


def dequant_natural(coefs: np.ndarray, qt: np.ndarray, sampling: int) -> np.ndarray:
    """int16 zigzag + per-component qtables -> int32 natural (jpg.mcu_data)."""
    from_zz = np.array(ZIGZAG)
    c = np.asarray(coefs, dtype=np.int32).reshape(-1, 64)
    comp = block_components(sampling, c.shape[0])
    q = np.asarray(qt, dtype=np.int32).reshape(3, 64)[comp]
    out = np.zeros_like(c)
    out[:, from_zz] = c * q
    return out


ZIGZAG = [0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
          12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
          35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
          58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63]


# --- golden fixtures -----------------------------------------------------------
def manifest():
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


def golden_cases():
    return sorted(manifest()["cases"].keys())


def load_case(name):
    z = np.load(os.path.join(GOLDEN, name + ".npz"))
    return {k: z[k] for k in z.files}


# --- synthetic coefficient frames (legal domain by construction) ---------------
def synthetic_coefs(width, height, sampling, seed=0, quality_scale=1.0):
    """Quantised zigzag coefficients of a synthetic frame: per-block random
    smooth+noise pixels -> float FDCT -> quantise with IJG-like tables.  Fast
    enough for multi-megapixel frames; the legal domain is guaranteed because
    the coefficients come from bounded samples."""
    rng = np.random.default_rng(seed)
    nblk = frame_blocks(width, height, sampling)
    k = np.arange(8)
    cc = np.where(k == 0, 1 / np.sqrt(2), 1.0)
    m = np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16) * cc[:, None] / 2
    base = rng.integers(-100, 100, (nblk, 1, 1))
    grad = rng.normal(0, 6, (nblk, 2, 1, 1))
    yy, xx = np.meshgrid(np.arange(8), np.arange(8), indexing="ij")
    pix = base + grad[:, 0] * yy + grad[:, 1] * xx + rng.normal(0, 20, (nblk, 8, 8))
    pix = np.clip(pix, -128, 127)
    F = np.einsum("ux,nxy,vy->nuv", m, pix, m).reshape(nblk, 64)
    qt = std_qtables(quality_scale)
    comp = block_components(sampling, nblk)
    qnat = np.zeros((3, 64), np.int32)
    qnat[:, ZIGZAG] = qt
    coef_nat = np.rint(F / qnat[comp]).astype(np.int32)
    coefs = np.ascontiguousarray(coef_nat[:, ZIGZAG].astype(np.int16))
    return coefs, qt


def std_qtables(scale=1.0):
    """JPEG Annex K luminance/chrominance tables (zigzag/file order), scaled."""
    lum = np.array([16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55,
                    14, 13, 16, 24, 40, 57, 69, 56, 14, 17, 22, 29, 51, 87, 80, 62,
                    18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113, 92,
                    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99])
    chr_ = np.array([17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                     24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99] + [99] * 32)
    nat = np.stack([lum, chr_, chr_])
    zz = np.empty_like(nat)
    zz[:, :] = nat[:, ZIGZAG]   # natural -> file order
    return np.clip(np.rint(zz * scale), 1, 255).astype(np.int32)


# sampling (include/hjd.h codes) -> (MCU px width, MCU px height, blocks per MCU,
# luma blocks per MCU); 3 (4:2:2), 4 (gray), 5 (4:1:1, Y H4V1) and 6 (4:4:0,
# Y H1V2) are the extensions of oracle.h
GEOM = {0: (8, 8, 3, 1), 1: (16, 16, 6, 4), 3: (16, 8, 4, 2), 4: (8, 8, 1, 1), 5: (32, 8, 6, 4), 6: (8, 16, 4, 2)}


def frame_blocks(width, height, sampling):
    pw, ph, bpm, _ = GEOM[sampling]
    return ((width - 1) // pw + 1) * ((height - 1) // ph + 1) * bpm


def block_components(sampling, nblocks):
    """Component (0 Y, 1 Cb, 2 Cr) of each block of an MCU-major block list."""
    _, _, bpm, nluma = GEOM[sampling]
    return np.array(([0] * nluma + [1, 2][: bpm - nluma]) * (nblocks // bpm))
