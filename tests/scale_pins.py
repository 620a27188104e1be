"""Config-5 scale pins of the host Huffman decoder: seeded JPEG generators
(the files are MBs, so they are regenerated, not committed) and the hashes of
the reference's own mcu_data for each (tests/golden/make_golden.py writes
them into manifest.json "scale" from oracle/_ref/libref.so, src/decoder.cpp:
338-342).  TEST INFRASTRUCTURE ONLY (tests/, bench.py's config-5 check).

Hashes per file:
  jpeg_sha256        the generated JPEG (a different Pillow/libjpeg build would
                     make different files: the pin then reads "unpinned",
                     not "mismatch");
  mcu_data_sha256    the reference's jpg.mcu_data: int32 natural-order
                     dequantised blocks, MCU-major (the Fast_IDCT inputs);
  coefs_q16_sha256   the same blocks as this library's int16 zigzag quantised
                     coefficients (mcu_data[zz[k]] / qt[k], exact).

The restart-interval case (dri_read_boundary) pins the reference's
read_more_data defect (src/decoder.cpp:122-146: an RSTn whose 0xFF is the
last byte of a 2,048-byte read loses its marker byte, and the reference then
fails with "expected RSTn"): a FHD q50 file re-encoded from reference-pinned
coefficients with DRI = 5 MCUs (tests/jpeg_writer.py), whose coefficients are
therefore known without the reference decoding it.
"""
from __future__ import annotations

import hashlib
import io
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], dtype=np.int64)

# name -> (generator, parameters); "pool" = bench.encode_pool (config 5's own
# pool: 64 distinct 4K q90 4:2:0 files), "synthetic" = gradient + sigma-20 noise
# through Pillow (tests/golden/make_golden.py synthetic_rgb / encode_jpeg)
SCALE_CASES = {
    "bench_pool_4k420_q90": ("pool", dict(w=3840, h=2160, sampling=1, n=64, seed0=7919)),
    "4k444_q90": ("pool", dict(w=3840, h=2160, sampling=0, n=1, seed0=7919)),
    "fhd420_q50": ("synthetic", dict(w=1920, h=1080, quality=50, subsampling=2, seed=501)),
    "odd2049x1111_q30": ("synthetic", dict(w=2049, h=1111, quality=30, subsampling=2, seed=502)),
    "q100_opt_1001x777": ("synthetic", dict(w=1001, h=777, quality=100, subsampling=2, seed=503, optimize=True)),
}

DRI_INTERVAL = 5


def sha(b) -> str:
    if isinstance(b, np.ndarray):
        b = np.ascontiguousarray(b).tobytes()
    return hashlib.sha256(b).hexdigest()


def synthetic_rgb(w, h, seed, sigma=20.0):
    """gradient + iid gaussian noise, clipped (as make_golden)."""
    rng = np.random.default_rng(seed)
    x = np.arange(w)[None, :].astype(np.float64)
    y = np.arange(h)[:, None].astype(np.float64)
    img = np.stack([x * 255.0 / w + 0 * y, y * 255.0 / h + 0 * x, (x + y) * 255.0 / (w + h)], axis=-1)
    img = img + rng.normal(0, sigma, (h, w, 3))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def encode_jpeg(rgb, quality, subsampling, **kw) -> bytes:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(rgb, "RGB").save(buf, format="JPEG", quality=quality, subsampling=subsampling, **kw)
    return buf.getvalue()


def generate(name):
    """The case's JPEG files (list of bytes)."""
    kind, p = SCALE_CASES[name]
    if kind == "pool":
        if REPO not in sys.path:
            sys.path.insert(0, REPO)
        import bench
        return bench.encode_pool(p["w"], p["h"], p["sampling"], p["n"], seed0=p["seed0"])
    kw = {k: v for k, v in p.items() if k not in ("w", "h", "quality", "subsampling", "seed")}
    return [encode_jpeg(synthetic_rgb(p["w"], p["h"], p["seed"]), p["quality"], p["subsampling"], **kw)]


def generate_one(name, k=0):
    """File k of the case (a pool file alone: encode_pool seeds file i with seed0 + i)."""
    kind, p = SCALE_CASES[name]
    if kind != "pool":
        return generate(name)[k]
    if REPO not in sys.path:
        sys.path.insert(0, REPO)
    import bench
    return bench.encode_pool(p["w"], p["h"], p["sampling"], 1, seed0=p["seed0"] + k)[0]


def dri_file(base: bytes, coefs_q16: np.ndarray) -> bytes:
    """`base`'s coefficients re-encoded as one interleaved scan with DRI =
    DRI_INTERVAL MCUs (same tables; tests/jpeg_writer.py)."""
    import jpeg_writer as JW
    data, _ = JW.rewrite_scans(base, coefs_q16, [(0, 1, 2)], DRI_INTERVAL)
    return data


def manifest_scale():
    import json
    with open(os.path.join(HERE, "golden", "manifest.json")) as f:
        return json.load(f).get("scale", {})


def check_coefs(rec: dict, jpeg: bytes, coefs_q16: np.ndarray, qt: np.ndarray, sampling: int,
                natural: bool = True) -> str:
    """'pinned' (the coefficients hash to the reference's), 'unpinned' (this
    box generated a different JPEG, so the pin does not apply) or 'MISMATCH'.
    natural=False checks the int16 form only (bench.py: it is the reference's
    mcu_data divided by the file's tables, exactly, so it pins the same data)."""
    if sha(jpeg) != rec["jpeg_sha256"]:
        return "unpinned"
    if sha(np.ascontiguousarray(coefs_q16, dtype="<i2")) != rec["coefs_q16_sha256"]:
        return "MISMATCH"
    if not natural:
        return "pinned"
    bpm = 6 if sampling == 1 else 3
    comp = np.array(([0] * (bpm - 2) + [1, 2]) * (coefs_q16.shape[0] // bpm))
    nat = np.zeros(coefs_q16.shape, np.int32)
    nat[:, ZIGZAG] = coefs_q16.astype(np.int32) * np.asarray(qt, np.int32).reshape(3, 64)[comp]
    if sha(np.ascontiguousarray(nat, dtype="<i4")) != rec["mcu_data_sha256"]:
        return "MISMATCH"
    return "pinned"
