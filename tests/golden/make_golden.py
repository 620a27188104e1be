#!/usr/bin/env python3
"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Run in the build container (needs /root/reference and `make -C oracle`):

    python tests/golden/make_golden.py

What it does (everything it writes is data: inputs and the reference's outputs):
  * decodes each case JPEG with the reference's CPU path (USE_CPU_ONLY),
    compiled from /root/reference/src into oracle/_ref/libref.so, capturing
    every Fast_IDCT input/output block (src/decoder.cpp:448-452) and the BMP the
    reference writes (src/decoder.cpp:420-494);
  * derives the int16 quantised zigzag coefficients the kernel consumes as
    mcu_data[zz[k]] / qt[k] (exact: src/decoder.cpp:340 multiplied them);
  * records IDCT known-answer blocks (Fast_IDCT, src/cpuIDCT8x8.cpp:25) and the
    sha256 of the reference colour conversion over all of [-256,255]^3
    (YUV_to_RGB32, src/decoder.cpp:367).
The JPEG inputs are the reference's own sample (test/JPEG_example_JPG_RIP_050.jpg)
and small synthetic frames encoded here with Pillow (SURVEY.md s8(d) recipe).
"""
from __future__ import annotations

import ctypes
import hashlib
import io
import json
import os
import shutil
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_LIB = os.path.join(REPO, "oracle", "_ref", "libref.so")
REF_SAMPLE = "/root/reference/test/JPEG_example_JPG_RIP_050.jpg"

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63], dtype=np.int64)


def parse_headers(data: bytes):
    """Minimal marker walk: DQT tables (file order), SOF0 components."""
    assert data[:2] == b"\xff\xd8"
    pos, qts, comps, dims = 2, {}, [], None
    while pos < len(data):
        assert data[pos] == 0xFF, hex(pos)
        marker = data[pos + 1]
        if marker == 0xDA:
            break
        seg_len = int.from_bytes(data[pos + 2:pos + 4], "big")
        seg = data[pos + 4:pos + 2 + seg_len]
        if marker == 0xDB:
            p = 0
            while p < len(seg):
                pq, tq = seg[p] >> 4, seg[p] & 15
                p += 1
                n = 64 * (pq + 1)
                vals = np.frombuffer(seg[p:p + n], dtype=">u2" if pq else "u1").astype(np.int32)
                qts[tq] = vals
                p += n
        elif marker == 0xC0:
            h, w, nc = int.from_bytes(seg[1:3], "big"), int.from_bytes(seg[3:5], "big"), seg[5]
            dims = (w, h)
            for c in range(nc):
                cid, samp, tq = seg[6 + 3 * c:9 + 3 * c]
                comps.append((cid, samp, tq))
        pos += 2 + seg_len
    return dims, comps, qts


def sampling_of(comps):
    s = [c[1] for c in comps]
    if s == [0x22, 0x11, 0x11]:
        return 1  # HJD_YUV420 == reference ColorSpace::YUV411
    if s == [0x11, 0x11, 0x11]:
        return 0
    raise ValueError(f"unsupported sampling {s}")


class Ref:
    def __init__(self):
        self.lib = ctypes.CDLL(REF_LIB)
        self.lib.ref_init()
        i32p = ctypes.POINTER(ctypes.c_int32)
        self.lib.ref_fast_idct_n.argtypes = [i32p, ctypes.c_int64]
        self.lib.ref_yuv_to_rgb32_n.argtypes = [i32p, i32p, i32p, ctypes.POINTER(ctypes.c_uint32), ctypes.c_int64]
        self.lib.ref_load_jpg.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]

    def decode(self, jpg_path):
        cwd = os.getcwd()
        tmp = tempfile.mkdtemp(prefix="hjd_ref_")
        try:
            os.chdir(tmp)
            rc = self.lib.ref_load_jpg(os.path.abspath(jpg_path).encode(), b"cap_in.bin", b"cap_out.bin")
            assert rc == 0
            cap_in = np.fromfile("cap_in.bin", dtype=np.int32).reshape(-1, 64)
            cap_out = np.fromfile("cap_out.bin", dtype=np.int32).reshape(-1, 64)
            bmp = open("m:\\output.bmp", "rb").read()
        finally:
            os.chdir(cwd)
            shutil.rmtree(tmp, ignore_errors=True)
        return cap_in, cap_out, bmp

    def try_decode(self, jpg_path):
        """Decode in a forked child (the reference may abort on a file it
        rejects); returns (accepted, its stdout log).  load_jpg returns true
        whatever happened (src/parser.cpp:416-418): accepted = it wrote its BMP."""
        tmp = tempfile.mkdtemp(prefix="hjd_ref_")
        try:
            log = os.path.join(tmp, "log.txt")
            pid = os.fork()
            if pid == 0:
                try:
                    os.chdir(tmp)
                    fd = os.open(log, os.O_WRONLY | os.O_CREAT)
                    os.dup2(fd, 1)
                    self.lib.ref_load_jpg(os.path.abspath(jpg_path).encode(), None, None)
                    libc = ctypes.CDLL(None)
                    libc.fflush(None)
                finally:
                    os._exit(0)
            _, st = os.waitpid(pid, 0)
            ok = st == 0 and os.path.exists(os.path.join(tmp, "m:\\output.bmp"))
            return ok, open(log, errors="replace").read()
        finally:
            shutil.rmtree(tmp, ignore_errors=True)

    def fast_idct(self, blocks):
        b = np.ascontiguousarray(blocks, dtype=np.int32).copy()
        self.lib.ref_fast_idct_n(b.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), b.shape[0])
        return b

    def csc(self, y, u, v):
        out = np.empty(y.shape, dtype=np.uint32)
        p = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
        self.lib.ref_yuv_to_rgb32_n(p(y), p(u), p(v), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), y.size)
        return out


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def synthetic_rgb(w, h, seed, sigma=20.0):
    """gradient + iid gaussian noise, clipped."""
    rng = np.random.default_rng(seed)
    x = np.arange(w)[None, :].astype(np.float64)
    y = np.arange(h)[:, None].astype(np.float64)
    r = x * 255.0 / w + 0 * y
    g = y * 255.0 / h + 0 * x
    b = (x + y) * 255.0 / (w + h)
    img = np.stack([r, g, b], axis=-1) + rng.normal(0, sigma, (h, w, 3))
    return np.clip(np.rint(img), 0, 255).astype(np.uint8)


def encode_jpeg(rgb, quality, subsampling, **kw) -> bytes:
    from PIL import Image
    buf = io.BytesIO()
    Image.fromarray(rgb, "RGB").save(buf, format="JPEG", quality=quality, subsampling=subsampling, **kw)
    return buf.getvalue()


CASES = [
    # name, (w, h), quality, subsampling (PIL: 0 = 4:4:4, 2 = 4:2:0), extra save kwargs
    ("syn420_96x64_q90", (96, 64), 90, 2, {}),
    ("syn420_odd_37x29_q90", (37, 29), 90, 2, {}),
    ("syn444_64x40_q90", (64, 40), 90, 0, {}),
    ("syn444_odd_41x23_q75", (41, 23), 75, 0, {}),
    ("syn444_48x32_q100", (48, 32), 100, 0, {}),
    ("syn420_160x48_q95_dri", (160, 48), 95, 2, {"restart_marker_blocks": 7}),
    ("syn420_80x80_q50_opt", (80, 80), 50, 2, {"optimize": True}),
    ("syn420_272x32_q90_wide", (272, 32), 90, 2, {}),
    ("syn444_264x16_q90_wide", (264, 16), 90, 0, {}),
]


def golden_case(ref: Ref, name: str, jpg_bytes: bytes, meta: dict):
    jpg_path = os.path.join(HERE, name + ".jpg")
    with open(jpg_path, "wb") as f:
        f.write(jpg_bytes)
    (w, h), comps, qts = parse_headers(jpg_bytes)
    sampling = sampling_of(comps)
    cap_in, cap_out, bmp = ref.decode(jpg_path)
    bpm = 6 if sampling == 1 else 3
    msz = 16 if sampling == 1 else 8
    nblk = ((w - 1) // msz + 1) * ((h - 1) // msz + 1) * bpm
    assert cap_in.shape[0] == nblk, (cap_in.shape, nblk)
    qt = np.stack([qts[c[2]] for c in comps]).astype(np.int32)  # [3][64], file order
    comp_of_blk = np.array(([0] * (bpm - 2) + [1, 2]) * (nblk // bpm))
    nat = cap_in[:, ZIGZAG]  # zigzag order
    q = qt[comp_of_blk]
    assert (nat % q == 0).all(), "mcu_data not divisible by qtable"
    coefs = (nat // q).astype(np.int64)
    assert (np.abs(coefs) < 32768).all()
    coefs = coefs.astype(np.int16)
    px = np.frombuffer(bmp[54:], dtype=np.uint32)
    bgrx = px[: w * h].reshape(h, w).copy()
    np.savez_compressed(os.path.join(HERE, name + ".npz"), coefs_q16=coefs, qt=qt,
                        width=np.int32(w), height=np.int32(h), sampling=np.int32(sampling), bgrx=bgrx)
    rec = dict(meta, width=w, height=h, sampling=sampling, blocks=int(nblk),
               jpeg_sha256=hashlib.sha256(jpg_bytes).hexdigest(),
               mcu_data_sha256=sha(cap_in), idct_sha256=sha(cap_out),
               bgrx_sha256=sha(bgrx), bmp_sha256=hashlib.sha256(bmp).hexdigest(), bmp_bytes=len(bmp))
    print(f"{name}: {w}x{h} samp={sampling} blocks={nblk} bgrx={rec['bgrx_sha256'][:12]}")
    return rec


def fdct_blocks(pix):
    """float forward DCT of [n][8][8] level-shifted samples (JPEG Annex A)."""
    k = np.arange(8)
    c = np.where(k == 0, 1 / np.sqrt(2), 1.0)
    m = np.cos((2 * k[None, :] + 1) * k[:, None] * np.pi / 16) * c[:, None] / 2  # [u][x]
    return np.einsum("ux,nxy,vy->nuv", m, pix, m)


def idct_vectors(ref: Ref):
    rng = np.random.default_rng(1234)
    blocks = []
    # known answers: DC-only and the [-256,255] clamp edge
    for dc in (2100, -2100, 2016, 0, 1, -1, 7, -8, 1023, -1024, 4088, -4096):
        b = np.zeros(64, np.int32); b[0] = dc; blocks.append(b)
    b = np.zeros(64, np.int32); b[0], b[1], b[8] = 1000, -900, 700; blocks.append(b)
    # forward DCT + quantisation of bounded pixels: the reference's legal domain
    n = 500
    kinds = rng.integers(0, 4, n)
    pix = rng.integers(-128, 128, (n, 8, 8)).astype(np.float64)
    pix[kinds == 1] = np.where((np.indices((8, 8)).sum(0) % 2) == 0, 127, -128)[None]   # checkerboard
    pix[kinds == 2] = np.clip(pix[kinds == 2].cumsum(axis=2) / 4, -128, 127)            # smooth-ish
    pix[kinds == 3] = rng.choice([-128, 127], (int((kinds == 3).sum()), 8, 8))         # extremes
    F = fdct_blocks(pix).reshape(n, 64)
    q = rng.integers(1, 64, (n, 64))
    q[rng.random(n) < 0.3] = 1
    coef = np.rint(F / q) * q
    blocks.extend(coef.astype(np.int32))
    inp = np.stack(blocks).astype(np.int32)
    out = ref.fast_idct(inp)
    np.savez_compressed(os.path.join(HERE, "idct_vectors.npz"), inp=inp, out=out)
    print(f"idct vectors: {inp.shape[0]} blocks, max|in|={np.abs(inp).max()} out range [{out.min()},{out.max()}]")
    return {"idct_vectors": int(inp.shape[0]), "idct_vectors_out_sha256": sha(out)}


def csc_exhaustive(ref: Ref):
    h = hashlib.sha256()
    u, v = np.meshgrid(np.arange(-256, 256, dtype=np.int32), np.arange(-256, 256, dtype=np.int32), indexing="ij")
    u = u.ravel().copy(); v = v.ravel().copy()
    for y in range(-256, 256):
        yy = np.full(u.shape, y, np.int32)
        h.update(ref.csc(yy, u, v).tobytes())
    # small readable sample
    rng = np.random.default_rng(7)
    ys, us, vs = (rng.integers(-256, 256, 4096).astype(np.int32) for _ in range(3))
    np.savez_compressed(os.path.join(HERE, "csc_sample.npz"), y=ys, u=us, v=vs, out=ref.csc(ys, us, vs))
    return {"csc_exhaustive_sha256": h.hexdigest(),
            "csc_order": "index = ((Y+256)<<18) | ((U+256)<<9) | (V+256), uint32 little-endian"}


def q16_of_mcu_data(cap_in, jpg_bytes):
    """The reference's mcu_data (int32 natural, dequantised) as int16 zigzag
    quantised coefficients (exact: src/decoder.cpp:340 multiplied them)."""
    (w, h), comps, qts = parse_headers(jpg_bytes)
    sampling = sampling_of(comps)
    bpm = 6 if sampling == 1 else 3
    qt = np.stack([qts[c[2]] for c in comps]).astype(np.int32)
    comp_of_blk = np.array(([0] * (bpm - 2) + [1, 2]) * (cap_in.shape[0] // bpm))
    nat = cap_in[:, ZIGZAG]
    q = qt[comp_of_blk]
    assert (nat % q == 0).all()
    return (nat // q).astype(np.int16), (w, h, sampling)


def scale_pins(ref: Ref):
    """Config-5 scale: the reference's mcu_data hashes of seeded files that are
    regenerated rather than committed (tests/scale_pins.py), and the
    restart-marker read-boundary case (src/decoder.cpp:122-146)."""
    sys.path.insert(0, os.path.dirname(HERE))
    import scale_pins as SP
    out = {}
    tmp = tempfile.mkdtemp(prefix="hjd_scale_")
    try:
        for name, (kind, params) in SP.SCALE_CASES.items():
            files = []
            for k, jpg in enumerate(SP.generate(name)):
                path = os.path.join(tmp, "f.jpg")
                with open(path, "wb") as f:
                    f.write(jpg)
                cap_in, _, _ = ref.decode(path)
                q16, (w, h, sampling) = q16_of_mcu_data(cap_in, jpg)
                files.append({"jpeg_sha256": SP.sha(jpg), "jpeg_bytes": len(jpg), "blocks": int(cap_in.shape[0]),
                              "mcu_data_sha256": SP.sha(np.ascontiguousarray(cap_in, dtype="<i4")),
                              "coefs_q16_sha256": SP.sha(np.ascontiguousarray(q16, dtype="<i2"))})
            out[name] = {"generator": kind, "params": params, "width": w, "height": h, "sampling": sampling,
                         "files": files}
            print(f"scale {name}: {len(files)} file(s) {w}x{h} samp={sampling}")
        # DRI read boundary: FHD q50 bases (seed 501, 601, ...) until the
        # reference loses an RST marker on the DRI re-encode
        for seed in [501] + list(range(601, 640)):
            base = SP.encode_jpeg(SP.synthetic_rgb(1920, 1080, seed), 50, 2)
            path = os.path.join(tmp, "base.jpg")
            with open(path, "wb") as f:
                f.write(base)
            cap_in, _, _ = ref.decode(path)
            q16, _ = q16_of_mcu_data(cap_in, base)
            dri = SP.dri_file(base, q16)
            with open(path, "wb") as f:
                f.write(dri)
            ok, log = ref.try_decode(path)
            line = next((ln for ln in log.splitlines() if "expected RST" in ln), "")
            print(f"dri seed {seed}: reference {'accepts' if ok else 'rejects'} {line.strip()[:80]}")
            if not ok and line:
                out["dri_read_boundary"] = {
                    "base": {"generator": "synthetic", "w": 1920, "h": 1080, "quality": 50, "subsampling": 2,
                             "seed": seed},
                    "restart_interval": SP.DRI_INTERVAL, "base_jpeg_sha256": SP.sha(base),
                    "jpeg_sha256": SP.sha(dri), "jpeg_bytes": len(dri),
                    "mcu_data_sha256": SP.sha(np.ascontiguousarray(cap_in, dtype="<i4")),
                    "coefs_q16_sha256": SP.sha(np.ascontiguousarray(q16, dtype="<i2")),
                    "reference_log": line.strip()}
                break
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    return out


def main():
    if "--scale-only" in sys.argv:   # refresh manifest["scale"] only
        ref = Ref()
        path = os.path.join(HERE, "manifest.json")
        manifest = json.load(open(path))
        manifest["scale"] = scale_pins(ref)
        with open(path, "w") as f:
            json.dump(manifest, f, indent=1, sort_keys=True)
        print("wrote", path)
        return
    if not os.path.exists(REF_LIB):
        sys.exit("build the reference first: make -C oracle")
    ref = Ref()
    manifest = {"generator": "tests/golden/make_golden.py", "reference_lib": "oracle/_ref/libref.so",
                "cases": {}}
    sample = open(REF_SAMPLE, "rb").read()
    manifest["cases"]["JPEG_example_JPG_RIP_050"] = golden_case(
        ref, "JPEG_example_JPG_RIP_050", sample, {"source": "reference test/JPEG_example_JPG_RIP_050.jpg"})
    for i, (name, (w, h), qual, sub, kw) in enumerate(CASES):
        jpg = encode_jpeg(synthetic_rgb(w, h, seed=100 + i), qual, sub, **kw)
        manifest["cases"][name] = golden_case(ref, name, jpg, {"source": f"Pillow q={qual} subsampling={sub} {kw}"})
    manifest.update(idct_vectors(ref))
    manifest.update(csc_exhaustive(ref))
    manifest["scale"] = scale_pins(ref)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", os.path.join(HERE, "manifest.json"))


if __name__ == "__main__":
    main()
