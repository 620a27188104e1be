"""GPU: examples/jpeg2bmp -- a plain C program (gcc, no Python, no torch) using
only the C ABI (include/hjd.h, include/hjd_host.h) and the HIP runtime for
device buffers -- turns JPEG files into the reference program's 32-bpp BMP
files.  Pixels must equal the reference's BGRX on its golden sample, and the
oracle's pixels on the host-decoded coefficients of the other files (GPU
Huffman path for sequential files with one scan or several, and the
host-Huffman + plan path for a progressive file)."""
import io
import os
import subprocess
import tempfile

import numpy as np
import pytest

import jpeg_writer as JW
import oracle_py as O

pytestmark = pytest.mark.gpu
EXE = os.path.join(O.REPO, "examples", "jpeg2bmp")


def _bmp_pixels(path, w, h):
    data = open(path, "rb").read()
    assert len(data) == 54 + 4 * w * h
    return np.frombuffer(data[54:], dtype="<u4").reshape(h, w)


def test_c_program_decodes_to_bmp(hjd):
    from PIL import Image
    assert os.access(EXE, os.X_OK), "examples/jpeg2bmp not built (run __graft_entry__.build())"
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, (77, 133, 3), dtype=np.uint8)
    files = {"golden.jpg": open(os.path.join(O.GOLDEN, "JPEG_example_JPG_RIP_050.jpg"), "rb").read()}
    for name, kw in (("q85_444.jpg", dict(quality=85, subsampling=0)),
                     ("prog_420.jpg", dict(quality=80, subsampling=2, progressive=True))):
        b = io.BytesIO()
        Image.fromarray(img).save(b, format="JPEG", **kw)
        files[name] = b.getvalue()
    base = files["q85_444.jpg"]
    files["3scan_444.jpg"] = JW.rewrite_scans(base, hjd.decode_coefs(base)[0], [(2,), (0,), (1,)], 4)[0]
    with tempfile.TemporaryDirectory() as d:
        paths = []
        for name, data in files.items():
            open(os.path.join(d, name), "wb").write(data)
            paths.append(os.path.join(d, name))
        p = subprocess.run([EXE, d] + paths, capture_output=True, text=True, timeout=100)
        assert p.returncode == 0, p.stdout + p.stderr
        for name, data in files.items():
            coefs, info = hjd.decode_coefs(data)
            got = _bmp_pixels(os.path.join(d, name + ".bmp"), info.width, info.height)
            if name == "golden.jpg":
                np.testing.assert_array_equal(got, O.load_case("JPEG_example_JPG_RIP_050")["bgrx"])
            else:
                np.testing.assert_array_equal(got, O.decode_q16(coefs, np.array(info.qt), info.width, info.height,
                                                                info.sampling))
        assert "process 2" in p.stdout
        lines = {ln.split(":")[0].rsplit("/", 1)[-1]: ln for ln in p.stdout.splitlines()}
        assert "scans several" in lines["3scan_444.jpg"] and "(GPU Huffman)" in lines["3scan_444.jpg"]
        assert "(host Huffman)" in lines["prog_420.jpg"]
