"""Seed files for tools/fuzz/run.sh: baseline, progressive (with and without
restarts) and multi-scan sequential JPEGs of a small noisy image."""
import io
import sys

import numpy as np
from PIL import Image

import jpeg_writer as JW
import ocljpegdecoder_amd as hjd

out = sys.argv[1]
rng = np.random.default_rng(3)
img = Image.fromarray(rng.integers(0, 256, (40, 56, 3), dtype=np.uint8))
files = {}
for sub in (0, 1, 2):
    for prog in (False, True):
        for kw in ({}, {"restart_marker_blocks": 2}):
            b = io.BytesIO()
            img.save(b, format="JPEG", quality=80, subsampling=sub, progressive=prog, **kw)
            files[f"s{sub}_p{int(prog)}_r{len(kw)}"] = b.getvalue()
b = io.BytesIO()
img.convert("L").save(b, format="JPEG", quality=80, progressive=True)
files["gray_p1"] = b.getvalue()
base = files["s2_p0_r0"]
coefs, _ = hjd.decode_coefs(base)
files["ms_3scan_dri"] = JW.rewrite_scans(base, coefs, [(0,), (2,), (1,)], 3)[0]
files["ms_y_cbcr"] = JW.rewrite_scans(base, coefs, [(0,), (1, 2)])[0]
for k, v in files.items():
    open(f"{out}/{k}.jpg", "wb").write(v)
print(len(files), "seed files")
