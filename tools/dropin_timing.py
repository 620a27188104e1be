#!/usr/bin/env python3
"""Time the reference program end to end on the GPU box, both builds, same files:

  oracle/_ref/ref_cpu     the reference's USE_CPU_ONLY build (its own CPU IDCT + colour)
  oracle/_ref/ref_dropin  the reference's GPU build linked to libhjd.so (idct.h shim)

Files: synthetic 4K 4:2:0 and 4:4:4 JPEGs (Pillow q90, gradient + sigma-20 noise, the
SURVEY s8(d) frame) plus FHD 4:2:0.  The drop-in decodes every file several times in
ONE process (the reference's main.cpp takes many files), so the first image pays the
context/stream/allocation cost and the rest show the steady state of the persistent
lifecycle (idct_compat.hip).  Copy modes (HJD_COMPAT_COPY) and the reference's
per-image teardown (HJD_COMPAT_TEARDOWN=1) are timed too.

Per stage: the reference's own clock() prints (src/parser.cpp:373-397,
src/decoder.cpp:357-416; CPU microseconds), the shim's wall-clock stage times
([hjd-compat] lines), and the wall time of each process.

    python tools/dropin_timing.py OUT.json
"""
import io
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(REPO, "oracle", "_ref")


def make_jpeg(w, h, sub, seed):
    from PIL import Image
    rng = np.random.default_rng(seed)
    x = np.arange(w, dtype=np.float32)[None, :]
    y = np.arange(h, dtype=np.float32)[:, None]
    img = np.stack([x * 255 / w + 0 * y, y * 255 / h + 0 * x, (x + y) * 255 / (w + h)], axis=-1)
    img = np.clip(img + rng.normal(0, 20, (h, w, 3)).astype(np.float32), 0, 255).astype(np.uint8)
    b = io.BytesIO()
    Image.fromarray(img).save(b, format="JPEG", quality=90, subsampling=sub)
    return b.getvalue()


CLOCK_KEYS = {
    "parse_us": r"Time elapsed for parsing basic info: (\d+)",
    "init_us": r"Time elapsed for initialization: (\d+)",
    "huffman_us": r"Time elapsed for huffman decoding: (\d+)",
    "idct_colour_us": r"Time elapsed for IDCT and color space conversion: (\d+)",
    "h2d_us": r"Time elapsed for writing data to device: (\d+)",
    "kernel_us": r"Time elapsed for running the IDCT kernel: (\d+)",
    "d2h_us": r"Time elapsed for reading data from device: (\d+)",
}


def run(prog, files, cwd, env=None):
    t0 = time.perf_counter()
    r = subprocess.run([prog, *files], cwd=cwd, capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, **(env or {})))
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"{prog} rc={r.returncode}: {r.stdout[-1500:]} {r.stderr[-1500:]}")
    # split the reference's stdout per image ("Processing <file>", src/main.cpp:33)
    per = []
    for chunk in r.stdout.split("Processing ")[1:]:
        d = {}
        for k, pat in CLOCK_KEYS.items():
            m = re.search(pat, chunk)
            if m:
                d[k] = int(m.group(1))
        per.append(d)
    shim = [dict(kv.split("=", 1) for kv in l.split()[1:]) for l in r.stderr.splitlines()
            if l.startswith("[hjd-compat]")]
    for d, s in zip(per, shim):
        d["shim"] = s
    return {"wall_s": round(wall, 3), "images": per}


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else "dropin_timing.json"
    tmp = tempfile.mkdtemp(prefix="hjd_dropin_timing_")
    res = {"cpu": open("/proc/cpuinfo").read().split("model name")[1].split("\n")[0].strip(": "),
           "note": "clock() values are the reference's own prints (process CPU microseconds); [hjd-compat] "
                   "stage times are wall clock inside the shim", "runs": {}}
    try:
        files = {}
        for name, (w, h, sub) in {"4k420": (3840, 2160, 2), "4k444": (3840, 2160, 0),
                                  "fhd420": (1920, 1080, 2)}.items():
            p = os.path.join(tmp, name + ".jpg")
            with open(p, "wb") as f:
                f.write(make_jpeg(w, h, sub, seed=len(name)))
            files[name] = p
        reps = 4
        for name, p in files.items():
            res["runs"][f"ref_cpu/{name}"] = run(os.path.join(REF, "ref_cpu"), [p] * 2, tmp)
            for mode in ("staged", "pageable", "register"):
                res["runs"][f"ref_dropin/{name}/{mode}"] = run(
                    os.path.join(REF, "ref_dropin"), [p] * reps, tmp,
                    {"HJD_COMPAT_STATS": "1", "HJD_COMPAT_COPY": mode})
            res["runs"][f"ref_dropin/{name}/staged_teardown"] = run(
                os.path.join(REF, "ref_dropin"), [p] * reps, tmp,
                {"HJD_COMPAT_STATS": "1", "HJD_COMPAT_TEARDOWN": "1"})
            print(name, "done", flush=True)
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    with open(out_path, "w") as f:
        json.dump(res, f, indent=1)
    # compact table: steady-state image (the last one) of each run
    for k, v in res["runs"].items():
        last = v["images"][-1]
        s = last.get("shim", {})
        print(f"{k:34s} wall {v['wall_s']:7.3f}s  huff {last.get('huffman_us', 0) / 1e3:7.1f}ms  "
              f"idct+colour(stage) {last.get('idct_colour_us', 0) / 1e3:7.1f}ms  "
              f"h2d {s.get('h2d_ms', '-'):>8} kern {s.get('kernel_ms', '-'):>7} d2h {s.get('d2h_ms', '-'):>8} "
              f"allocs {s.get('allocs', '-')}")


if __name__ == "__main__":
    main()
