"""Host time per phase of one-image GPU decodes (HJD_GDEC_HOST_TIMES): the
FHD q90 JPEG of bench.py's fhd420_jpeg workload, decoded --n times from
pageable bytes (host destuff) and then from pinned bytes, for each library in
--libs (product or build/variants/<name>), each in a child process.

    python tools/fhd_host_times.py [--libs product+skew1024] [--n 300]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, time
sys.path.insert(0, REPO); sys.path.insert(0, REPO + "/tests")
import torch, bench, ocljpegdecoder_amd as hjd
data = bench.encode_pool(1920, 1080, 1, 1, seed0=4242)[0]
info = hjd.parse(data)
ctx = hjd.Context(0)
out = torch.empty((1080, 1920), dtype=torch.int32, device="cuda")
for label, src in (("pageable", data), ("pinned", hjd.pinned_bytes(data))):
    gd = hjd.GpuDecoder(ctx, 1, len(data), info.nblocks)
    for _ in range(20):
        gd.decode([src], [out]); gd.sync()
    gd.close()
    gd = hjd.GpuDecoder(ctx, 1, len(data), info.nblocks)
    t = time.perf_counter()
    for _ in range(N):
        gd.decode([src], [out]); gd.sync()
    dt = (time.perf_counter() - t) / N
    print(label, "ms/image", round(dt * 1e3, 4), file=sys.stderr, flush=True)
    gd.close()
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--libs", default="product")
    ap.add_argument("--n", type=int, default=300)
    a = ap.parse_args()
    res = []
    for lib in a.libs.split("+"):
        env = dict(os.environ, HJD_GDEC_HOST_TIMES="1")
        env.pop("HJD_LIB", None)
        if lib != "product":
            env["HJD_LIB"] = os.path.join(REPO, "build", "variants", lib, "libhjd.so")
        code = f"REPO = {REPO!r}\nN = {a.n}\n" + CHILD
        p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
        if p.returncode:
            raise SystemExit(f"{lib}: {p.stderr[-2000:]}")
        res.append({"lib": lib, "lines": [ln for ln in p.stderr.splitlines() if "hjd_gdec host" in ln or "ms/image" in ln]})
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
