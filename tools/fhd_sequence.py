"""One latency decoder over a sequence of the same JPEG (a camera stream of
alike frames): wall time of every decode + sync, so that the cost of the
lead-in ladder's step-downs (a repaired frame now and then) shows in the mean,
not only the median.

    python tools/fhd_sequence.py --pil 1920x1080x90x0x5 --n 400 [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pil", required=True, help="WxHxQxSUBxSEED (tests/test_entropy_emulation._pil)")
    ap.add_argument("--n", type=int, default=400)
    ap.add_argument("--json")
    a = ap.parse_args()
    import torch
    import ocljpegdecoder_amd as hjd
    from test_entropy_emulation import _pil
    w, h, q, sub, seed = (int(x) for x in a.pil.split("x"))
    data = _pil(w, h, q, sub, seed=seed)
    info = hjd.parse(data)
    ctx = hjd.Context(0)
    out = torch.empty((info.height, info.width), dtype=torch.int32, device="cuda")
    ms, bits = [], []
    with hjd.GpuDecoder(ctx, 1, len(data), info.nblocks) as gd:
        for _ in range(a.n):
            t0 = time.perf_counter()
            gd.decode([data], [out])
            st = gd.sync()[0]
            ms.append((time.perf_counter() - t0) * 1e3)
            bits.append(st & 1)
    ms = np.array(ms[1:])   # (the first call carries one-time setup)
    res = {"image": a.pil, "n": a.n - 1, "lib": os.environ.get("HJD_LIB", "product"),
           "mean_ms": round(float(ms.mean()), 4), "median_ms": round(float(np.median(ms)), 4),
           "p99_ms": round(float(np.percentile(ms, 99)), 4), "repaired_calls": int(sum(bits[1:])),
           "repaired_at": [i + 1 for i, b in enumerate(bits[1:]) if b][:40]}
    print(json.dumps(res))
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
