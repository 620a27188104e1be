"""Single-image GPU-decode latency of the FHD q90 JPEG (bench.py's
fhd420_jpeg input) under tuning environments, each config in a child process
with the product library: ms per image from pageable bytes and from pinned
bytes (N decodes each, after 20 warm-up), and whether the pixels equal the
pixels of the host Huffman decode + the same fused kernel.

    python tools/fhd_env_sweep.py --configs "HJD_SUB_BITS=384+HJD_SPEC_LEAD=512;HJD_SUB_BITS=512" [--n 300] [--rounds 2]
        [--pil 1920x1080x95x2x3]

(';' separates configs, '+' the variables of one config; an empty config is
the default.)
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
import numpy as np, torch, bench, ocljpegdecoder_amd as hjd
if PIL_SPEC:
    from test_entropy_emulation import _pil
    w_, h_, q_, sub_, seed_ = PIL_SPEC
    data = _pil(w_, h_, q_, sub_, seed=seed_)
else:
    data = bench.encode_pool(1920, 1080, 1, 1, seed0=4242)[0]
info = hjd.parse(data)
ctx = hjd.Context(0)
out = torch.empty((info.height, info.width), dtype=torch.int32, device="cuda")
# reference pixels: host Huffman decode, the same fused kernel
coefs, _ = hjd.decode_coefs(data)
plan = hjd.Plan(ctx, [hjd.FrameSpec(info.width, info.height, info.sampling, qt_index=(0, 1, 2))], hjd.IN_Q16_ZIGZAG,
                qtables=info.qt)
ref = torch.empty_like(out)
plan.launch(torch.from_numpy(coefs).cuda(), ref)
torch.cuda.synchronize()
res = {}
for label, src in (("pageable", data), ("pinned", hjd.pinned_bytes(data))):
    gd = hjd.GpuDecoder(ctx, 1, len(data), info.nblocks)
    for _ in range(20):
        gd.decode([src], [out]); gd.sync()
    ok = bool(torch.equal(out, ref))
    t = time.perf_counter()
    for _ in range(N):
        gd.decode([src], [out]); gd.sync()
    res[label] = round((time.perf_counter() - t) / N * 1e3, 4)
    res[label + "_ok"] = ok
    gd.close()
print("RESULT", res)
'''


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="")
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--pil", default="", help="W,H,Q,SUB,SEED: a synthetic Pillow JPEG instead of the bench's")
    a = ap.parse_args()
    pil = tuple(int(v) for v in a.pil.replace("x", ",").split(",")) if a.pil else None
    configs = a.configs.split(";")
    rows = []
    for r in range(a.rounds):
        for cfg in (configs if r % 2 == 0 else configs[::-1]):
            env = dict(os.environ)
            for kv in filter(None, cfg.split("+")):
                k, v = kv.split("=", 1)
                env[k] = v
            code = f"REPO = {REPO!r}\nN = {a.n}\nPIL_SPEC = {pil!r}\n" + CHILD
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode:
                raise SystemExit(f"{cfg}: {p.stderr[-2000:]}")
            line = next(ln for ln in p.stdout.splitlines() if ln.startswith("RESULT"))
            rows.append({"config": cfg or "default", "round": r, **eval(line[len("RESULT "):])})
            print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    print(json.dumps({"what": "fhd420 JPEG single-image latency per tuning config (product library)",
                      "n": a.n, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
