#!/usr/bin/env python3
"""Per-launch time of the persistent and the latency kernel vs launch size
(tuning for HJD_KERNEL_AUTO's task threshold; run on the GPU box).

    python tools/latency_sweep.py > gpurun_out/lat.json

For each (geometry, frames): HIP-event time of K back-to-back launches of one
plan with each kernel mode; one JSON line per case.
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch
    import bench
    import ocljpegdecoder_amd as hjd

    dev = torch.device("cuda", 0)
    ctx = hjd.Context(0)
    qt = bench.std_qtables(1.0)
    cases = [(1920, 1080, 1, 1), (1920, 1080, 0, 1), (1920, 1080, 1, 2), (3840, 2160, 1, 1), (3840, 2160, 0, 1),
             (3840, 2160, 1, 2), (3840, 2160, 1, 4), (1280, 720, 1, 1), (640, 480, 1, 1)]
    for w, h, s, nf in cases:
        mw, mh, bpm, _ = hjd.mcu_geometry(w, h, s)
        nblk = mw * mh * bpm
        coefs = torch.empty((nf, nblk, 64), dtype=torch.int16, device=dev)
        for i in range(nf):
            coefs[i] = bench.synth_frame_gpu(torch, nblk, s, qt, seed=i, device=dev)
        out = torch.empty((nf, h, w), dtype=torch.int32, device=dev)
        specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
                 for i in range(nf)]
        plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
        res = {"w": w, "h": h, "sampling": s, "frames": nf, "tasks": plan.tasks}
        ref = None
        for name, mode in (("persistent", hjd.KERNEL_PERSISTENT), ("latency", hjd.KERNEL_LATENCY)):
            plan.set_kernel(mode)
            for _ in range(20):
                plan.launch(coefs, out)
            torch.cuda.synchronize()
            k = 400
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(k):
                plan.launch(coefs, out)
            e1.record()
            torch.cuda.synchronize()
            res[name + "_us"] = round(e0.elapsed_time(e1) / k * 1e3, 2)
            if ref is None:
                ref = out.clone()
            else:
                res["identical"] = bool(torch.equal(ref, out))
        res["mpx_s_best"] = round(nf * w * h / min(res["persistent_us"], res["latency_us"]), 1)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
