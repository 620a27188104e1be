#!/usr/bin/env python3
"""Launch-bound pixel launches: eager back-to-back launches vs a HIP graph
(torch.cuda.CUDAGraph stream capture of the same hjd_plan_launch calls).

    python tools/graph_probe.py [--workload fhd420] [--launches 200] [--reps 5]

Prints one JSON object: per-launch microseconds (HIP events on the launch
stream) for eager launches and for graph replays, the single-launch
launch+synchronize wall time of each, and whether the graph's output equals
the eager output.  Tuning tool (configs[1] is launch-latency bound: SURVEY.md
s8(d) config 2)."""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="fhd420")
    ap.add_argument("--launches", type=int, default=200)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()

    import torch
    import bench
    import ocljpegdecoder_amd as hjd

    wl = dict(bench.WORKLOADS[args.workload])
    w, h, s, nf = wl["width"], wl["height"], wl["sampling"], wl["frames"]
    mw, mh, bpm, _ = hjd.mcu_geometry(w, h, s)
    nblk = mw * mh * bpm
    qt = bench.std_qtables(1.0)
    dev = torch.device("cuda", 0)
    coefs = torch.empty((nf, nblk, 64), dtype=torch.int16, device=dev)
    for i in range(nf):
        coefs[i] = bench.synth_frame_gpu(torch, nblk, s, qt, seed=i, device=dev)
    out_e = torch.zeros((nf, h, w), dtype=torch.int32, device=dev)
    out_g = torch.zeros_like(out_e)
    ctx = hjd.Context(0)
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
             for i in range(nf)]
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
    K = args.launches

    stream = torch.cuda.current_stream()
    for _ in range(10):
        plan.launch(coefs, out_e, stream)
    torch.cuda.synchronize()

    def timed(fn):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) * 1e3 / K   # us per launch

    def eager():
        for _ in range(K):
            plan.launch(coefs, out_e, stream)

    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(stream)
    with torch.cuda.stream(side):
        plan.launch(coefs, out_g, side)   # warm on the capture stream
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        cs = torch.cuda.current_stream()
        for _ in range(K):
            plan.launch(coefs, out_g, cs)
    g1 = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g1):
        plan.launch(coefs, out_g, torch.cuda.current_stream())
    torch.cuda.synchronize()

    res = {"workload": args.workload, "frames": nf, "launches": K, "eager_us": [], "graph_us": [],
           "eager_single_wall_us": [], "graph_single_wall_us": []}
    for _ in range(args.reps):
        res["eager_us"].append(round(timed(eager), 3))
        res["graph_us"].append(round(timed(g.replay), 3))
        for key, fn in (("eager_single_wall_us", lambda: plan.launch(coefs, out_e, stream)),
                        ("graph_single_wall_us", g1.replay)):
            ts = []
            for _ in range(50):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append((time.perf_counter() - t0) * 1e6)
            res[key].append(round(statistics.median(ts), 2))
    res["outputs_equal"] = bool(torch.equal(out_e, out_g))
    res["px_per_launch"] = plan.pixels
    for k in ("eager_us", "graph_us"):
        res[k.replace("_us", "_Mpx_s_best")] = round(plan.pixels / min(res[k]), 1)
    plan.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
