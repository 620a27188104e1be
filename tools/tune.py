#!/usr/bin/env python3
"""Interleaved A/B of kernel variants and grid sizes in ONE process
(cdna_hip_programming.md s5.4 rule 24).

    python tools/tune.py [--workload 4k420] [--frames 256] [--rounds 5] [--variants 0,1] [--grids 0,1024,2048]

Prints, per (variant, grid), the median and min launch time and GB/s of
algorithmic bytes, as one JSON object on stdout.
"""
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="4k420")
    ap.add_argument("--frames", type=int, default=256)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="0,1")
    ap.add_argument("--grids", default="0")
    ap.add_argument("--kernels", default="1", help="hjd_kernel_mode list: 1 persistent, 2 latency")
    ap.add_argument("--no-check", action="store_true", help="ablation variants: outputs differ by design")
    ap.add_argument("--chunks", default="", help="hjd_plan_set_chunk configs (tasks per wave), e.g. s1,s2,s16; "
                                                 "replaces --grids")
    ap.add_argument("--stages", default="0", help="stage variants (hjd_debug_plan_launch_stages): 0 = the product, "
                                                  "80 memory only, 4 no stores, ... (outputs wrong by design)")
    args = ap.parse_args()

    import torch
    import bench
    import ocljpegdecoder_amd as hjd

    wl = dict(bench.WORKLOADS[args.workload])
    w, h, s, nf = wl["width"], wl["height"], wl["sampling"], args.frames
    mw, mh, bpm, _ = hjd.mcu_geometry(w, h, s)
    nblk = mw * mh * bpm
    qt = bench.std_qtables(1.0)
    dev = torch.device("cuda", 0)
    coefs = torch.empty((nf, nblk, 64), dtype=torch.int16, device=dev)
    npool = min(8, nf)
    for i in range(npool):
        coefs[i] = bench.synth_frame_gpu(torch, nblk, s, qt, seed=i, device=dev)
    for i in range(npool, nf):
        coefs[i].copy_(coefs[i % npool])
    out = torch.empty((nf, h, w), dtype=torch.int32, device=dev)
    ctx = hjd.Context(0)
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
             for i in range(nf)]
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
    nbytes = plan.coef_bytes + 4 * plan.pixels
    variants = [int(v) for v in args.variants.split(",")]
    grids = [int(g) for g in args.grids.split(",")]
    kernels = [int(k) for k in args.kernels.split(",")]
    stream = torch.cuda.current_stream()
    stages = [int(x) for x in args.stages.split(",")]
    if args.chunks:
        grids = args.chunks.split(",")
    times = {(k, v, g, st): [] for k in kernels for v in variants for g in grids for st in stages}
    ref = None
    for rnd in range(args.rounds):
        for k, v, g, st in times:
            plan.set_kernel(k)
            plan.set_variant(v)
            grid = g
            if isinstance(g, str):   # --chunks
                plan.set_chunk(int(g[1:]))
                grid = 0

            def go():
                if st:
                    plan.launch_stages(st, coefs, out, stream, grid_blocks=grid)
                else:
                    plan.launch(coefs, out, stream, grid_blocks=grid)
            go()   # warm
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                go()
            e1.record(stream)
            torch.cuda.synchronize()
            times[(k, v, g, st)].append(e0.elapsed_time(e1) / args.reps)
            if rnd == 0 and not args.no_check and not st:
                sig = int(out[:, ::97, ::89].sum().item())
                ref = sig if ref is None else ref
                assert sig == ref, f"kernel {k} variant {v} grid {g} output differs"
    res = {"workload": args.workload, "frames": nf, "bytes_per_launch": nbytes, "signature": ref,
           "box": bench.box_identity(torch), "results": []}
    for (k, v, g, st), ts in times.items():
        med = statistics.median(ts)
        res["results"].append({"kernel": k, "variant": v, "grid": g, "stages": st, "median_ms": round(med, 4),
                               "min_ms": round(min(ts), 4),
                               "GBps_median": round(nbytes / med / 1e6, 1),
                               "GBps_best": round(nbytes / min(ts) / 1e6, 1)})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
