#!/usr/bin/env python3
"""Does the 4:2:0 slowdown follow the buffers rather than the box?  (round 4)

    python tools/alloc_var.py [--workload 4k420] [--frames 1024] [--allocs 5] [--reps 5]

In one process, allocates the bench's coefficient and output buffers afresh
`--allocs` times (freeing the previous ones and emptying torch's cache in
between; each allocation after the first shifted by a different pad buffer so
it lands elsewhere), and times the product kernel and its memory-only variant
(stages 80) on each allocation with HIP events.  Prints one JSON object: per
allocation the buffers' device addresses and the times.  If the times differ
between allocations of one process as much as between processes, the slow
state belongs to where the buffers landed, not to the box.
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
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--allocs", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
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
    ctx = hjd.Context(0)
    stream = torch.cuda.current_stream()
    pool = torch.empty((8, nblk, 64), dtype=torch.int16, device=dev)
    for i in range(8):
        pool[i] = bench.synth_frame_gpu(torch, nblk, s, qt, seed=i, device=dev)
    nbytes = None
    rows = []
    for a in range(args.allocs):
        pad = torch.empty((a * 3 + 1) << 28, dtype=torch.uint8, device=dev) if a else None   # 256 MiB steps
        coefs = torch.empty((nf, nblk, 64), dtype=torch.int16, device=dev)
        for i in range(nf):
            coefs[i].copy_(pool[i % 8])
        out = torch.empty((nf, h, w), dtype=torch.int32, device=dev)
        specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
                 for i in range(nf)]
        plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
        nbytes = plan.coef_bytes + 4 * plan.pixels
        res = {"alloc": a, "coefs_addr": hex(coefs.data_ptr()), "out_addr": hex(out.data_ptr()),
               "pad_bytes": 0 if pad is None else pad.numel()}
        for st in (0, 80, 0, 80):
            def go():
                if st:
                    plan.launch_stages(st, coefs, out, stream)
                else:
                    plan.launch(coefs, out, stream)
            go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                go()
            e1.record(stream)
            torch.cuda.synchronize()
            res.setdefault("product_ms" if st == 0 else "memory_only_ms", []).append(
                round(e0.elapsed_time(e1) / args.reps, 4))
        rows.append(res)
        plan.close()
        del coefs, out, plan, pad
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
    prod = [min(r["product_ms"]) for r in rows]
    mem = [min(r["memory_only_ms"]) for r in rows]
    print(json.dumps({"workload": args.workload, "frames": nf, "bytes_per_launch": nbytes,
                      "box": bench.box_identity(torch), "allocations": rows,
                      "product_ms_range": [min(prod), max(prod)], "memory_only_ms_range": [min(mem), max(mem)],
                      "product_spread_pct": round((max(prod) / min(prod) - 1) * 100, 2),
                      "memory_only_spread_pct": round((max(mem) / min(mem) - 1) * 100, 2),
                      "frac_range": [round(nbytes / (max(prod) / 1e3) / 8e12, 4),
                                     round(nbytes / (min(prod) / 1e3) / 8e12, 4)]}))


if __name__ == "__main__":
    main()
