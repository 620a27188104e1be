#!/usr/bin/env python3
"""Memory-side time of the pixel kernel against where its buffers sit (round 4).

    python tools/offset_sweep.py [--workload 4k420] [--frames 1024] [--step-mib 2] [--points 32]

One arena is allocated once; the coefficient and output buffers are carved
out of it at chosen byte offsets, so the physical pages stay the same and only
the buffers' placement inside them changes.  Sweep A moves the coefficient
buffer in --step-mib steps with the output fixed; sweep B moves the output.
Each point times the memory-only variant (stages 80) and the product with HIP
events.  Prints one JSON object.
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="4k420")
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--step-mib", type=float, default=2.0)
    ap.add_argument("--points", type=int, default=32)
    ap.add_argument("--reps", type=int, default=3)
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
    cbytes = nf * nblk * 64 * 2
    obytes = nf * h * w * 4
    step = int(args.step_mib * (1 << 20)) // 256 * 256
    span = step * args.points
    arena = torch.empty(cbytes + obytes + 2 * span + (1 << 21), dtype=torch.uint8, device=dev)
    base = (-arena.data_ptr()) % (1 << 21)   # start at a 2 MiB boundary of the arena
    pool = torch.empty((8, nblk, 64), dtype=torch.int16, device=dev)
    for i in range(8):
        pool[i] = bench.synth_frame_gpu(torch, nblk, s, qt, seed=i, device=dev)
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
             for i in range(nf)]
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)

    def views(coff, ooff):
        c = arena[base + coff: base + coff + cbytes].view(torch.int16).view(nf, nblk, 64)
        o = arena[base + span + cbytes + ooff: base + span + cbytes + ooff + obytes].view(torch.int32).view(nf, h, w)
        return c, o

    def measure(c, o):
        for i in range(nf):
            c[i].copy_(pool[i % 8])
        r = {}
        for st in (80, 0):
            def go():
                if st:
                    plan.launch_stages(st, c, o, stream)
                else:
                    plan.launch(c, o, stream)
            go()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(args.reps):
                go()
            e1.record(stream)
            torch.cuda.synchronize()
            r["memory_only_ms" if st else "product_ms"] = round(e0.elapsed_time(e1) / args.reps, 4)
        return r

    sweeps = {"coefs_moved": [], "out_moved": []}
    for k in range(args.points):
        c, o = views(k * step, 0)
        sweeps["coefs_moved"].append({"offset_mib": round(k * step / (1 << 20), 3), **measure(c, o)})
    for k in range(args.points):
        c, o = views(0, k * step)
        sweeps["out_moved"].append({"offset_mib": round(k * step / (1 << 20), 3), **measure(c, o)})
    summ = {}
    for name, rows in sweeps.items():
        m = [r["memory_only_ms"] for r in rows]
        p = [r["product_ms"] for r in rows]
        summ[name] = {"memory_only_ms": [min(m), max(m)], "product_ms": [min(p), max(p)],
                      "memory_only_spread_pct": round((max(m) / min(m) - 1) * 100, 2),
                      "product_spread_pct": round((max(p) / min(p) - 1) * 100, 2)}
    print(json.dumps({"workload": args.workload, "frames": nf, "step_mib": args.step_mib, "points": args.points,
                      "arena_addr": hex(arena.data_ptr() + base), "box": bench.box_identity(torch),
                      "summary": summ, "sweeps": sweeps}))


if __name__ == "__main__":
    main()
