#!/usr/bin/env python3
"""Physically contiguous buffers against default ones (round 4, placement study).

    python tools/contig_var.py [--workload 4k420] [--frames 1024] [--allocs 3] [--reps 5]

Allocates the bench's coefficient and output buffers with hipExtMallocWithFlags
-- flags 0 (default) and hipDeviceMallocContiguous (4) -- `--allocs` times
each, alternating, with a pad allocation of a different size in front each
time, and times the product kernel and its memory-only variant on each (HIP
events).  Prints one JSON object.  Question: do contiguous buffers avoid the
slow placements of tools/alloc_var.py?
"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

HIP_CONTIGUOUS = 0x4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="4k420")
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--allocs", type=int, default=3)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()

    import torch
    import bench
    import ocljpegdecoder_amd as hjd

    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]

    def alloc(nbytes, flags):
        p = ctypes.c_void_p()
        rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), flags)
        return (p.value, rc)

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
    torch.cuda.synchronize()
    fbytes = nblk * 64 * 2
    cbytes, obytes = nf * fbytes, nf * h * w * 4
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
             for i in range(nf)]
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
    rows = []
    for a in range(args.allocs):
        for flags in (0, HIP_CONTIGUOUS):
            pad, prc = alloc(((a * 3 + 1) << 28), 0)
            cp, crc = alloc(cbytes, flags)
            op, orc = alloc(obytes, flags)
            row = {"alloc": a, "flags": flags, "rc": [prc, crc, orc]}
            if crc == 0 and orc == 0:
                for i in range(nf):
                    hip.hipMemcpy(ctypes.c_void_p(cp + i * fbytes), ctypes.c_void_p(pool[i % 8].data_ptr()), fbytes, 3)
                row["coefs_addr"], row["out_addr"] = hex(cp), hex(op)
                for st in (0, 80, 0, 80):
                    def go():
                        if st:
                            plan.launch_stages(st, cp, op, stream)
                        else:
                            plan.launch(cp, op, stream)
                    go()
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record(stream)
                    for _ in range(args.reps):
                        go()
                    e1.record(stream)
                    torch.cuda.synchronize()
                    row.setdefault("product_ms" if st == 0 else "memory_only_ms", []).append(
                        round(e0.elapsed_time(e1) / args.reps, 4))
            for p in (cp, op, pad):
                if p:
                    hip.hipFree(ctypes.c_void_p(p))
            rows.append(row)
    plan.close()
    summ = {}
    for flags in (0, HIP_CONTIGUOUS):
        rs = [r for r in rows if r["flags"] == flags and "memory_only_ms" in r]
        if rs:
            m = [min(r["memory_only_ms"]) for r in rs]
            p = [min(r["product_ms"]) for r in rs]
            summ["contiguous" if flags else "default"] = {"memory_only_ms": [min(m), max(m)], "product_ms": [min(p), max(p)]}
    print(json.dumps({"workload": args.workload, "frames": nf, "box": bench.box_identity(torch), "summary": summ,
                      "allocations": rows}))


if __name__ == "__main__":
    main()
