#!/usr/bin/env python3
"""GPU entropy decode throughput (hjd_gdec) on synthetic 4K JPEGs.

    python tools/entropy_bench.py [--frames 16] [--reps 10] [--sub-bits 1024] [--sampling 420] [--pixels]

Prints one JSON object: wall-clock Mpx/s over `reps` batched calls on one
stream (host staging of call i+1 overlaps the device work of call i) and the
device time per batch from HIP events.  Kernel-level times come from running
this under rocprofv3 --kernel-trace --stats.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--sub-bits", type=int, default=0)
    ap.add_argument("--sampling", default="420", choices=["420", "444"])
    ap.add_argument("--pool", type=int, default=8)
    ap.add_argument("--pixels", action="store_true", help="also run the fused pixel kernel (full decode)")
    ap.add_argument("--pinned", action="store_true",
                    help="JPEG bytes in pinned host memory (destuffed on the GPU unless HJD_DESTUFF=host)")
    ap.add_argument("--no-check", action="store_true",
                    help="timing experiments whose outputs are wrong by design (HJD_LIB variants)")
    args = ap.parse_args()

    import torch
    import bench
    import ocljpegdecoder_amd as hjd

    w, h = 3840, 2160
    s = 1 if args.sampling == "420" else 0
    pool = bench.encode_pool(w, h, s, args.pool, seed0=99)
    datas = [pool[i % len(pool)] for i in range(args.frames)]
    infos = [hjd.parse(d) for d in datas]
    host_datas = datas
    if args.pinned:
        pinned = [hjd.pinned_bytes(d) for d in pool]
        datas = [pinned[i % len(pool)] for i in range(args.frames)]
    nblk = sum(i.nblocks for i in infos)
    scan = sum(len(d) for d in host_datas)
    ctx = hjd.Context(0)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    coefs = torch.empty((nblk, 64), dtype=torch.int16, device=dev)
    outs = [torch.empty((h, w), dtype=torch.int32, device=dev) for _ in datas]
    gd = hjd.GpuDecoder(ctx, args.frames, scan, nblk, args.sub_bits)

    def call():
        if args.pixels:
            gd.decode(datas, outs, stream)
        else:
            gd.decode_coefs(datas, coefs, stream)

    def sync():
        try:
            return gd.sync()
        except Exception:
            if not args.no_check:
                raise
            return [0] * args.frames

    call()
    status = sync()
    # exactness spot check against the host decoder (first distinct frames)
    if not args.pixels and not args.no_check:
        offs = gd.decode_coefs(datas, coefs, stream)
        gd.sync()
        got = coefs.cpu().numpy()
        for i in range(min(2, len(datas))):
            ref, _ = hjd.decode_coefs(host_datas[i])
            assert (got[offs[i]:offs[i] + infos[i].nblocks] == ref).all(), "GPU coefficients differ"
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(args.reps):
        call()
    e1.record(stream)
    sync()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    dev_ms = e0.elapsed_time(e1) / args.reps
    px = w * h * args.frames
    print(json.dumps({
        "what": "GPU entropy decode" + (" + fused pixel kernel" if args.pixels else " (coefficients only)"),
        "frames_per_batch": args.frames, "sampling": args.sampling, "sub_bits": args.sub_bits or 1024,
        "mean_jpeg_bytes": scan // args.frames, "wall_Mpx_s": round(px * args.reps / wall / 1e6, 1),
        "device_ms_per_batch": round(dev_ms, 3), "device_Mpx_s": round(px / (dev_ms / 1e3) / 1e6, 1),
        "scan_GBps_device": round(scan / (dev_ms / 1e3) / 1e9, 2),
        "fallback_frames": sum(1 for x in status if x & 1)}))
    gd.close()


if __name__ == "__main__":
    main()
