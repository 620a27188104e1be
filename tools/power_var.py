#!/usr/bin/env python3
"""Run-to-run spread of the pixel kernel against board power (round-4 box study).

    python tools/power_var.py [--workload 4k444] [--frames 1024] [--rounds 24] [--reps 3]

Alternates the product kernel and its memory-only variant (stages 80) on one
plan, timing each segment with HIP events, while a thread samples the GPU's
hwmon power / clock files (sysfs, every 50 ms; no subprocess).  Prints one
JSON object: per segment its time and the board power over its wall-clock
window, and per variant the spread of the times and the power at the fastest
and slowest segments.  The question: when the product is slow, is the board at
its power limit while the memory-only variant of the same buffers is not?
"""
import argparse
import glob
import json
import os
import statistics
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def hwmon_files():
    """{name: path} of the amdgpu hwmon power / clock inputs (first card that has them)."""
    for hw in sorted(glob.glob("/sys/class/drm/card*/device/hwmon/hwmon*")):
        files = {}
        for key, pats in (("power_uW", ("power1_average", "power1_input")), ("sclk_Hz", ("freq1_input",)),
                          ("mclk_Hz", ("freq2_input",)), ("temp_mC", ("temp1_input",)),
                          ("temp_mem_mC", ("temp3_input",))):
            for p in pats:
                f = os.path.join(hw, p)
                if os.path.exists(f):
                    files[key] = f
                    break
        if "power_uW" in files:
            return files
    return {}


class Sampler(threading.Thread):
    def __init__(self, files, period=0.05):
        super().__init__(daemon=True)
        self.files, self.period, self.samples, self.stop = files, period, [], False

    def run(self):
        while not self.stop:
            row = {"t": time.time()}
            for k, f in self.files.items():
                try:
                    with open(f) as fh:
                        row[k] = int(fh.read().strip())
                except (OSError, ValueError):
                    pass
            self.samples.append(row)
            time.sleep(self.period)

    def window(self, t0, t1, key):
        v = [s[key] for s in self.samples if t0 <= s["t"] <= t1 and key in s]
        return (round(statistics.mean(v), 1), max(v), len(v)) if v else (None, None, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="4k444")
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--rounds", type=int, default=24)
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
    coefs = torch.empty((nf, nblk, 64), dtype=torch.int16, device=dev)
    for i in range(min(8, nf)):
        coefs[i] = bench.synth_frame_gpu(torch, nblk, s, qt, seed=i, device=dev)
    for i in range(8, nf):
        coefs[i].copy_(coefs[i % 8])
    out = torch.empty((nf, h, w), dtype=torch.int32, device=dev)
    ctx = hjd.Context(0)
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
             for i in range(nf)]
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
    stream = torch.cuda.current_stream()
    files = hwmon_files()
    sampler = Sampler(files)
    sampler.start()
    segs = []
    for rnd in range(args.rounds):
        for st in (0, 80):
            def go():
                if st:
                    plan.launch_stages(st, coefs, out, stream)
                else:
                    plan.launch(coefs, out, stream)
            go()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.time()
            e0.record(stream)
            for _ in range(args.reps):
                go()
            e1.record(stream)
            torch.cuda.synchronize()
            t1 = time.time()
            p = sampler.window(t0, t1, "power_uW")
            c = sampler.window(t0, t1, "sclk_Hz")
            segs.append({"round": rnd, "stages": st, "ms": round(e0.elapsed_time(e1) / args.reps, 4),
                         "t0": round(t0, 3), "t1": round(t1, 3),
                         "power_W_mean": None if p[0] is None else round(p[0] / 1e6, 1),
                         "power_W_max": None if p[1] is None else round(p[1] / 1e6, 1),
                         "sclk_MHz_mean": None if c[0] is None else round(c[0] / 1e6, 1), "samples": p[2]})
    sampler.stop = True
    summary = {}
    for st in (0, 80):
        ss = [x for x in segs if x["stages"] == st]
        ms = [x["ms"] for x in ss]
        fast, slow = min(ss, key=lambda x: x["ms"]), max(ss, key=lambda x: x["ms"])
        summary["product" if st == 0 else "memory_only"] = {
            "ms_min": min(ms), "ms_median": statistics.median(ms), "ms_max": max(ms),
            "spread_pct": round((max(ms) / min(ms) - 1) * 100, 2),
            "fastest": {k: fast[k] for k in ("round", "ms", "power_W_mean", "sclk_MHz_mean")},
            "slowest": {k: slow[k] for k in ("round", "ms", "power_W_mean", "sclk_MHz_mean")}}
    print(json.dumps({"workload": args.workload, "frames": nf, "reps": args.reps, "box": bench.box_identity(torch),
                      "hwmon": files, "summary": summary, "segments": segs}))


if __name__ == "__main__":
    main()
