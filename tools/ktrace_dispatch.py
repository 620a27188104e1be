#!/usr/bin/env python3
"""Split a rocprofv3 kernel trace of a bench.py run into warmup and timed
dispatches of the pixel kernel, per workload.

    python tools/ktrace_dispatch.py <rocprof_dir> <bench_json> <name> [--warmup 3 --steps 20]

bench.py (default command) launches, in this order: W warmup + K timed
launches of the 4:2:0 batch (decode_kernel<1,...>), then W + K of the 4:4:4
batch (decode_kernel<0,...>), then (config-5 leg) the stream's kernels in a
child process.  The first W + K dispatches of each decode_kernel
instantiation, in start-time order, are therefore the bench's own; the
stream child's pixel dispatches come after them.  Writes
profiles/<name>_dispatch.json, which bench.py cites as kernel_trace_source:
per workload the dispatch durations, the timed mean, and the frac it implies
against the line's algorithmic bytes; plus the bench line of the same run.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"4k420": "hjd::decode_kernel<1,", "4k444": "hjd::decode_kernel<0,"}   # matched without spaces
# (the product's exact instantiation is picked per workload from the bench line's launch variant)
PEAK = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("bench_json")
    ap.add_argument("name")
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--frames", type=int, default=1024)
    ap.add_argument("--command", default="python bench.py")
    args = ap.parse_args()
    rows = []
    for p in sorted(glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True)):
        with open(p, newline="") as f:
            for r in csv.DictReader(f):
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    line = None
    with open(args.bench_json) as f:
        for l in f:
            if l.startswith("{"):
                line = json.loads(l)
    out = {"name": args.name, "command": args.command, "source_dir": os.path.relpath(args.dir, REPO),
           "warmup": args.warmup, "steps": args.steps,
           "workloads": split(rows, line, args.warmup, args.steps, args.frames)}
    dst = os.path.join(REPO, "profiles", f"{args.name}_dispatch.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps({k: {kk: vv for kk, vv in v.items() if kk != "dispatch_ms"} for k, v in out["workloads"].items()},
                     indent=1))


def split(rows, line, warmup, steps, frames):
    """{workload: summary} from (start, end, kernel name) dispatch rows sorted by
    start and the bench line of the traced run (None if absent)."""
    workloads = {}
    n = warmup + steps
    clocks = [s for s, e, k in rows if "clock_probe_kernel" in k]
    for wl, key in KERNELS.items():
        src = (line if wl == "4k420" else (line or {}).get("config4_444")) or {}
        var = (src.get("launch") or {}).get("variant") or 0
        # the product's instantiation: launch variant bits, + the d16 gather bit
        # at 4:4:4 when the trace has it (hjd_runtime.hip launch_decode)
        names = {k.replace(" ", "") for _s, _e, k in rows}
        inst = f"{key}0,{var}>"
        d16 = f"{key}0,{var | 128}>"
        if any(d16 in nm for nm in names):
            inst = d16
        ds = [(s, e) for s, e, k in rows if inst in k.replace(" ", "")]
        if not ds:
            continue
        # the bench's own launches come before its clock probe (bench.py pixel_batch:
        # autotune, warmup + timed, then clock_under_load, stage variants, ceiling):
        # the W + K dispatches right before the first clock probe after this
        # workload's first dispatch (all of them when no probe ran)
        stop = next((c for c in clocks if c > ds[0][0]), None)
        before = [(s, e) for s, e in ds if stop is None or s < stop]
        d = [(e - s) / 1e6 for s, e in before[-n:]]
        if len(d) < n:
            continue
        timed = d[warmup:]
        e = {"kernel": inst, "frames_per_launch": frames, "dispatch_ms": [round(x, 6) for x in d],
             "dispatches_of_kernel_before_timed": len(before) - n,
             "warmup_dispatches": warmup, "timed_dispatches": len(timed),
             "timed_mean_ms": round(sum(timed) / len(timed), 6), "timed_min_ms": round(min(timed), 6),
             "timed_max_ms": round(max(timed), 6)}
        if line:
            rf = src.get("roofline") or {}
            if rf:
                algo = rf["algorithmic_bytes_per_launch"]
                e["bench_kernel_ms_per_launch_same_run"] = rf["kernel_ms_per_launch"]
                e["bench_frac_same_run"] = rf["frac"]
                e["frac_from_timed_dispatches"] = round(algo / (e["timed_mean_ms"] / 1e3) / 1e9 / PEAK, 4)
                e["bench_ms_per_step_same_run"] = src.get("ms_per_step")
                e["bench_value_same_run"] = src.get("value")
        workloads[wl] = e
    return workloads


if __name__ == "__main__":
    main()
