#!/usr/bin/env python3
"""Summarise rocprofv3 CSV output into profiles/<name>.json (+ copy the stats CSV).

    python tools/prof_summary.py <rocprof_dir> <name> --workload 4k420 [--kernel decode_kernel]

Kernel trace  (<prefix>_kernel_stats.csv / _kernel_trace.csv): per-kernel calls and
              average duration.
PMC           (<prefix>_counter_collection.csv, one or more passes): per-dispatch
              counters of the hot kernel.  HBM bytes per launch follow
              MI355X_MICROARCH.md s HBM: FETCH_SIZE and WRITE_SIZE are KiB; on
              gfx950 FETCH_SIZE reads 1/2 of a wide coalesced stream's bytes, so
              hbm = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (the raw values are kept).
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import shutil
import statistics

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def read_csv(path):
    with open(path, newline="") as f:
        return list(csv.DictReader(f))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("name")
    ap.add_argument("--workload", default="4k420")
    ap.add_argument("--kernel", default="decode_kernel")
    ap.add_argument("--note", default="")
    ap.add_argument("--box", default="", help="box identity of the profiled run (e.g. GPU serial), recorded for "
                                              "bench.py's traffic_other_run")
    ap.add_argument("--frames", type=int, default=1024, help="frames per launch of the profiled command (bench.py)")
    args = ap.parse_args()
    out = {"name": args.name, "workload": args.workload, "kernel_match": args.kernel, "note": args.note,
           "frames_per_launch": args.frames, "box": args.box or "not recorded",
           "source_dir": os.path.relpath(args.dir, REPO)}

    stats = sorted(glob.glob(os.path.join(args.dir, "**", "*kernel_stats.csv"), recursive=True))
    if stats:
        rows = read_csv(stats[0])
        out["kernel_stats"] = [{"name": r["Name"][:160], "calls": int(r["Calls"]),
                                "avg_ns": float(r["AverageNs"]), "min_ns": float(r["MinNs"]),
                                "max_ns": float(r["MaxNs"]), "pct": float(r["Percentage"])}
                               for r in rows[:8]]
        hot = [r for r in out["kernel_stats"] if args.kernel in r["name"]]
        if hot:
            out["hot_kernel_avg_ms"] = hot[0]["avg_ns"] / 1e6
        shutil.copy(stats[0], os.path.join(REPO, "profiles", f"{args.name}_kernel_stats.csv"))

    pmc_files = sorted(glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True))
    if pmc_files:
        per_counter = {}
        for pf in pmc_files:
            for r in read_csv(pf):
                if args.kernel not in r.get("Kernel_Name", ""):
                    continue
                per_counter.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        med = {k: statistics.median(v) for k, v in per_counter.items()}
        out["pmc_median_per_dispatch"] = med
        out["pmc_dispatches"] = {k: len(v) for k, v in per_counter.items()}
        if "FETCH_SIZE" in med and "WRITE_SIZE" in med:
            fetch = 2 * med["FETCH_SIZE"] * 1024.0
            write = med["WRITE_SIZE"] * 1024.0
            out["hbm_read_bytes_per_launch"] = fetch
            out["hbm_write_bytes_per_launch"] = write
            out["hbm_bytes_per_launch"] = fetch + write
            out["hbm_correction"] = "read = 2 x FETCH_SIZE KiB (gfx950 half-count), write = WRITE_SIZE KiB"
    dst = os.path.join(REPO, "profiles", f"{args.name}.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1)[:3000])


if __name__ == "__main__":
    main()
