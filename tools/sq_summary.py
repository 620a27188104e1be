#!/usr/bin/env python3
"""Per-dispatch SQ / TCC counter summary of one fused-kernel instantiation.

    python tools/sq_summary.py <rocprof_dir> "<kernel match>" [--tasks-per-dispatch N] [--min-ms 1.0]

Reads every *counter_collection.csv under the directory (one file per
rocprofv3 pass), keeps the dispatches of the kernel whose name contains the
match (spaces ignored) and that last at least --min-ms (the bench's batch
launches, not its small ones), drops the first such dispatch of each pass
(warmup) and averages the rest.  Units (MI355X_MICROARCH.md): SQ_WAVE_CYCLES,
SQ_WAIT_*, SQ_ACTIVE_INST_* and SQ_BUSY_CYCLES count quad-cycles;
GRBM_GUI_ACTIVE is summed over the 8 XCDs, so the effective clock is
GRBM_GUI_ACTIVE / 8 / kernel time.  Derived: VALU busy = ACTIVE_INST_VALU x 4 /
(cycles x 1024 SIMDs); average resident waves per SIMD = WAVE_CYCLES x 4 /
(cycles x 1024).  Profiled passes run at a lower clock than un-profiled ones,
so compare derived fractions, not times, with the bench.
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import json
import os


def collect(root, match, min_ms):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    for p in sorted(glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True)):
        rows = [r for r in csv.DictReader(open(p)) if match in r["Kernel_Name"].replace(" ", "")]
        ids = sorted({int(r["Dispatch_Id"]) for r in rows})
        for r in rows:
            k = (p, int(r["Dispatch_Id"]))
            per[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        keep = [i for i in ids if dur[(p, i)] >= min_ms][1:]   # drop the pass's warmup dispatch
        for i in ids:
            if i not in keep:
                per.pop((p, i), None)
    tot = collections.defaultdict(list)
    for k, v in per.items():
        for a, b in v.items():
            tot[a].append((b, dur[k]))
    return {a: (sum(x for x, _ in v) / len(v), sum(d for _, d in v) / len(v), len(v)) for a, v in tot.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("match")
    ap.add_argument("--tasks-per-dispatch", type=float, default=0)
    ap.add_argument("--min-ms", type=float, default=1.0)
    a = ap.parse_args()
    c = collect(a.dir, a.match.replace(" ", ""), a.min_ms)
    v = {k: x[0] for k, x in c.items()}
    out = {"kernel_match": a.match, "dispatches_averaged": {k: x[2] for k, x in c.items()},
           "counters_per_dispatch": {k: round(x, 1) for k, x in v.items()}}
    if "GRBM_GUI_ACTIVE" in c:
        cyc = v["GRBM_GUI_ACTIVE"] / 8
        ms = c["GRBM_GUI_ACTIVE"][1]
        d = {"kernel_ms_profiled": round(ms, 4), "effective_clock_GHz": round(cyc / ms / 1e6, 3)}
        if "SQ_ACTIVE_INST_VALU" in v:
            d["valu_busy_frac"] = round(v["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 1024), 3)
        if "SQ_ACTIVE_INST_LDS" in v:
            d["lds_issue_busy_frac"] = round(v["SQ_ACTIVE_INST_LDS"] * 4 / (cyc * 1024), 3)
        if "SQ_BUSY_CYCLES" in v:
            d["sq_busy_frac"] = round(v["SQ_BUSY_CYCLES"] * 4 / (cyc * 8 * 4), 3)
        for k in ("TCC_EA0_WRREQ_STALL_sum", "TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum"):
            if k in v:
                d[k.replace("_sum", "") + "_per_cycle"] = round(v[k] / cyc, 3)
        out["derived"] = d
    if "SQ_WAVES" in v:
        w = v["SQ_WAVES"]
        per_wave = {k: round(v[k] / w, 1) for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
                                                     "SQ_INSTS_VMEM_WR") if k in v}
        out["per_wave"] = per_wave
        if a.tasks_per_dispatch:
            out["per_task"] = {k: round(v[k] / a.tasks_per_dispatch, 1) for k in per_wave}
        if "SQ_WAVE_CYCLES" in v:
            wc = v["SQ_WAVE_CYCLES"]
            out["wave_cycle_split"] = {k: round(v[k] / wc, 3) for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                                                                       "SQ_ACTIVE_INST_ANY") if k in v}
            if "GRBM_GUI_ACTIVE" in v:
                out["derived"]["avg_waves_per_simd"] = round(wc * 4 / (v["GRBM_GUI_ACTIVE"] / 8 * 1024), 2)
    if "SQ_LDS_BANK_CONFLICT" in v and "SQ_INSTS_LDS" in v:
        out["lds_bank_conflict_cycles_per_lds_inst"] = round(v["SQ_LDS_BANK_CONFLICT"] / v["SQ_INSTS_LDS"], 3)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
