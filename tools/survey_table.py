#!/usr/bin/env python3
"""Collect tools/gpu_r04_survey.sh sessions into one table:
    python tools/survey_table.py gpurun_out/r04o gpurun_out/r04q ... > profiles/r04_survey_boxes.json
One row per session: GPU serial; per shape the bench fraction, product and
memory-only times, and the write / read DRAM-credit stalls per kernel cycle
(default launch shape, 256 frames); the streaming probe's best rates."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SHAPES = (("4k420", "decode_kernel<1,0,0>", 1036800), ("4k444", "decode_kernel<0,0,128>", 2073600))


def row(o):
    bpath = os.path.join(o, "survey_bench.json")
    if not os.path.exists(bpath):
        bpath = os.path.join(o, "bench_quick.json")
    b = json.load(open(bpath))
    out = {"session": os.path.basename(o.rstrip("/")), "serial": b["box"].get("serial")}
    for wl, k, t in SHAPES:
        x = b if wl == "4k420" else b["config4_444"]
        d = json.loads(subprocess.run([sys.executable, os.path.join(REPO, "tools", "sq_summary.py"),
                                       os.path.join(o, f"tcc_{wl}"), k, "--tasks-per-dispatch", str(t)],
                                      capture_output=True, text=True).stdout)["derived"]
        out[wl] = {"frac": x["roofline"]["frac"], "product_ms": x["stages"]["product_ms"],
                   "memory_only_ms": x["stages"]["memory_only_ms"],
                   "wr_credit_stall_per_cycle": d.get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_per_cycle"),
                   "rd_credit_stall_per_cycle": d.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_per_cycle"),
                   "profiled_clock_GHz": d.get("effective_clock_GHz")}
    out["probe_GBps"] = json.load(open(os.path.join(o, "box_probe.json"))).get("best_GBps_nt_xcd")
    pro = os.path.join(o, "bench_quick.json")   # the prologue's bench, an earlier process of the same call
    if bpath != pro and os.path.exists(pro):
        p = json.load(open(pro))
        out["prologue_process"] = {wl: {"frac": x["roofline"]["frac"], "product_ms": x["stages"]["product_ms"],
                                        "memory_only_ms": x["stages"]["memory_only_ms"]}
                                   for wl, x in (("4k420", p), ("4k444", p["config4_444"]))}
    return out


if __name__ == "__main__":
    rows = [row(o) for o in sys.argv[1:]]
    print(json.dumps({"what": "box survey sessions (tools/gpu_r04_survey.sh): bench fractions, same-run stage "
                              "times and L2 write/read DRAM-credit stalls at the default launch shape",
                      "rows": rows}, indent=1))
