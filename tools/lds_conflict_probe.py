"""Attribute the fused kernel's LDS bank conflicts: one
plan of synthetic 3840x2160 frames (default 4:4:4, 64 frames), launched as
the product kernel and as the stage-ablation variants (hjd_debug_plan_launch_
stages: 16 no IDCT -- no zigzag gather, transpose or sample write-back --,
8 no colour stage, 64 no colour math, 256 the gather without bank conflicts),
each `--reps` times, and then `--timed` interleaved rounds of the product
and the conflict-free gather timed with HIP events (what the conflicts cost).  Run under

    rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAVES --kernel-trace \
        --output-format csv -d <dir> -o lds -- python3 tools/lds_conflict_probe.py

and summarise with --summarise <dir>: per kernel variant, conflict cycles per
task and per dispatch.  The launch order is printed (JSON) so the dispatches
can be matched to the variants.
"""
import argparse
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

VARIANTS = [(0, "product"), (16, "no_idct"), (8, "no_colour"), (64, "no_csc"), (256, "broadcast_gather")]


def run(a):
    import torch
    import ocljpegdecoder_amd as hjd
    import oracle_py as O
    w, h, s, nf = 3840, 2160, a.sampling, a.frames
    coefs, qt = O.synthetic_coefs(w, h, s, seed=5)
    nblk = coefs.shape[0]
    ctx = hjd.Context(0)
    specs = [hjd.FrameSpec(w, h, s, coef_offset=i * nblk, out_offset=i * h * w * 4, qt_index=(0, 1, 2))
             for i in range(nf)]
    plan = hjd.Plan(ctx, specs, hjd.IN_Q16_ZIGZAG, qtables=qt)
    d_coefs = torch.from_numpy(coefs).cuda().repeat(nf, 1)
    out = torch.empty((nf, h, w), dtype=torch.int32, device="cuda")
    order = []
    for st, name in VARIANTS:
        for _ in range(a.reps):
            if st == 0:
                plan.launch(d_coefs, out)
            else:
                plan.launch_stages(st, d_coefs, out)
            order.append(name)
        torch.cuda.synchronize()
        if st == 0:   # the product's output is right
            got = out[0].cpu().numpy().view("uint32")
            assert (got == O.decode_q16(coefs, qt, w, h, s)).all()
    timed = {"product": [], "broadcast_gather": []}
    for _ in range(a.timed):
        for st, name in ((0, "product"), (256, "broadcast_gather")):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(5):
                plan.launch(d_coefs, out) if st == 0 else plan.launch_stages(st, d_coefs, out)
            e1.record()
            torch.cuda.synchronize()
            timed[name].append(round(e0.elapsed_time(e1) / 5, 4))
    print(json.dumps({"order": order, "tasks": plan.tasks, "frames": nf, "sampling": s,
                      "shape": plan.launch_shape(), "ms_per_launch": timed,
                      "how": "HIP events around 5 launches, interleaved rounds (no profiler when --timed runs alone)"}))
    plan.close()
    ctx.close()


def summarise(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    by = {}
    for r in rows:
        if "decode_kernel" not in r["Kernel_Name"]:
            continue
        key = (r["Dispatch_Id"], r["Kernel_Name"])
        by.setdefault(key, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    out = {}
    for (did, name), c in sorted(by.items(), key=lambda kv: int(kv[0][0])):
        k = name[name.index("decode_kernel"):].split("(")[0]
        agg = out.setdefault(k, {"dispatches": 0})
        agg["dispatches"] += 1
        for cn, v in c.items():
            agg[cn] = agg.get(cn, 0.0) + v
    for k, agg in out.items():
        n = agg["dispatches"]
        for cn in list(agg):
            if cn != "dispatches":
                agg[cn] = agg[cn] / n
        if agg.get("SQ_ACTIVE_INST_LDS"):
            agg["conflict_frac_of_lds_active"] = round(agg.get("SQ_LDS_BANK_CONFLICT", 0) / agg["SQ_ACTIVE_INST_LDS"], 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--sampling", type=int, default=0)
    ap.add_argument("--frames", type=int, default=64)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--timed", type=int, default=0)
    ap.add_argument("--summarise")
    a = ap.parse_args()
    summarise(a.summarise) if a.summarise else run(a)
