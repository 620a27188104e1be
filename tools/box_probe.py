#!/usr/bin/env python3
"""Box probe: what THIS MI355X box's HBM sustains for the fused kernel's byte
mixes, so that kernel fractions from different boxes can be compared
(VERDICT r3 "Next" #1: 4:2:0 lost ~10 % on some boxes while 4:4:4 did not).

    python tools/box_probe.py [--gib 56] [--reps 5] > box_probe.json

Runs hjd_debug_rw_mix (csrc/hjd_probe.hip) in ONE process over one pair of
buffers: read:write mixes in KiB per wave-unit -- 0:8 (write only), 6:0 (read
only), 6:8 (a 4:2:0 task), 6:4 (a 4:4:4 task), 4:4 (copy) -- each at 1, 2, 4
and 16 units per wave, with the fused kernel's launch shape (nt loads and
stores, XCD-contiguous group order) and two controls (launch order; plain
stores).  Reports GB/s = (read + written bytes) / mean launch time (HIP
events, `reps` launches after one warmup), plus the box identity and the d16
gather probe.  Diagnostics only; nothing here is on the product path.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def box_identity():
    """Host name, GPU serial / unique id and the smi's static memory facts
    (best effort: smi text kept raw)."""
    out = {"hostname": socket.gethostname()}
    for key, cmd in (("rocm_smi_serial", ["rocm-smi", "--showserial", "--showuniqueid", "--json"]),
                     ("rocm_smi_clocks", ["rocm-smi", "--showclocks", "--json"]),
                     ("rocm_smi_power", ["rocm-smi", "--showpower", "--showmaxpower", "--json"]),
                     ("rocm_smi_partition", ["rocm-smi", "--showcomputepartition", "--showmemorypartition", "--json"]),
                     ("rocm_smi_fw", ["rocm-smi", "--showfwinfo", "--json"])):
        try:
            r = subprocess.run(cmd, capture_output=True, text=True, timeout=30)
            txt = r.stdout.strip()
            try:
                out[key] = json.loads(txt)
            except ValueError:
                out[key] = txt[-2000:]
        except Exception as e:   # smi missing or refused: not fatal
            out[key] = f"unavailable: {e}"
    return out


def rw_sweep(torch, hjd, ctx, gib, reps):
    dev = torch.device("cuda", ctx.device)
    src = torch.empty(int(gib * 3 / 7 * (1 << 30)) // 4096 * 4096, dtype=torch.uint8, device=dev)
    dst = torch.empty(int(gib * 4 / 7 * (1 << 30)) // 4096 * 4096, dtype=torch.uint8, device=dev)
    src.fill_(1)
    dst.zero_()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    rows = []
    configs = []
    for mix in ((0, 8), (6, 0), (6, 8), (6, 4), (4, 4)):
        for upw in (1, 2, 4, 16):
            configs.append((mix, upw, 3))
            if mix[0] and mix[1]:
                configs.append((mix, upw, 7))   # pipelined: next unit's loads before this unit's stores
        configs.append((mix, 2, 1))   # launch order (no XCD remap)
        configs.append((mix, 2, 2))   # plain (temporal) loads and stores
    for (r, w), upw, flags in configs:
        nbytes = ctx.debug_rw_mix(src, dst, r, w, upw, flags, stream)   # warmup
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            ctx.debug_rw_mix(src, dst, r, w, upw, flags, stream)
        e1.record(stream)
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        rows.append({"mix_kib": f"{r}:{w}", "units_per_wave": upw, "nt": bool(flags & 1), "xcd_order": bool(flags & 2),
                     "pipelined": bool(flags & 4),
                     "bytes_per_launch": nbytes, "ms": round(ms, 4), "GBps": round(nbytes / ms / 1e6, 1)})
        print(json.dumps(rows[-1]), file=sys.stderr, flush=True)
    del src, dst
    torch.cuda.empty_cache()
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gib", type=float, default=56.0, help="bytes per launch (src + dst buffers), GiB")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    import torch
    import ocljpegdecoder_amd as hjd
    t0 = time.time()
    res = {"what": "box probe: HBM streaming rates of the fused kernel's byte mixes (hjd_debug_rw_mix)",
           "utc": time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime()), "box": box_identity()}
    torch.cuda.set_device(a.device)
    ctx = hjd.Context(a.device)
    res["device_name"] = torch.cuda.get_device_properties(a.device).name
    res["gcn_arch"] = getattr(torch.cuda.get_device_properties(a.device), "gcnArchName", None)
    res["d16_gather"] = dict(zip(("probe_zeroes_low_half", "selected"), ctx.d16_gather()))
    res["rw_mix"] = rw_sweep(torch, hjd, ctx, a.gib, a.reps)
    best = {}
    for r in res["rw_mix"]:
        if r["nt"] and r["xcd_order"]:
            best[r["mix_kib"]] = max(best.get(r["mix_kib"], 0), r["GBps"])
    res["best_GBps_nt_xcd"] = best
    res["seconds"] = round(time.time() - t0, 1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
