#!/usr/bin/env python3
"""GPU busy fraction and kernel concurrency from a rocprofv3 kernel-trace CSV.

    python tools/trace_busy.py path/to/*_kernel_trace.csv [--from-frac 0.33]
"""
import collections
import csv
import sys


def main():
    path = sys.argv[1]
    frac = float(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[2] == "--from-frac" else 0.33
    rows = list(csv.DictReader(open(path)))
    ev = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0 if "anonymous" not in r["Kernel_Name"] else 1][:40])
                for r in rows if "fillBuffer" not in r["Kernel_Name"] and "copyBuffer" not in r["Kernel_Name"])
    t_lo = ev[int(len(ev) * frac)][0]
    t_hi = max(e for _, e, _ in ev)
    win = [(max(s, t_lo), min(e, t_hi), n) for s, e, n in ev if e > t_lo and s < t_hi]
    busy, cur = 0, None
    for s, e, _ in sorted(win):
        if cur is None or s > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [s, e]
        else:
            cur[1] = max(cur[1], e)
    busy += cur[1] - cur[0]
    pts = sorted([(s, 1) for s, _, _ in win] + [(e, -1) for _, e, _ in win])
    conc, c, last = collections.Counter(), 0, pts[0][0]
    for t, d in pts:
        conc[c] += t - last
        c += d
        last = t
    tot = sum(conc.values())
    per = collections.Counter()
    for s, e, n in win:
        per[n] += e - s
    print(f"window {(t_hi - t_lo) / 1e6:.1f} ms, GPU busy {busy / 1e6:.1f} ms ({busy / (t_hi - t_lo) * 100:.0f}%)")
    print("concurrent kernels (share of window):", {k: f"{v / tot * 100:.0f}%" for k, v in sorted(conc.items())})
    print("kernel time (sum of durations):", {k: f"{v / 1e6:.1f} ms" for k, v in per.most_common()})


if __name__ == "__main__":
    main()
