"""Same-box A/B of the single-JPEG latency (bench.py --workload fhd420_jpeg):
the product library against build/variants/<name>/libhjd.so builds (HJD_LIB),
interleaved over --rounds, each run a child process.

    python tools/fhd_ab.py --variants base[+other] [--rounds 3] [--steps 200]

Prints one JSON document: every run's latencies and per-library medians.
"""
import argparse
import json
import os
import statistics
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, steps, extra):
    env = dict(os.environ)
    env.pop("HJD_LIB", None)
    if lib != "product":
        env["HJD_LIB"] = os.path.join(REPO, "build", "variants", lib, "libhjd.so")
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--workload", "fhd420_jpeg", "--no-cpu",
           "--steps", str(steps), "--warmup", "20", *extra]
    p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300)
    if p.returncode != 0:
        raise SystemExit(f"{lib}: bench failed ({p.returncode}): {p.stderr[-2000:]}")
    d = json.loads(p.stdout.strip().splitlines()[-1])
    return {"lib": lib, "latency_ms_per_image": d["latency_ms_per_image"], "ok": d["output_checked_vs_oracle"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--extra", default="")
    a = ap.parse_args()
    libs = ["product"] + a.variants.replace("+", ",").split(",")
    extra = a.extra.split(",") if a.extra else []
    runs = []
    for r in range(a.rounds):
        for lib in (libs if r % 2 == 0 else libs[::-1]):
            runs.append(one(lib, a.steps, extra))
            print(json.dumps(runs[-1]), file=sys.stderr, flush=True)
    med = {}
    for lib in libs:
        rs = [x for x in runs if x["lib"] == lib]
        med[lib] = {k: statistics.median(x["latency_ms_per_image"][k] for x in rs)
                    for k in rs[0]["latency_ms_per_image"]}
        med[lib]["all_ok"] = all(x["ok"] for x in rs)
    print(json.dumps({"what": "fhd420_jpeg latency A/B, interleaved child runs", "steps": a.steps,
                      "rounds": a.rounds, "median_ms": med, "runs": runs}, indent=1))


if __name__ == "__main__":
    main()
