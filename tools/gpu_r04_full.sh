#!/bin/bash
# Round-4 full check of the tree: the whole GPU suite, smoke, the driver's
# default bench command (all legs: 4:2:0 headline, 4:4:4, configs[1] FHD
# launch + JPEG, config-5 stream D2H-off and D2H-on, CPU port + reference on
# all cores), then the box probe.  Usage: tools/gpu_r04_full.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04b}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests/ -x -m gpu > $O/tests.log 2>&1 \
    || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python -u bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -30 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["config4_444"]
for n, x in (("420", d), ("444", c)):
    r = x["roofline"]
    print(n, x["value"], "frac", r["frac"], "box_ceiling", r.get("box_ceiling_GBps"), r.get("frac_of_box_ceiling"),
          "clock", (x.get("clock_under_load") or {}).get("sclk_GHz_median"), "stages", x["stages"])
print("box", d["box"])
for k in ("fhd420", "fhd420_jpeg", "config5_stream", "config5_stream_d2h"):
    v = d.get(k) or {}
    print(k, {kk: v.get(kk) for kk in ("value", "us_per_launch_kernel", "ms_per_image", "output_checked_vs_oracle",
                                       "h2d_ceiling", "d2h_ceiling", "error")})
cb = d.get("cpu_baseline") or {}
print("cpu", cb.get("value"), cb.get("cores"), "ref", d.get("cpu_reference"))
PY
timeout -k 10 300 python -u tools/box_probe.py > $O/box_probe.json 2> $O/box_probe.err || { echo BOXPROBE FAILED; tail -20 $O/box_probe.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/box_probe.json'))
print('d16', d['d16_gather'], 'best', d['best_GBps_nt_xcd'])"
echo "session done"
