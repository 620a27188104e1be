#!/bin/bash
# Round 4: tasks-per-wave sweep of the product and of its memory-only variant
# (same process, interleaved rounds), then the pixel bench with the image-row
# box ceiling.  Usage: tools/gpu_r04_tpw.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04c}
mkdir -p $O
cd $R
timeout -k 10 400 python -u tools/tune.py --workload 4k444 --frames 256 --rounds 3 --variants 0 \
    --grids 518400,259200,129600,64800,32400 --stages 0,80 --no-check > $O/tpw_444.json 2> $O/tpw_444.err \
    || { echo TUNE444 FAILED; tail -20 $O/tpw_444.err; exit 1; }
timeout -k 10 400 python -u tools/tune.py --workload 4k420 --frames 256 --rounds 3 --variants 0 \
    --grids 259200,129600,64800,32400 --stages 0,80 --no-check > $O/tpw_420.json 2> $O/tpw_420.err \
    || { echo TUNE420 FAILED; tail -20 $O/tpw_420.err; exit 1; }
python3 - $O <<'PY'
import json, sys
for wl in ("444", "420"):
    d = json.load(open(f"{sys.argv[1]}/tpw_{wl}.json"))
    for r in d["results"]:
        print(wl, r["grid"], r["stages"], r["median_ms"], r["GBps_median"])
PY
timeout -k 10 600 python -u bench.py --no-stream --no-cpu --no-fhd > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for n, x in (("420", d), ("444", d["config4_444"])):
    r = x["roofline"]
    print(n, x["value"], "frac", r["frac"], "ceiling", r.get("box_ceiling_GBps"), r.get("frac_of_box_ceiling"),
          (x.get("box_ceiling") or {}).get("rows"), "clock", (x.get("clock_under_load") or {}).get("sclk_GHz_median"))
print(d["box"])
PY
