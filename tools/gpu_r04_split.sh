#!/bin/bash
# Round 4: each XCD walking its eighth of the grid in S concurrent parts
# (HJD_XCD_SPLIT=S, build/variants/splitS) against the default (S = 1), on
# fresh allocations (tools/alloc_var.py), alternating processes.
# Usage: tools/gpu_r04_split.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04y}
mkdir -p $O
cd $R
for rep in 1 2; do
  for lib in def split2 split4 split8; do
    if [ $lib = def ]; then unset HJD_LIB; else export HJD_LIB=$R/build/variants/$lib/libhjd.so; fi
    for wl in 4k420 4k444; do
      timeout -k 10 300 python -u tools/alloc_var.py --workload $wl --allocs 4 --reps 3 > $O/s_${wl}_${lib}_$rep.json 2> $O/s_${wl}_${lib}_$rep.err \
          || { echo ALLOC $lib $wl FAILED; tail -5 $O/s_${wl}_${lib}_$rep.err; exit 1; }
    done
  done
done
unset HJD_LIB
python3 - $O <<'PY'
import json, sys, glob, statistics
for p in sorted(glob.glob(f"{sys.argv[1]}/s_*.json")):
    d = json.load(open(p))
    m = [min(a["memory_only_ms"]) for a in d["allocations"]]
    pr = [min(a["product_ms"]) for a in d["allocations"]]
    print(p.rsplit("/", 1)[1], "mem", m, "prod", pr, "prod_mean", round(statistics.mean(pr), 3))
PY
