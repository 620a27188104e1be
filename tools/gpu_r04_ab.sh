#!/bin/bash
# Round 4 A/B of the current library against build/variants/$BASE (default
# base0), alternating processes, product + memory-only variant, both shapes.
# Usage: BASE=base0 tools/gpu_r04_ab.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04ab}
B=${BASE:-base0}
mkdir -p $O
cd $R
for rep in $(seq 1 ${REPS:-2}); do
  for lib in cur $B; do
    if [ $lib = cur ]; then unset HJD_LIB; else export HJD_LIB=$R/build/variants/$lib/libhjd.so; fi
    for wl in 4k420 4k444; do
      timeout -k 10 300 python -u tools/tune.py --workload $wl --frames 256 --rounds 3 --variants 0 \
          --stages 0,80 > $O/ab_${wl}_${lib}_$rep.json 2> $O/ab_${wl}_${lib}_$rep.err \
          || { echo TUNE $lib $wl FAILED; tail -5 $O/ab_${wl}_${lib}_$rep.err; exit 1; }
    done
  done
done
unset HJD_LIB
python3 - $O <<'PY'
import json, sys, glob, collections
res = collections.defaultdict(list)
for p in sorted(glob.glob(f"{sys.argv[1]}/ab_*.json")):
    _, wl, lib, rep = p.rsplit("/", 1)[1][:-5].split("_")
    for r in json.load(open(p))["results"]:
        res[(wl, r.get("stages", 0), lib)].append(r["median_ms"])
for k in sorted(res):
    print(*k, [round(x, 4) for x in res[k]])
PY
