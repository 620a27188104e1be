#!/bin/bash
# Round 4: is the placement sensitivity a property of the task order?  The
# same allocation sequence (tools/alloc_var.py reproduces its per-allocation
# pattern across processes on one box) under the default XCD order (each XCD
# one contiguous eighth of the grid), HJD_XCD=0 (dispatch order) and
# HJD_XCD_CHUNK=4.  Usage: tools/gpu_r04_xcdplace.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04x}
mkdir -p $O
cd $R
for rep in 1 2; do
  for lib in def xcd0 xcdc4; do
    if [ $lib = def ]; then unset HJD_LIB; else export HJD_LIB=$R/build/variants/$lib/libhjd.so; fi
    for wl in 4k420 4k444; do
      timeout -k 10 300 python -u tools/alloc_var.py --workload $wl --allocs 4 --reps 3 > $O/x_${wl}_${lib}_$rep.json 2> $O/x_${wl}_${lib}_$rep.err \
          || { echo ALLOC $lib $wl FAILED; tail -5 $O/x_${wl}_${lib}_$rep.err; exit 1; }
    done
  done
done
unset HJD_LIB
python3 - $O <<'PY'
import json, sys, glob
for p in sorted(glob.glob(f"{sys.argv[1]}/x_*.json")):
    d = json.load(open(p))
    print(p.rsplit("/", 1)[1], [min(a["memory_only_ms"]) for a in d["allocations"]], [min(a["product_ms"]) for a in d["allocations"]])
PY
