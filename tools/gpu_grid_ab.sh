#!/bin/bash
# Same-box A/B of two builds of libhjd.so on the pixel kernel, each over a list
# of persistent grid sizes (tuning tool):
#   tools/gpu_grid_ab.sh TAG BASE_LIB WORKLOAD GRIDS [WORKLOAD GRIDS ...]
# GRIDS is tune.py's comma list (0 = the default grid).  Runs the pixel-kernel
# GPU tests on the in-tree library first, then tune.py alternately on BASE_LIB
# (via HJD_LIB) and the in-tree library, 3 times each, one process per run.
set -u
TAG=$1; BASE=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_extensions.py \
    tests/test_gpu_batch_scale.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
while [ $# -ge 2 ]; do
  wl=$1; grids=$2; shift 2
  for rep in 1 2 3; do
    HJD_LIB=$R/$BASE timeout -k 10 240 python tools/tune.py --workload $wl --frames 256 --variants 0 --grids $grids --rounds 5 \
        > $O/base_${wl}_$rep.json 2> $O/base_${wl}_$rep.err || { echo BASE FAILED; tail $O/base_${wl}_$rep.err; exit 1; }
    timeout -k 10 240 python tools/tune.py --workload $wl --frames 256 --variants 0 --grids $grids --rounds 5 \
        > $O/new_${wl}_$rep.json 2> $O/new_${wl}_$rep.err || { echo NEW FAILED; tail $O/new_${wl}_$rep.err; exit 1; }
    echo "$wl rep $rep done"
  done
done
python3 - "$O" <<'EOF'
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*_*_*.json"))):
    for r in json.load(open(f))["results"]:
        print(os.path.basename(f), "grid", r["grid"], r["median_ms"], r["GBps_median"])
EOF
