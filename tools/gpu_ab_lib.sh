#!/bin/bash
# Same-box A/B of two builds of libhjd.so on the pixel kernel (tuning tool):
#   tools/gpu_ab_lib.sh TAG BASE_LIB [WORKLOADS...]
# Runs the pixel-kernel GPU tests on the in-tree library first, then
# tools/tune.py alternately on BASE_LIB (via HJD_LIB) and the in-tree library,
# 3 times each per workload, one process per run.
set -u
TAG=${1:-ab}; BASE=${2:-build/variants/base/libhjd.so}; shift 2
WLS=${@:-4k420 4k444}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_extensions.py \
    -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in $WLS; do
  for rep in 1 2 3; do
    HJD_LIB=$R/$BASE timeout -k 10 180 python tools/tune.py --workload $wl --frames 256 --variants 0 --rounds 5 \
        > $O/base_${wl}_$rep.json 2> $O/base_${wl}_$rep.err || { echo BASE FAILED; tail $O/base_${wl}_$rep.err; exit 1; }
    timeout -k 10 180 python tools/tune.py --workload $wl --frames 256 --variants 0 --rounds 5 \
        > $O/new_${wl}_$rep.json 2> $O/new_${wl}_$rep.err || { echo NEW FAILED; tail $O/new_${wl}_$rep.err; exit 1; }
  done
done
python3 - "$O" <<'EOF'
import glob, json, os, sys
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*_*_*.json"))):
    r = json.load(open(f))["results"][0]
    print(os.path.basename(f), r["median_ms"], r["GBps_median"])
EOF
