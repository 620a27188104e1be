#!/bin/bash
# 4:4:4 gather forms on one library: the d16 gather (default on sramecc+) vs
# HJD_D16=0 (v_perm gather), alternated; then the pixel-kernel GPU tests.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03d16b}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_batch_scale.py \
    tests/test_gpu_extensions.py -x -q -s --timeout 200 --timeout-method thread > $O/tests.log 2>&1 \
    || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
grep -m2 "d16 gather" $O/tests.log; tail -1 $O/tests.log
for i in $(seq 1 ${2:-3}); do
  for V in perm d16; do
    E=""; [ $V = perm ] && E=0
    HJD_D16=${E:-1} timeout -k 10 180 python tools/tune.py --workload 4k444 --frames 256 --variants 0 --rounds 5 --reps 1 \
        > $O/${V}_$i.json 2> $O/${V}_$i.err || { echo RUN FAILED $V; tail $O/${V}_$i.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/${V}_$i.json')); r=d['results'][0]; print('$V', $i, r['median_ms'], r['GBps_median'], d['signature'])"
  done
done
