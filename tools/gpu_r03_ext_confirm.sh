#!/bin/bash
# Confirm the per-shape chunk defaults: extension GPU tests, then the default
# grid on each affected workload (no HJD_TASKS_PER_WAVE), two rounds.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03extc}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_extensions.py tests/test_gpu_kernels.py -x -q --timeout 120 \
    --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; echo TESTS FAILED; exit 1; }
tail -1 $O/tests.log
for rnd in 1 2; do
  for wl in 4kgray 4k411 4k420_i32 4k444_i32 4k420 4k444; do
    timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-stream > $O/${wl}_$rnd.json 2> $O/${wl}_$rnd.err \
        || { echo "$wl FAILED"; tail $O/${wl}_$rnd.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['output_checked_vs_oracle'])" $O/${wl}_$rnd.json "$wl $rnd"
  done
done
