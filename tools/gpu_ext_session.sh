#!/bin/bash
# Sampling extensions (4:2:2, gray): full GPU suite, then bench lines.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ext}
mkdir -p $O
cd $R
timeout -k 10 1500 python -m pytest tests/ -x -q -m gpu > $O/tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in 4k422 4kgray 4k420; do
  timeout -k 10 600 python bench.py --workload $wl --no-cpu --no-stream > $O/$wl.json 2> $O/$wl.err || { echo BENCH FAILED $wl; tail $O/$wl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_per_launch'])"
done
