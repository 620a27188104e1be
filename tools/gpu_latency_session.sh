#!/bin/bash
# Latency kernel: full GPU suite, the persistent-vs-latency sweep, FHD bench.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-lat}
mkdir -p $O
cd $R
timeout -k 10 1500 python -m pytest tests/ -x -q -m gpu > $O/tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python tools/latency_sweep.py > $O/sweep.json 2> $O/sweep.err || { echo SWEEP FAILED; tail $O/sweep.err; exit 1; }
cat $O/sweep.json
for k in 200; do
  timeout -k 10 300 python bench.py --workload fhd420 --steps $k --warmup 20 --no-cpu --no-stream > $O/fhd_$k.json 2> $O/fhd_$k.err || { echo BENCH FAILED; tail $O/fhd_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/fhd_$k.json')); print('fhd steps', $k, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
