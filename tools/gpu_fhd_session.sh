#!/bin/bash
# FHD (configs[1]) latency study + the device-side random entropy sweep.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-fhd}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q -k random_sweep > $O/sweep.log 2>&1 || { echo SWEEP FAILED; tail -30 $O/sweep.log; exit 1; }
tail -1 $O/sweep.log
for k in 10 200; do
  timeout -k 10 300 python bench.py --workload fhd420 --steps $k --warmup 20 --no-cpu --no-stream > $O/fhd_$k.json 2> $O/fhd_$k.err || { echo BENCH FAILED; tail $O/fhd_$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/fhd_$k.json')); print('steps', $k, d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o fhd -- python3 $R/bench.py --workload fhd420 --steps 200 --warmup 20 --no-cpu --no-stream > $O/kt.json 2> $O/kt.err || { echo PROF FAILED; tail $O/kt.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec head -3 {} \;
