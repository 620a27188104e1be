#!/bin/bash
# Full GPU suite + smoke + the pixel bench lines (4k420 default, 4k444, fhd420).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-confirm}
mkdir -p $O
cd $R
timeout -k 10 1500 python -m pytest tests/ -x -q -m gpu > $O/tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
for wl in 4k444 fhd420; do
  extra="--no-cpu"; [ $wl = fhd420 ] && extra="--no-cpu --steps 200 --warmup 20"
  timeout -k 10 600 python bench.py --workload $wl $extra > $O/$wl.json 2> $O/$wl.err || { echo BENCH FAILED $wl; tail $O/$wl.err; exit 1; }
done
python3 -c "
import json
for f in ('bench', '4k444', 'fhd420'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_per_launch'], (d.get('cpu_baseline') or {}).get('value'))"
