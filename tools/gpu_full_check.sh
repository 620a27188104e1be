#!/bin/bash
# Round-end rehearsal: full GPU test suite, smoke(), default bench (N=1) and
# the config-4/config-5 bench lines.  Usage: gpu_full_check.sh TAG
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-full}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest --timeout 120 --timeout-method thread tests/ -x -q -m gpu > $O/tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 python bench.py --workload 4k444 --no-cpu --no-stream > $O/bench444.json 2> $O/bench444.err || { echo BENCH444 FAILED; exit 1; }
timeout -k 10 600 python bench.py --workload stream4k420 --steps 3 --warmup 1 > $O/stream.json 2> $O/stream.err || { echo STREAM FAILED; exit 1; }
python3 -c "
import json
for f in ('bench444', 'stream'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d.get('roofline') and d['roofline']['frac'])"
