#!/bin/bash
# BGR24 sink: full GPU suite, then bench lines against their BGRX counterparts.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-bgr24}
mkdir -p $O
cd $R
timeout -k 10 1500 python -m pytest tests/ -x -q -m gpu > $O/tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for wl in 4k420_bgr24 4k420 stream4k420_d2h_bgr24 stream4k420_d2h; do
  extra=""; case $wl in stream*) extra="--steps 3 --warmup 1";; *) extra="--no-cpu";; esac
  timeout -k 10 600 python bench.py --workload $wl $extra > $O/$wl.json 2> $O/$wl.err || { echo BENCH FAILED $wl; tail $O/$wl.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/$wl.json')); r=d.get('roofline') or {}; print('$wl', d['value'], r.get('frac'), (d.get('end_to_end') or {}).get('output_checked_vs_oracle'))"
done
