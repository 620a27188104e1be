#!/bin/bash
# Round-3 closing check of the final tree: the
# whole GPU suite, smoke, the driver's default bench command, and the same
# command under a rocprofv3 kernel trace (split into warmup/timed dispatches
# offline by tools/ktrace_dispatch.py).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03j}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests/ -x -m gpu > $O/tests.log 2>&1 \
    || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['config4_444']; s=d['config5_stream']; print('bench', d['value'], d['roofline']['frac'], '444', c['value'], c['roofline']['frac'], 'stream', s.get('value'), s.get('timed_frame_ids'), s.get('error'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o bench -- \
    python3 $R/bench.py > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTRACE FAILED; tail -20 $O/kt_bench.err; exit 1; }
echo "ktrace done"
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $p --output-format csv -d $O/pmc_$p -o pmc -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-stream > $O/pmc_$p.json 2> $O/pmc_$p.err || { echo PMC $p FAILED; tail -20 $O/pmc_$p.err; exit 1; }
done
echo "pmc passes done"
