#!/bin/bash
# Round 3: the driver's default bench command, then the same command under a
# rocprofv3 kernel trace (split into warmup/timed dispatches offline by
# tools/ktrace_dispatch.py), then the HBM PMC passes of the pixel launches.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03bench}
mkdir -p $O
cd $R
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); c=d['config4_444']; s=d['config5_stream']; print('bench', d['value'], d['roofline']['frac'], '444', c['value'], c['roofline']['frac'], 'stream', s.get('value'), s.get('timed_frame_ids'), s.get('h2d_ceiling'), s.get('error'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o bench -- \
    python3 $R/bench.py > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTRACE FAILED; tail -20 $O/kt_bench.err; exit 1; }
echo ktrace done
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $p --output-format csv -d $O/pmc_$p -o pmc -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-stream > $O/pmc_$p.json 2> $O/pmc_$p.err || { echo PMC $p FAILED; tail -20 $O/pmc_$p.err; exit 1; }
done
echo "bench session $1 done"
