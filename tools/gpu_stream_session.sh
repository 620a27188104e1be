#!/bin/bash
# GPU session: entropy/stream parity tests, then the config-5 stream bench
# (GPU entropy) and a kernel trace of it.  Usage: gpu_stream_session.sh TAG [batch...]
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-gs}
shift
BATCHES=${@:-64}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for B in $BATCHES; do
  HJD_STREAM_BATCH=$B timeout -k 10 600 python bench.py --workload stream4k420 --steps 3 --warmup 1 > $O/stream_b$B.json 2> $O/stream_b$B.err || { echo STREAM FAILED; tail -20 $O/stream_b$B.err; exit 1; }
  echo "batch $B: $(python3 -c "import json;d=json.load(open('$O/stream_b$B.json'));print(d['value'], d['ms_per_step'], d['end_to_end'])")"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o stream -- python3 $R/bench.py --workload stream4k420 --steps 2 --warmup 1 > $O/kt.json 2> $O/kt.err || { echo PROF FAILED; tail $O/kt.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1,2,3,4 | grep -v fillBuffer
