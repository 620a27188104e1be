#!/bin/bash
# GPU session: entropy/stream parity tests, then the config-5 stream bench
# (GPU entropy) over batch/slot settings and a kernel trace.
# Usage: gpu_stream_session.sh TAG "B:S B:S ..."
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-gs}
CFGS=${2:-64:5}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for C in $CFGS; do
  B=${C%%:*}; S=${C##*:}
  HJD_STREAM_BATCH=$B HJD_STREAM_SLOTS=$S timeout -k 10 600 python bench.py --workload stream4k420 --steps 3 --warmup 1 > $O/stream_b${B}_s${S}.json 2> $O/stream_b${B}_s${S}.err || { echo STREAM FAILED; tail -20 $O/stream_b${B}_s${S}.err; exit 1; }
  echo "batch $B slots $S: $(python3 -c "import json;d=json.load(open('$O/stream_b${B}_s${S}.json'));print(d['value'], d['ms_per_step'], d['end_to_end'])")"
done
timeout -k 10 120 python tools/h2d_bw.py | tee $O/h2d.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o stream -- python3 $R/bench.py --workload stream4k420 --steps 2 --warmup 1 > $O/kt.json 2> $O/kt.err || { echo PROF FAILED; tail $O/kt.err; exit 1; }
python3 $R/tools/trace_busy.py $O/kt/stream_kernel_trace.csv
