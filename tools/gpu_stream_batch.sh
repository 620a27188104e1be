#!/bin/bash
# Config-5 GPU-entropy stream at several (frames per batch, S) settings, same
# box, two reps.   tools/gpu_stream_batch.sh TAG BATCH:S ...
set -u
TAG=${1:-stream_b}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for cfg in "$@"; do
    B=${cfg%%:*}; S=${cfg##*:}
    HJD_STREAM_BATCH=$B HJD_SUB_BITS=$S timeout -k 10 300 python bench.py --workload stream4k420 --steps 3 --warmup 1 \
        > $O/b${B}_s${S}_$rep.json 2> $O/b${B}_s${S}_$rep.err || { echo STREAM $cfg FAILED; tail $O/b${B}_s${S}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/b${B}_s${S}_$rep.json')); print('B=$B S=$S rep $rep', d['value'], d['end_to_end']['jpeg_GBps_in'])"
  done
done
