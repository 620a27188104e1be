#!/bin/bash
# Config-5 GPU-entropy stream (bench.py stream4k420) at several subsequence
# lengths S (HJD_SUB_BITS), same box, two reps.   tools/gpu_stream_subbits.sh TAG S...
set -u
TAG=${1:-stream_s}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for rep in 1 2; do
  for S in "$@"; do
    HJD_SUB_BITS=$S timeout -k 10 300 python bench.py --workload stream4k420 --steps 3 --warmup 1 \
        > $O/s${S}_$rep.json 2> $O/s${S}_$rep.err || { echo STREAM $S FAILED; tail $O/s${S}_$rep.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/s${S}_$rep.json')); print('S=$S rep $rep', d['value'], d['end_to_end'])"
  done
done
