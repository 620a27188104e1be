#!/bin/bash
# Config-5 stream sweep over entropy/stream settings (tuning):
#   tools/gpu_stream_sweep.sh TAG "SUB_BITS:BATCH:SLOTS ..." [ROUNDS]
# One bench.py stream run (3 timed steps of 1024 frames) per setting and round,
# settings interleaved within each round; prints value per setting.
set -u
TAG=$1; SETS=$2; ROUNDS=${3:-2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for rnd in $(seq 1 $ROUNDS); do
  for s in $SETS; do
    IFS=: read sb bt sl <<< "$s"
    HJD_SUB_BITS=$sb HJD_STREAM_BATCH=$bt HJD_STREAM_SLOTS=$sl timeout -k 10 300 python bench.py --workload stream4k420 \
        --steps 3 --warmup 1 --no-cpu > $O/s_${sb}_${bt}_${sl}_$rnd.json 2> $O/s_${sb}_${bt}_${sl}_$rnd.err || { echo RUN $s FAILED; tail $O/s_${sb}_${bt}_${sl}_$rnd.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'round', sys.argv[3], d['value'])" $O/s_${sb}_${bt}_${sl}_$rnd.json $s $rnd
  done
done
