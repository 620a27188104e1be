#!/bin/bash
# Tasks-per-wave sweep of the pixel kernel (HJD_TASKS_PER_WAVE), same box:
#   tools/gpu_tpw_sweep.sh TAG WORKLOAD "T1 T2 ..." [ROUNDS]
set -u
TAG=$1; WL=$2; TS=$3; ROUNDS=${4:-2}
O=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for rnd in $(seq 1 $ROUNDS); do
  for t in $TS; do
    HJD_TASKS_PER_WAVE=$t timeout -k 10 300 python bench.py --workload $WL --no-cpu --no-stream \
        > $O/${WL}_${t}_$rnd.json 2> $O/${WL}_${t}_$rnd.err || { echo RUN $t FAILED; tail $O/${WL}_${t}_$rnd.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['roofline']['frac'])" \
        $O/${WL}_${t}_$rnd.json $t $rnd
  done
done
