#!/bin/bash
# Profiling session on the GPU box (run via gpurun from the repo root).
#   tools/gpu_profile.sh <tag>
# kernel trace + stats of the default bench, PMC passes (tools/pmc_hbm.txt) for
# 4k420 and 4k444 with 256-frame batches.  Every GPU step has its own timeout;
# the script stops at the first failure.
set -u
TAG=${1:-prof}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace -o bench -- \
    python3 $R/bench.py --steps 10 --warmup 2 --no-cpu > $OUT/ktrace_bench.json 2> $OUT/ktrace_bench.err || exit 1
for wl in 4k420 4k444; do
  timeout -k 10 900 rocprofv3 -i $R/tools/pmc_hbm.txt --output-format csv -d $OUT/pmc_$wl -o pmc -- \
      python3 $R/bench.py --workload $wl --frames 256 --steps 3 --warmup 1 --no-cpu > $OUT/pmc_$wl.json 2> $OUT/pmc_$wl.err || exit 1
done
echo "profile $TAG done"
