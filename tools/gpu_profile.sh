#!/bin/bash
# Profiling session on the GPU box (run via gpurun from the repo root).
#   tools/gpu_profile.sh <tag> [workload...]
# For each workload: rocprofv3 kernel trace + stats of bench.py, then the HBM
# PMC passes (tools/pmc_traffic.txt: FETCH_SIZE, WRITE_SIZE in separate passes)
# on the same bench command.  Every GPU step has its own timeout; the script
# stops at the first failure.
set -u
TAG=${1:-prof}; shift
WLS=${@:-4k420}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for wl in $WLS; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/ktrace_$wl -o bench -- \
      python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-cpu --no-stream > $OUT/ktrace_$wl.json 2> $OUT/ktrace_$wl.err || exit 1
  timeout -k 10 900 rocprofv3 -i $R/tools/pmc_traffic.txt --output-format csv -d $OUT/pmc_$wl -o pmc -- \
      python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-stream > $OUT/pmc_$wl.json 2> $OUT/pmc_$wl.err || exit 1
done
echo "profile $TAG done"
