#!/bin/bash
# Kernel durations (rocprof) of the persistent and latency kernels per case.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-lat2}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d $O/kt -o lat -- python3 $R/tools/latency_sweep.py > $O/sweep.json 2> $O/sweep.err || { echo PROF FAILED; tail $O/sweep.err; exit 1; }
cat $O/sweep.json
