#!/bin/bash
# Entropy kernels vs subsequence length S (same box): rocprofv3 kernel trace of
# tools/entropy_bench.py (64 x 4K 4:2:0 frames) for each S.
#   tools/gpu_subbits_sweep.sh TAG S...
set -u
TAG=${1:-ent_s}; shift
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for S in "$@"; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${S}_$rep -o ent -- \
        python3 $R/tools/entropy_bench.py --frames 64 --reps 3 --sub-bits $S ${EB_ARGS:-} > $O/run_${S}_$rep.json 2> $O/run_${S}_$rep.err \
        || { echo PROF $S FAILED; tail $O/run_${S}_$rep.err; exit 1; }
    echo "S=$S $rep: $(find $O/kt_${S}_$rep -name '*kernel_stats.csv' -exec cat {} \; | grep -E 'ent_(sync|write)' | cut -d, -f4 | tr '\n' ' ')"
  done
done
