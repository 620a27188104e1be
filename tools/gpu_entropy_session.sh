#!/bin/bash
# GPU session for the entropy decoder: parity tests, then per-S kernel traces
# of tools/entropy_bench.py (64 x 4K 4:2:0 frames per batch).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ent}
shift
SLIST=${@:-1024 2048 4096}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for S in $SLIST; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$S -o ent -- python3 $R/tools/entropy_bench.py --frames 64 --reps 3 --sub-bits $S > $O/kt_$S.json 2> $O/kt_$S.err || { echo PROF FAILED $S; tail $O/kt_$S.err; exit 1; }
  echo "== S=$S"; cat $O/kt_$S.json
  find $O/kt_$S -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1,2,4 | grep -v fillBuffer
done
