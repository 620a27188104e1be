#!/bin/bash
# GPU session for the entropy decoder: parity tests, S x batch sweep, kernel trace.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ent}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for S in 1024 2048 4096; do
  for N in 16 64; do
    timeout -k 10 300 python tools/entropy_bench.py --frames $N --reps 5 --sub-bits $S > $O/bench_S${S}_N${N}.json 2> $O/bench_S${S}_N${N}.err || { echo BENCH FAILED $S $N; tail $O/bench_S${S}_N${N}.err; exit 1; }
    cat $O/bench_S${S}_N${N}.json
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o ent -- python3 $R/tools/entropy_bench.py --frames 64 --reps 3 --sub-bits ${2:-2048} > $O/ktrace.json 2> $O/ktrace.err || { echo PROF FAILED; exit 1; }
find $O/ktrace -name "*kernel_stats.csv" -exec cat {} \;
