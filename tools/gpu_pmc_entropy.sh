#!/bin/bash
# Entropy kernels: GPU parity tests, kernel trace (64 x 4K frames, S=2048) and
# the SQ counter passes of tools/pmc_entropy.txt (32 frames).  Usage: TAG
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pmc_ent}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o ent -- python3 $R/tools/entropy_bench.py --frames 64 --reps 3 > $O/kt.json 2> $O/kt.err || { echo PROF FAILED; tail $O/kt.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1,4 | grep ent_
timeout -k 10 600 rocprofv3 -i $R/tools/pmc_entropy.txt --output-format csv -d $O/p -o ent -- python3 $R/tools/entropy_bench.py --frames 32 --reps 1 > $O/run.json 2> $O/run.err || { echo PMC FAILED; tail -20 $O/run.err; exit 1; }
python3 $R/tools/pmc_entropy_summary.py $O/p
