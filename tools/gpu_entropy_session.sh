set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ent1
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python tools/entropy_bench.py --frames 16 --reps 10 > $O/bench_coefs.json 2> $O/bench_coefs.err || { echo BENCH FAILED; tail $O/bench_coefs.err; exit 1; }
cat $O/bench_coefs.json
timeout -k 10 300 python tools/entropy_bench.py --frames 16 --reps 10 --pixels > $O/bench_px.json 2> $O/bench_px.err || { echo BENCH2 FAILED; exit 1; }
cat $O/bench_px.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o ent -- python3 $R/tools/entropy_bench.py --frames 16 --reps 5 > $O/ktrace.json 2> $O/ktrace.err || { echo PROF FAILED; exit 1; }
find $O/ktrace -name "*kernel_stats.csv" -exec cat {} \;
