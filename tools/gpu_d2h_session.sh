set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/d2h1
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py tests/test_dropin.py -x -q -m gpu > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --workload stream4k420_d2h --steps 3 --warmup 1 > $O/d2h.json 2> $O/d2h.err || { echo D2H FAILED; tail -20 $O/d2h.err; exit 1; }
cat $O/d2h.json
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
