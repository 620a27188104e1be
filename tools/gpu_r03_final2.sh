#!/bin/bash
# Round-3 closing run after the stream change: bench-rank GPU tests, then the
# driver's default bench command.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03g}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_ranks.py -x -v --timeout 300 --timeout-method thread \
    > $O/bench_ranks_tests.log 2>&1 || { tail -30 $O/bench_ranks_tests.log; echo TESTS FAILED; exit 1; }
tail -1 $O/bench_ranks_tests.log
timeout -k 10 900 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err \
    || { tail -20 $O/bench.err; echo BENCH FAILED; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['roofline']['frac'], d['config4_444']['value'], d['config4_444']['roofline']['frac'], d['config5_stream']['value'], d['config5_stream']['h2d_ceiling']['frac'])"
