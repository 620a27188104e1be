#!/bin/bash
# Batch-wide AC step tables: entropy GPU tests, then latency and a stream-leg A/B against the previous library.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03steps}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_entropy.py tests/test_gpu_entropy_spec.py tests/test_gpu_multiscan.py tests/test_gpu_destuff.py tests/test_stream.py -x > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_r03_latab.sh ${1:-r03steps}_lat prev steps
for rep in 1 2; do
  for v in prev steps; do
    HJD_LIB=build/variants/$v/libhjd.so timeout -k 10 300 python bench.py --workload stream4k420 --no-cpu --steps 3 --warmup 1 > $O/stream_${v}_$rep.json 2> $O/stream_${v}_$rep.err || { echo STREAM $v FAILED; tail $O/stream_${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('stream', sys.argv[2], d['value'], d.get('output_checked_vs_oracle'))" $O/stream_${v}_$rep.json $v
  done
done
