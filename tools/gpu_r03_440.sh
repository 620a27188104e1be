#!/bin/bash
# 4:4:0 colour stage with shared chroma rows: extension GPU tests, then a
# same-box A/B against the previous library (build/variants/base), 3 rounds.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03_440}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_extensions.py tests/test_gpu_kernels.py tests/test_gpu_parity.py -x -q \
    --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; echo TESTS FAILED; exit 1; }
tail -1 $O/tests.log
for rnd in 1 2 3; do
  for lib in base new; do
    if [ $lib = base ]; then export HJD_LIB=build/variants/base/libhjd.so; else unset HJD_LIB; fi
    timeout -k 10 300 python bench.py --workload 4k440 --no-cpu --no-stream > $O/${lib}_$rnd.json 2> $O/${lib}_$rnd.err \
        || { echo "$lib FAILED"; tail $O/${lib}_$rnd.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['output_checked_vs_oracle'])" $O/${lib}_$rnd.json "$lib $rnd"
  done
done
unset HJD_LIB
