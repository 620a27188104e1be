#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03steps2}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_entropy.py tests/test_gpu_entropy_spec.py tests/test_gpu_multiscan.py tests/test_gpu_destuff.py tests/test_stream.py tests/test_gpu_extensions.py -x > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_r03_lat5.sh ${1:-r03steps2}_lat
cut -d, -f1-4 $O/../${1:-r03steps2}_lat/kt/fhd_kernel_stats.csv | head -8
