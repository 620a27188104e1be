#!/bin/bash
# 4:4:4 split-colour variant (HJD_SPLIT444): same-box A/B against the in-tree
# library, then the pixel-kernel GPU tests on the variant library.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03split}
cd $R
bash tools/gpu_r03_pfab.sh ${1:-r03split} 3 split || exit 1
HJD_LIB=$R/build/variants/split/libhjd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py \
    tests/test_gpu_batch_scale.py -x -q --timeout 200 --timeout-method thread > $O/split_tests.log 2>&1 \
    || { echo SPLIT TESTS FAILED; tail -30 $O/split_tests.log; exit 1; }
tail -1 $O/split_tests.log
