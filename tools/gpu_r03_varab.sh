#!/bin/bash
# One library variant (build/variants/$3): same-box A/B against the in-tree
# library, then the pixel-kernel GPU tests on the variant library.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$1
cd $R
bash tools/gpu_r03_pfab.sh $1 $2 $3 || exit 1
HJD_LIB=$R/build/variants/$3/libhjd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py \
    tests/test_gpu_batch_scale.py tests/test_gpu_extensions.py -x -q --timeout 200 --timeout-method thread > $O/variant_tests.log 2>&1 \
    || { echo VARIANT TESTS FAILED; tail -30 $O/variant_tests.log; exit 1; }
tail -1 $O/variant_tests.log
