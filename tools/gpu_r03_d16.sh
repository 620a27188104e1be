#!/bin/bash
# d16-gather session: hardware probe, full GPU suite on the HJD_D16 library,
# then a same-box A/B of the base and d16 libraries (tuning).
set -u
R=$GRAFT_REPO_ROOT
T=${1:-r03d16}
O=$R/gpurun_out/$T
mkdir -p $O
cd $R
timeout -k 10 60 ./build/d16_probe > $O/probe.txt 2>&1 || { cat $O/probe.txt; echo PROBE FAILED; exit 1; }
cat $O/probe.txt
HJD_LIB=build/variants/d16/libhjd.so timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 \
    --timeout-method thread > $O/tests_d16.log 2>&1 || { tail -30 $O/tests_d16.log; echo TESTS FAILED; exit 1; }
tail -1 $O/tests_d16.log
bash tools/gpu_r03_ab3.sh $T/ab base d16
