#!/bin/bash
# Multi-scan GPU entropy path: its tests, then the entropy/destuff/stream suites it touches.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03ms}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_multiscan.py -x > $O/ms.log 2>&1 || { echo MS TESTS FAILED; tail -40 $O/ms.log; exit 1; }
tail -1 $O/ms.log
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_entropy.py tests/test_gpu_destuff.py tests/test_gpu_entropy_spec.py tests/test_stream.py -x > $O/ent.log 2>&1 || { echo ENT TESTS FAILED; tail -40 $O/ent.log; exit 1; }
tail -1 $O/ent.log
