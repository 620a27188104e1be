#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04e}
mkdir -p $O
cd $R
bash tools/gpu_r04_prologue.sh ${1:-r04e} || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -m gpu > $O/tests_kernels.log 2>&1 \
    || { echo KERNEL TESTS FAILED; tail -30 $O/tests_kernels.log; exit 1; }
tail -1 $O/tests_kernels.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 -i $R/tools/pmc_tcc_write.txt --output-format csv -d $O/tcc -o tcc -- \
    python3 $R/bench.py --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream --no-stages --no-fhd --no-autotune > $O/tcc.json 2> $O/tcc.err || { echo "TCC pass failed"; tail -5 $O/tcc.err; }
echo session done
