#!/bin/bash
# Entropy kernels: GPU tests on the in-tree library, then a same-box A/B of
# the kernel times (rocprofv3 kernel trace of tools/entropy_bench.py, 64 x 4K
# 4:2:0 frames) across library builds (HJD_LIB; "new" = the in-tree library).
#   tools/gpu_entropy_ab.sh TAG LIB...      (e.g. build/variants/base/libhjd.so)
set -u
TAG=${1:-ent_ab}; shift
LIBS="$@"
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_entropy.py tests/test_stream.py tests/test_gpu_extensions.py \
    -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
for rep in 1 2; do
  for lib in new $LIBS; do
    v=$(basename $(dirname $lib))
    if [ $lib = new ]; then v=new; unset HJD_LIB; else export HJD_LIB=$R/$lib; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_${v}_$rep -o ent -- \
        python3 $R/tools/entropy_bench.py --frames 64 --reps 3 ${EB_ARGS:-} > $O/run_${v}_$rep.json 2> $O/run_${v}_$rep.err \
        || { echo PROF $v FAILED; tail $O/run_${v}_$rep.err; exit 1; }
    echo "$v $rep: $(find $O/kt_${v}_$rep -name '*kernel_stats.csv' -exec cat {} \; | grep -E 'ent_(sync|write)' | cut -d, -f4 | tr '\n' ' ')"
  done
done
unset HJD_LIB
