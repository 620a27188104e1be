#!/bin/bash
# Branch-light sync step: entropy GPU tests on the new library, latency A/B and kernel traces, stream-batch sync kernel A/B.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03syncstep}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_entropy.py tests/test_gpu_entropy_spec.py tests/test_gpu_multiscan.py tests/test_gpu_destuff.py tests/test_stream.py -x > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
bash tools/gpu_r03_chainab.sh ${O##*/}_lat prev new 2>&1 | grep -vE "passed"
cd /tmp && export TMPDIR=/tmp
for v in prev new; do
  HJD_LIB=$R/build/variants/$v/libhjd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktstream_$v -o st -- \
      python3 $R/bench.py --workload stream4k420 --no-cpu --steps 3 --warmup 1 > $O/ktstream_$v.json 2> $O/ktstream_$v.err || { echo KT FAILED; tail $O/ktstream_$v.err; exit 1; }
  echo "== stream $v"; grep -E "sync_k|write_k|link_k|steps_k" $O/ktstream_$v/st_kernel_stats.csv | cut -d, -f1,2,4
done
