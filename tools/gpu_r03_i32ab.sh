#!/bin/bash
# int32 (idct.h format) cross-task prefetch: parity tests, then same-box A/B of the i32 workloads.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03i32ab}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_batch_scale.py tests/test_gpu_kernels.py tests/test_dropin.py tests/test_gpu_extensions.py -x > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for wl in 4k420_i32 4k444_i32 4k420; do
    for v in old new; do
      HJD_LIB=build/variants/$v/libhjd.so timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-stream --no-444 --frames 512 > $O/${wl}_${v}_$rep.json 2> $O/${wl}_${v}_$rep.err || { echo $v FAILED; tail $O/${wl}_${v}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_per_launch'], d['output_checked_vs_oracle'])" $O/${wl}_${v}_$rep.json "$wl $v"
    done
  done
done
