#!/bin/bash
# Chain-kernel variant A/B: spec tests on the variant, latency A/B, kernel traces.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03chainab}
shift
mkdir -p $O
cd $R
for v in "$@"; do
  HJD_LIB=build/variants/$v/libhjd.so timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_entropy_spec.py tests/test_gpu_multiscan.py -x > $O/tests_$v.log 2>&1 || { echo TESTS $v FAILED; tail -30 $O/tests_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/tests_$v.log)"
done
bash tools/gpu_r03_latab.sh ${O##*/}_lat "$@"
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  HJD_LIB=$R/build/variants/$v/libhjd.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$v -o fhd -- \
      python3 $R/bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/kt_$v.json 2> $O/kt_$v.err || { echo KT FAILED; tail $O/kt_$v.err; exit 1; }
  echo "== $v"; grep -E "chain|cand|spec_k|write_k" $O/kt_$v/fhd_kernel_stats.csv | cut -d, -f1,4
done
