#!/bin/bash
# Chain-kernel change: speculative-sync GPU tests, then config-1 latency + kernel trace.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03chain}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_gpu_entropy_spec.py tests/test_gpu_multiscan.py -x > $O/tests.log 2>&1 || { echo SPEC TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/fhd_$rep.json 2> $O/fhd_$rep.err || { echo FHD FAILED; tail $O/fhd_$rep.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d.get('latency_ms_per_image'), d['output_checked_vs_oracle'])" $O/fhd_$rep.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o fhd -- \
    python3 $R/bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/kt.json 2> $O/kt.err || { echo KT FAILED; tail $O/kt.err; exit 1; }
cut -d, -f1-4 $O/kt/fhd_kernel_stats.csv | head -6
