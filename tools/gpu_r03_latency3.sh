#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03lat4}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_entropy_spec.py -x -m gpu > $O/tests.log 2>&1 || { echo SPEC TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
HJD_LIB=build/variants/chainprof/libhjd.so timeout -k 10 200 python bench.py --workload fhd420_jpeg --steps 3 --warmup 1 --no-cpu --no-stream > $O/chainprof.txt 2>&1 || { echo PROF FAILED; exit 1; }
grep "chain n" $O/chainprof.txt | tail -2
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/fhd_$tag.json 2> $O/fhd_$tag.err || { echo FHD $tag FAILED; tail $O/fhd_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['latency_ms_per_image'], d['output_checked_vs_oracle'])" $O/fhd_$tag.json $tag
}
for rep in 1 2; do
  run default_$rep
  run s768_l512_$rep HJD_SUB_BITS=768
  run s512_l512_$rep HJD_SUB_BITS=512
  run s1024_l256_$rep HJD_SUB_BITS=1024 HJD_SPEC_LEAD=256
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o fhd -- \
    python3 $R/bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/kt.json 2> $O/kt.err || { echo KT FAILED; tail $O/kt.err; exit 1; }
echo "latency session 3 done"
