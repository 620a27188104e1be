#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03lat2}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_entropy_spec.py -x -m gpu > $O/tests.log 2>&1 || { echo SPEC TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/fhd_$tag.json 2> $O/fhd_$tag.err || { echo FHD $tag FAILED; tail $O/fhd_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['latency_ms_per_image'], d['output_checked_vs_oracle'])" $O/fhd_$tag.json $tag
}
for rep in 1 2; do
  run default_$rep
  run s512_l768_$rep HJD_SPEC_LEAD=768
  run s768_l512_$rep HJD_SUB_BITS=768
  run s384_l768_$rep HJD_SUB_BITS=384 HJD_SPEC_LEAD=768
  run s1024_l256_$rep HJD_SUB_BITS=1024 HJD_SPEC_LEAD=256
done
cd /tmp && export TMPDIR=/tmp
for cfg in "spec512:HJD_SUB_BITS=512" "old1024:HJD_SYNC_SPEC=0"; do
  tag=${cfg%%:*}; ev=${cfg#*:}
  export $ev
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$tag -o fhd -- \
      python3 $R/bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/kt_$tag.json 2> $O/kt_$tag.err || { echo KT FAILED; tail $O/kt_$tag.err; exit 1; }
  unset ${ev%%=*}
done
echo "latency session 2 done"
