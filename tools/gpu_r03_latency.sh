#!/bin/bash
# Round 3: the speculative sync (latency decoders) on the device -- its GPU
# tests, then config 1 end to end (bench.py --workload fhd420_jpeg) across the
# subsequence length S and the spec runs' lead-in, against the round-based sync.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03lat}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_gpu_entropy_spec.py -x -m gpu > $O/tests.log 2>&1 || { echo SPEC TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
run() {  # tag, env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/fhd_$tag.json 2> $O/fhd_$tag.err || { echo FHD $tag FAILED; tail $O/fhd_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['ms_per_step'], d['latency_ms_per_image'], d['output_checked_vs_oracle'])" $O/fhd_$tag.json $tag
}
run default
run old512 HJD_SYNC_SPEC=0 HJD_SUB_BITS=512
run old1024 HJD_SYNC_SPEC=0 HJD_SUB_BITS=1024
for S in 256 512 1024; do
  for L in 256 512 1024; do
    run s${S}_l${L} HJD_SUB_BITS=$S HJD_SPEC_LEAD=$L
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o fhd -- \
    python3 $R/bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/kt_fhd.json 2> $O/kt_fhd.err || { echo KT FAILED; tail $O/kt_fhd.err; exit 1; }
echo "latency session done"
