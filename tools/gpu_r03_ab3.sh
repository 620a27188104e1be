#!/bin/bash
# Same-box A/B/C of pixel-kernel libraries under build/variants (tuning).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03ab3}
shift
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for wl in 4k444 4k420; do
    for v in "$@"; do
      HJD_LIB=build/variants/$v/libhjd.so timeout -k 10 300 python bench.py --workload $wl --no-cpu --no-stream --no-444 --frames 512 > $O/${wl}_${v}_$rep.json 2> $O/${wl}_${v}_$rep.err || { echo $v FAILED; tail $O/${wl}_${v}_$rep.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms_per_launch'], d['output_checked_vs_oracle'])" $O/${wl}_${v}_$rep.json "$wl $v"
    done
  done
done
