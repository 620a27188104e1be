#!/bin/bash
# Config-1 latency over S (HJD_SUB_BITS) and the spec lead-in (HJD_SPEC_LEAD), interleaved.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03latsweep}
mkdir -p $O
cd $R
for rep in 1 2; do
  for cfg in 512:512 384:512 448:448 384:384 640:512; do
    s=${cfg%%:*}; l=${cfg##*:}
    HJD_SUB_BITS=$s HJD_SPEC_LEAD=$l timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/s${s}_l${l}_$rep.json 2> $O/s${s}_l${l}_$rep.err || { echo $cfg FAILED; tail $O/s${s}_l${l}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); l=d['latency_ms_per_image']; print(sys.argv[2], l['gpu_huffman_pageable_bytes'], l['gpu_huffman_pinned_bytes_device_destuff'], d['output_checked_vs_oracle'])" $O/s${s}_l${l}_$rep.json "S=$s lead=$l"
  done
done
