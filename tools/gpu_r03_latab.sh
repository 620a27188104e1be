#!/bin/bash
# Config-1 latency A/B of library variants (build/variants/<name>), interleaved.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03latab}
shift
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for v in "$@"; do
    HJD_LIB=build/variants/$v/libhjd.so timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/${v}_$rep.json 2> $O/${v}_$rep.err || { echo $v FAILED; tail $O/${v}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); l=d['latency_ms_per_image']; print(sys.argv[2], l['gpu_huffman_pageable_bytes'], l['gpu_huffman_pinned_bytes_device_destuff'], d['output_checked_vs_oracle'])" $O/${v}_$rep.json $v
  done
done
