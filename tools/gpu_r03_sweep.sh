#!/bin/bash
# Round-3 closing sweep of the non-default workloads (extensions, idct.h int32
# format, config 1, stream variants) on the final build, one process each.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03sw}
mkdir -p $O
cd $R
for wl in 4k422 4kgray 4k411 4k440 4k420_bgr24 4k420_i32 4k444_i32 fhd420; do
  timeout -k 10 300 python bench.py --workload $wl --steps 10 --warmup 2 --no-cpu --no-stream > $O/$wl.json 2> $O/$wl.err \
      || { echo "$wl FAILED"; tail $O/$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline') or {}; print(sys.argv[2], d['value'], r.get('frac'), d['ms_per_step'], d.get('output_checked_vs_oracle'))" $O/$wl.json $wl
done
timeout -k 10 300 python bench.py --workload fhd420_jpeg --steps 50 --warmup 5 --no-cpu > $O/fhd420_jpeg.json 2> $O/fhd420_jpeg.err \
    || { echo "fhd420_jpeg FAILED"; tail $O/fhd420_jpeg.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/fhd420_jpeg.json')); print('fhd420_jpeg', d['latency_ms_per_image'], d['output_checked_vs_oracle'])"
for wl in stream4k420_d2h stream4k420_d2h_bgr24 stream4k420_host; do
  timeout -k 10 300 python bench.py --workload $wl --steps 8 --warmup 1 --no-cpu > $O/$wl.json 2> $O/$wl.err \
      || { echo "$wl FAILED"; tail $O/$wl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['end_to_end']['output_checked_vs_oracle'])" $O/$wl.json $wl
done
