#!/bin/bash
# Same-box A/B of the config-5 stream leg: steps submitted back to back (new
# default) vs a drain after every step (HJD_BENCH_STEP_SYNC=1).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03ss}
mkdir -p $O
cd $R
for rep in 1 2 3; do
  for mode in 0 1; do
    HJD_BENCH_STEP_SYNC=$mode timeout -k 10 240 python bench.py --gpus 1 --workload stream4k420 --steps 40 --warmup 1 \
        --no-cpu --frames 1024 > $O/stream_sync${mode}_$rep.json 2> $O/stream_sync${mode}_$rep.err \
        || { echo "mode $mode FAILED"; tail $O/stream_sync${mode}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); e=d['end_to_end']; print(sys.argv[2], d['value'], d['ms_per_step'], e['h2d_ceiling']['frac'], e['output_checked_vs_oracle'])" \
        $O/stream_sync${mode}_$rep.json "step_sync=$mode rep $rep"
  done
done
