#!/bin/bash
# Round-2 profile set of the current build (run via gpurun from the repo root):
#   1. pixel kernel, 4k420 + 4k444 bench commands: rocprofv3 kernel trace + stats,
#      then the HBM PMC passes (tools/pmc_traffic.txt, FETCH_SIZE / WRITE_SIZE separately);
#   2. pixel kernel SQ counters (tools/pmc_pixel.txt) on 256-frame batches;
#   3. entropy kernels: kernel trace + SQ passes (tools/pmc_entropy.txt) on 48-frame
#      4K batches (the stream's batch size, S = 4096 default);
#   4. config-5 stream kernel trace.
# Usage: tools/gpu_r02_profile.sh TAG [skip-pixel]
set -u
TAG=${1:-r02prof}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
if [ "${2:-}" != "skip-pixel" ]; then
for wl in 4k420 4k444; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_$wl -o bench -- \
      python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-cpu --no-stream > $O/ktrace_$wl.json 2> $O/ktrace_$wl.err || { echo KTRACE $wl FAILED; tail $O/ktrace_$wl.err; exit 1; }
  echo "ktrace $wl ok"
  timeout -k 10 900 rocprofv3 -i $R/tools/pmc_traffic.txt --output-format csv -d $O/pmc_$wl -o pmc -- \
      python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-stream > $O/pmc_$wl.json 2> $O/pmc_$wl.err || { echo PMC $wl FAILED; tail $O/pmc_$wl.err; exit 1; }
  echo "pmc $wl ok"
  timeout -k 10 600 rocprofv3 -i $R/tools/pmc_pixel.txt --output-format csv -d $O/sq_$wl -o px -- \
      python3 $R/bench.py --workload $wl --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream > $O/sq_$wl.json 2> $O/sq_$wl.err || { echo SQ $wl FAILED; tail $O/sq_$wl.err; exit 1; }
  python3 $R/tools/pmc_pixel_summary.py $O/sq_$wl > $O/sq_$wl.txt; cat $O/sq_$wl.txt
done
fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ent_kt -o ent -- \
    python3 $R/tools/entropy_bench.py --frames 48 --reps 5 --pinned > $O/ent_kt.json 2> $O/ent_kt.err || { echo ENT KT FAILED; tail $O/ent_kt.err; exit 1; }
cat $O/ent_kt.json
timeout -k 10 600 rocprofv3 -i $R/tools/pmc_entropy.txt --output-format csv -d $O/ent_pmc -o ent -- \
    python3 $R/tools/entropy_bench.py --frames 48 --reps 1 --pinned > $O/ent_pmc.json 2> $O/ent_pmc.err || { echo ENT PMC FAILED; tail -20 $O/ent_pmc.err; exit 1; }
python3 $R/tools/pmc_entropy_summary.py $O/ent_pmc > $O/ent_pmc.txt; cat $O/ent_pmc.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stream_kt -o stream -- \
    python3 $R/bench.py --workload stream4k420 --steps 3 --warmup 1 --no-cpu --no-stream > $O/stream_kt.json 2> $O/stream_kt.err || { echo STREAM KT FAILED; tail $O/stream_kt.err; exit 1; }
echo "profile $TAG done"
