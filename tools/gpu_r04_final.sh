#!/bin/bash
# Round-4 closing session: the whole GPU suite, smoke, the driver's default
# bench command, then SQ counters of both product kernels at the default
# launch shape (--no-autotune, 16 / 2 tasks per wave).  Usage: tools/gpu_r04_final.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04z}
mkdir -p $O
bash $R/tools/gpu_r04_full.sh ${1:-r04z} || exit 1
cd /tmp && export TMPDIR=/tmp
for wl in 4k444 4k420; do
  timeout -k 10 300 rocprofv3 -i $R/tools/pmc_pixel.txt --output-format csv -d $O/sq_$wl -o px -- \
      python3 $R/bench.py --workload $wl --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream --no-stages --no-444 --no-fhd --no-autotune \
      > $O/sq_$wl.json 2> $O/sq_$wl.err || { echo SQ $wl FAILED; tail $O/sq_$wl.err; exit 1; }
done
echo "final session done"
