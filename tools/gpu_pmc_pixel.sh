#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pmc_px}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for wl in 4k444 4k420; do
  timeout -k 10 600 rocprofv3 -i $R/tools/pmc_pixel.txt --output-format csv -d $O/$wl -o px -- python3 $R/bench.py --workload $wl --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream > $O/$wl.json 2> $O/$wl.err || { echo PMC FAILED; tail $O/$wl.err; exit 1; }
  echo "== $wl"; python3 $R/tools/pmc_pixel_summary.py $O/$wl
done
