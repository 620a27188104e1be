#!/bin/bash
set -u
R=$GRAFT_REPO_ROOT
bash $R/tools/gpu_full_check.sh r02s5_full3 || exit 1
O=$R/gpurun_out/r02s5_prof2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for wl in 4k420 4k444; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace_$wl -o bench -- \
      python3 $R/bench.py --workload $wl --steps 10 --warmup 2 --no-cpu --no-stream > $O/ktrace_$wl.json 2> $O/ktrace_$wl.err || { echo KTRACE $wl FAILED; exit 1; }
  timeout -k 10 900 rocprofv3 -i $R/tools/pmc_traffic.txt --output-format csv -d $O/pmc_$wl -o pmc -- \
      python3 $R/bench.py --workload $wl --steps 3 --warmup 1 --no-cpu --no-stream > $O/pmc_$wl.json 2> $O/pmc_$wl.err || { echo PMC $wl FAILED; exit 1; }
  timeout -k 10 600 rocprofv3 -i $R/tools/pmc_pixel.txt --output-format csv -d $O/sq_$wl -o px -- \
      python3 $R/bench.py --workload $wl --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream > $O/sq_$wl.json 2> $O/sq_$wl.err || { echo SQ $wl FAILED; exit 1; }
  python3 $R/tools/pmc_pixel_summary.py $O/sq_$wl > $O/sq_$wl.txt; cat $O/sq_$wl.txt
done
echo prof done
