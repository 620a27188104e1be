#!/bin/bash
# Round-3 ablation of the fused kernel (tuning-only library, wrong outputs by
# design) plus SQ counters of the product kernel: where 4:4:4's time goes.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03abl}
mkdir -p $O
cd $R
for wl in 4k444 4k420; do
  HJD_LIB=$R/build/ablation/libhjd.so timeout -k 10 300 python tools/tune.py --workload $wl --frames 256 --rounds 5 --variants 0,4,16,20,64,80 --no-check > $O/abl_$wl.json 2> $O/abl_$wl.err || { echo ABL FAILED; tail $O/abl_$wl.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/abl_$wl.json'))
print('$wl', [(r['variant'], r['median_ms'], r['GBps_median']) for r in d['results']])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 -i $R/tools/pmc_pixel.txt --output-format csv -d $O/pmc444 -o px -- python3 $R/bench.py --workload 4k444 --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream > $O/pmc444.json 2> $O/pmc444.err || { echo PMC FAILED; tail $O/pmc444.err; exit 1; }
python3 $R/tools/pmc_pixel_summary.py $O/pmc444
