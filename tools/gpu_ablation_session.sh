#!/bin/bash
# Ablation A/B of the fused kernel (tuning-only library, wrong outputs by design).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-abl}
mkdir -p $O
cd $R
for wl in 4k444 4k420; do
  HJD_LIB=$R/build/ablation/libhjd.so timeout -k 10 600 python tools/tune.py --workload $wl --frames 256 --rounds 5 --variants 0,4,8,16,24 --no-check > $O/abl_$wl.json 2> $O/abl_$wl.err || { echo ABL FAILED; tail $O/abl_$wl.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$O/abl_$wl.json'))
print('$wl', [(r['variant'], r['median_ms'], r['GBps_median']) for r in d['results']])"
done
