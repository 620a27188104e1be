#!/bin/bash
# Same-box A/B of library variants on the pixel kernel (tuning tool):
#   tools/gpu_r03_pfab.sh TAG ROUNDS VARIANT...
# Each round runs tools/tune.py (256 frames, outputs checked) on the in-tree
# library and on each build/variants/<VARIANT>/libhjd.so, 4:4:4 then 4:2:0,
# one process per run, so variants interleave in time.
set -u
TAG=${1:-ab}; N=${2:-2}; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  for V in default "$@"; do
    LIBV=""; [ "$V" != default ] && LIBV=$R/build/variants/$V/libhjd.so
    for wl in 4k444 4k420; do
      HJD_LIB=$LIBV timeout -k 10 180 python tools/tune.py --workload $wl --frames 256 --variants 0 --rounds 5 --reps 1 \
          > $O/${V}_${wl}_$i.json 2> $O/${V}_${wl}_$i.err || { echo RUN FAILED $V $wl; tail $O/${V}_${wl}_$i.err; exit 1; }
      python3 -c "import json; r=json.load(open('$O/${V}_${wl}_$i.json'))['results'][0]; print('$V $wl $i', r['median_ms'], r['GBps_median'], json.load(open('$O/${V}_${wl}_$i.json'))['signature'])"
    done
  done
done
