#!/bin/bash
# A/B of pixel-kernel library variants on one box (tuning only): bench.py for
# the default library and each build/variants/<name>, alternated ROUNDS times.
# Usage: gpu_pixel_ab.sh TAG ROUNDS name...
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-pxab}
N=${2:-2}
shift 2
mkdir -p $O
cd $R
for i in $(seq 1 $N); do
  for V in default "$@"; do
    # a variant is either build/variants/<name>/libhjd.so (same Python package)
    # or a snapshot build/variants/<name>/{bench.py,ocljpegdecoder_amd/} of an
    # older tree, run with its own bench and package
    B=bench.py; LIBV=""
    if [ "$V" != default ]; then
      if [ -f $R/build/variants/$V/bench.py ]; then B=$R/build/variants/$V/bench.py; else LIBV=$R/build/variants/$V/libhjd.so; fi
    fi
    for wl in 4k444 4k420; do
      HJD_LIB=$LIBV timeout -k 10 300 python $B --workload $wl --no-cpu > $O/${V}_${wl}_$i.json 2> $O/${V}_${wl}_$i.err || { echo BENCH FAILED $V $wl; tail $O/${V}_${wl}_$i.err; exit 1; }
      python3 -c "import json; d=json.load(open('$O/${V}_${wl}_$i.json')); print('$V', '$wl', $i, d['value'], d['roofline']['frac'])"
    done
  done
done
