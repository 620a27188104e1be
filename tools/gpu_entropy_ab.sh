#!/bin/bash
# A/B of entropy-kernel library variants (tuning only): kernel traces of
# tools/entropy_bench.py for the default library and each build/variants/<name>.
# Usage: gpu_entropy_ab.sh TAG S name...
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-ab}
S=${2:-2048}
shift 2
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for V in default "$@"; do
  if [ "$V" = default ]; then LIBV=""; else LIBV=$R/build/variants/$V/libhjd.so; fi
  HJD_LIB=$LIBV timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$V -o ent -- python3 $R/tools/entropy_bench.py --frames 64 --reps 3 --sub-bits $S > $O/kt_$V.json 2> $O/kt_$V.err || { echo PROF FAILED $V; tail $O/kt_$V.err; exit 1; }
  echo "== $V"; find $O/kt_$V -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1,4 | grep ent_
done
