#!/bin/bash
# Same-box A/B/C... of several builds of libhjd.so on the pixel kernel (tuning):
#   tools/gpu_multi_ab.sh TAG "NAME=LIB NAME=LIB ..." WORKLOAD [WORKLOAD ...]
# LIB "intree" means the in-tree library.  Runs the pixel-kernel GPU tests on
# the in-tree library first, then tools/tune.py on every library in turn,
# 3 rounds, one process per run (256-frame batches, default grid).
set -u
TAG=$1; LIBS=$2; shift 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_extensions.py \
    -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2 3; do
  for wl in "$@"; do
    for nl in $LIBS; do
      n=${nl%%=*}; l=${nl#*=}
      if [ "$l" = intree ]; then unset HJD_LIB; else export HJD_LIB=$R/$l; fi
      timeout -k 10 240 python tools/tune.py --workload $wl --frames 256 --variants 0 --rounds 5 \
          > $O/${n}_${wl}_$rep.json 2> $O/${n}_${wl}_$rep.err || { echo RUN $n FAILED; tail $O/${n}_${wl}_$rep.err; exit 1; }
    done
  done
  echo "rep $rep done"
done
unset HJD_LIB
python3 - "$O" <<'PY'
import collections, glob, json, os, statistics, sys
o = sys.argv[1]
rows = collections.defaultdict(list)
for f in sorted(glob.glob(os.path.join(o, "*_*_*.json"))):
    n, wl, rep = os.path.basename(f)[:-5].rsplit("_", 2)
    rows[(wl, n)].append(json.load(open(f))["results"][0]["median_ms"])
for (wl, n), v in sorted(rows.items()):
    print(f"{wl} {n:10s} median {statistics.median(v):.4f} ms  runs {' '.join('%.4f' % x for x in v)}")
PY
