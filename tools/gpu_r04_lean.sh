#!/bin/bash
# Round 4: lean wave start (host-computed task split, q tables beside the
# first prefetch) against the HEAD library (build/variants/base), alternating
# processes on one box, tasks-per-wave sweeps of product + memory-only.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04f}
mkdir -p $O
cd $R
bash tools/gpu_r04_prologue.sh ${1:-r04f} || exit 1
for rep in 1 2; do
  for lib in base new; do
    if [ $lib = base ]; then export HJD_LIB=$R/build/variants/base/libhjd.so; else unset HJD_LIB; fi
    timeout -k 10 300 python -u tools/tune.py --workload 4k444 --frames 256 --rounds 2 --variants 0 \
        --grids 259200,129600,64800,32400 --stages 0,80 > $O/lean_444_${lib}_$rep.json 2> $O/lean_444_${lib}_$rep.err \
        || { echo TUNE444 $lib FAILED; tail -5 $O/lean_444_${lib}_$rep.err; exit 1; }
    timeout -k 10 300 python -u tools/tune.py --workload 4k420 --frames 256 --rounds 2 --variants 0 \
        --grids 259200,129600,64800 --stages 0,80 > $O/lean_420_${lib}_$rep.json 2> $O/lean_420_${lib}_$rep.err \
        || { echo TUNE420 $lib FAILED; tail -5 $O/lean_420_${lib}_$rep.err; exit 1; }
  done
done
unset HJD_LIB
python3 - $O <<'PY'
import json, sys, glob, collections
res = collections.defaultdict(list)
for p in sorted(glob.glob(f"{sys.argv[1]}/lean_*_*.json")):
    parts = p.rsplit("/", 1)[1][:-5].split("_")
    wl, lib = parts[1], parts[2]
    for r in json.load(open(p))["results"]:
        res[(wl, r["grid"], r["stages"], lib)].append(r["median_ms"])
for k in sorted(res):
    print(*k, res[k])
PY
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_batch_scale.py -m gpu > $O/tests.log 2>&1 \
    || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
