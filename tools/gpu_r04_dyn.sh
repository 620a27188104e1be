#!/bin/bash
# Round 4: dynamic task chunks (per-XCD counters) against static chunks,
# product + memory-only, one process per sampling; parity of every chunking.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04g}
mkdir -p $O
cd $R
bash tools/gpu_r04_prologue.sh ${1:-r04g} || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -m gpu > $O/tests_kernels.log 2>&1 \
    || { echo KERNEL TESTS FAILED; tail -30 $O/tests_kernels.log; exit 1; }
tail -1 $O/tests_kernels.log
timeout -k 10 600 python -u tools/tune.py --workload 4k444 --frames 256 --rounds 3 --variants 0 \
    --chunks s16,s4,s2,d1,d2,d4,d8 --stages 0,80 > $O/dyn_444.json 2> $O/dyn_444.err \
    || { echo TUNE444 FAILED; tail -20 $O/dyn_444.err; exit 1; }
timeout -k 10 600 python -u tools/tune.py --workload 4k420 --frames 256 --rounds 3 --variants 0 \
    --chunks s2,s1,d1,d2,d4 --stages 0,80 > $O/dyn_420.json 2> $O/dyn_420.err \
    || { echo TUNE420 FAILED; tail -20 $O/dyn_420.err; exit 1; }
python3 - $O <<'PY'
import json, sys
for wl in ("444", "420"):
    d = json.load(open(f"{sys.argv[1]}/dyn_{wl}.json"))
    for r in d["results"]:
        print(wl, r["grid"], "st", r["stages"], r["median_ms"], r["GBps_median"])
PY
