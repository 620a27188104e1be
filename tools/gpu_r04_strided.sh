#!/bin/bash
# Round 4: the strided task order (hjd::kVarStrided) against the default
# chunked order, product and memory-only variant, same process, interleaved;
# parity of the strided kernels on the kernel tests.  Usage: <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04d}
mkdir -p $O
cd $R
timeout -k 10 600 python -u tools/tune.py --workload 4k444 --frames 256 --rounds 3 --variants 0,4 \
    --grids 0,512,768 --stages 0,80 > $O/str_444.json 2> $O/str_444.err \
    || { echo TUNE444 FAILED; tail -20 $O/str_444.err; exit 1; }
timeout -k 10 600 python -u tools/tune.py --workload 4k420 --frames 256 --rounds 3 --variants 0,4 \
    --grids 0,512,768 --stages 0,80 > $O/str_420.json 2> $O/str_420.err \
    || { echo TUNE420 FAILED; tail -20 $O/str_420.err; exit 1; }
python3 - $O <<'PY'
import json, sys
for wl in ("444", "420"):
    d = json.load(open(f"{sys.argv[1]}/str_{wl}.json"))
    for r in d["results"]:
        print(wl, "var", r["variant"], "grid", r["grid"], "st", r["stages"], r["median_ms"], r["GBps_median"])
PY
HJD_ORDER=strided timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
    tests/test_gpu_kernels.py tests/test_gpu_batch_scale.py tests/test_gpu_parity.py -m gpu > $O/tests_strided.log 2>&1 \
    || { echo STRIDED TESTS FAILED; tail -30 $O/tests_strided.log; exit 1; }
tail -1 $O/tests_strided.log
