#!/bin/bash
# Round-4 quick check of a kernel change: the kernel parity tests (files in
# $TESTS, default the kernel/parity/extension/batch files), then the pixel
# bench (4:2:0 + 4:4:4 with same-run stages and box ceiling).
# Usage: tools/gpu_r04_quick.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04q}
T=${TESTS:-tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_extensions.py tests/test_gpu_batch_scale.py}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread $T -m gpu > $O/tests.log 2>&1 \
    || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --no-stream --no-cpu --no-fhd > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail -20 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("box", d["box"].get("serial"))
for n, x in (("420", d), ("444", d["config4_444"])):
    s = x["stages"]; r = x["roofline"]
    print(n, "frac", r["frac"], "of_box", r.get("frac_of_box_ceiling"), "prod", s["product_ms"], "memonly", s["memory_only_ms"],
          "nostore", s["no_stores_ms"], "launch", x.get("launch"), "clock", (x.get("clock_under_load") or {}).get("sclk_GHz_median"))
PY
