#!/bin/bash
# Round 4: is the slow 4:2:0 state per allocation, per process or per box?
# Three processes of tools/alloc_var.py (five fresh allocations each) on
# 4:2:0, one on 4:4:4.  Usage: tools/gpu_r04_alloc.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04a2}
mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 300 python -u tools/alloc_var.py --workload 4k420 --allocs 5 > $O/alloc_4k420_$i.json 2> $O/alloc_4k420_$i.err \
      || { echo ALLOC 4k420 $i FAILED; tail -5 $O/alloc_4k420_$i.err; exit 1; }
done
timeout -k 10 300 python -u tools/alloc_var.py --workload 4k444 --allocs 4 > $O/alloc_4k444_1.json 2> $O/alloc_4k444_1.err \
    || { echo ALLOC 4k444 FAILED; tail -5 $O/alloc_4k444_1.err; exit 1; }
python3 - $O <<'PY'
import json, sys, glob
for p in sorted(glob.glob(f"{sys.argv[1]}/alloc_*.json")):
    d = json.load(open(p))
    print(p.rsplit("/", 1)[1], d["box"].get("serial"), "prod", d["product_ms_range"], "mem", d["memory_only_ms_range"],
          "spread", d["product_spread_pct"], d["memory_only_spread_pct"])
    for a in d["allocations"]:
        print("   ", a["alloc"], a["coefs_addr"], a["out_addr"], a["product_ms"], a["memory_only_ms"])
PY
