#!/bin/bash
# Round 4: physically contiguous buffers (hipDeviceMallocContiguous) against
# default ones, both shapes (tools/contig_var.py).  Usage: tools/gpu_r04_contig.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04w}
mkdir -p $O
cd $R
for wl in 4k420 4k444; do
  timeout -k 10 300 python -u tools/contig_var.py --workload $wl --allocs 3 > $O/contig_$wl.json 2> $O/contig_$wl.err \
      || { echo CONTIG $wl FAILED; tail -5 $O/contig_$wl.err; exit 1; }
done
python3 - $O <<'PY'
import json, sys, glob
for p in sorted(glob.glob(f"{sys.argv[1]}/contig_*.json")):
    d = json.load(open(p))
    print(p.rsplit("/", 1)[1], d["box"].get("serial"), json.dumps(d["summary"]))
    for a in d["allocations"]:
        print("   ", a["alloc"], a["flags"], a["rc"], a.get("coefs_addr"), a.get("out_addr"), a.get("product_ms"), a.get("memory_only_ms"))
PY
