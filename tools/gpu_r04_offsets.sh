#!/bin/bash
# Round 4: memory-side time against buffer placement inside one arena
# (tools/offset_sweep.py), fine (2 MiB) and coarse (96 MiB) steps, both shapes.
# Usage: tools/gpu_r04_offsets.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04u}
mkdir -p $O
cd $R
for wl in 4k420 4k444; do
  for st in 2 96; do
    timeout -k 10 300 python -u tools/offset_sweep.py --workload $wl --step-mib $st --points 32 > $O/off_${wl}_$st.json 2> $O/off_${wl}_$st.err \
        || { echo SWEEP $wl $st FAILED; tail -5 $O/off_${wl}_$st.err; exit 1; }
  done
done
python3 - $O <<'PY'
import json, sys, glob
for p in sorted(glob.glob(f"{sys.argv[1]}/off_*.json")):
    d = json.load(open(p))
    print(p.rsplit("/", 1)[1], d["box"].get("serial"), json.dumps(d["summary"]))
    for name, rows in d["sweeps"].items():
        print("  ", name, [r["memory_only_ms"] for r in rows])
PY
