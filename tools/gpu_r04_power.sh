#!/bin/bash
# Round-4 study of run-to-run spread against board power: three processes of
# tools/power_var.py on 4:4:4 (product and memory-only variant alternating,
# hwmon power sampled), one on 4:2:0.  Usage: tools/gpu_r04_power.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04p}
mkdir -p $O
cd $R
for i in 1 2 3; do
  timeout -k 10 240 python -u tools/power_var.py --workload 4k444 --rounds 40 --reps 20 > $O/power_4k444_$i.json 2> $O/power_4k444_$i.err \
      || { echo POWER 4k444 $i FAILED; tail -5 $O/power_4k444_$i.err; exit 1; }
done
timeout -k 10 240 python -u tools/power_var.py --workload 4k420 --rounds 40 --reps 20 > $O/power_4k420_1.json 2> $O/power_4k420_1.err \
    || { echo POWER 4k420 FAILED; tail -5 $O/power_4k420_1.err; exit 1; }
python3 - $O <<'PY'
import json, sys, glob
for p in sorted(glob.glob(f"{sys.argv[1]}/power_*.json")):
    d = json.load(open(p))
    print(p.rsplit("/", 1)[1], d["box"].get("serial"), "hwmon", sorted(d["hwmon"]))
    for k, v in d["summary"].items():
        print("  ", k, v["ms_min"], v["ms_median"], v["ms_max"], v["spread_pct"], "fast", v["fastest"], "slow", v["slowest"])
PY
