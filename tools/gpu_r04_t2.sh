#!/bin/bash
# Round 4: the 5-wave-per-SIMD 4:4:4 layout (HJD_T2, build/variants/t2) at
# short task chunks against the default layout, alternating processes.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04h}
mkdir -p $O
cd $R
bash tools/gpu_r04_prologue.sh ${1:-r04h} || exit 1
for rep in 1 2; do
  for lib in def t2; do
    if [ $lib = t2 ]; then export HJD_LIB=$R/build/variants/t2/libhjd.so; else unset HJD_LIB; fi
    timeout -k 10 300 python -u tools/tune.py --workload 4k444 --frames 256 --rounds 2 --variants 0 \
        --chunks s1,s2,s4,s8,s16 --stages 0 > $O/t2_444_${lib}_$rep.json 2> $O/t2_444_${lib}_$rep.err \
        || { echo TUNE $lib FAILED; tail -5 $O/t2_444_${lib}_$rep.err; exit 1; }
  done
done
unset HJD_LIB
python3 - $O <<'PY'
import json, sys, glob, collections
res = collections.defaultdict(list)
for p in sorted(glob.glob(f"{sys.argv[1]}/t2_444_*.json")):
    lib = p.rsplit("/", 1)[1].split("_")[2]
    for r in json.load(open(p))["results"]:
        res[(r["grid"], lib)].append(r["median_ms"])
for k in sorted(res):
    print(*k, res[k])
PY
