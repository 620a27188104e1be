#!/bin/bash
# Round 4 session prologue (VERDICT r3 "Next" #1): the pixel bench on whatever
# box this is (autotuned launch, same-run stages, box ceiling, clock), and --
# if its 4:2:0 line shows the slow-box drop (frac <= 0.79) -- the slow-box
# capture in the same session: box probe (rw-mix rates incl. write-only),
# tasks-per-wave x store-policy sweep of the product and its memory-only
# variant, TCC write / DRAM-credit counters, smi under load, kernel trace.
# Usage: tools/gpu_r04_prologue.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04p}
mkdir -p $O
cd $R
timeout -k 10 600 python -u bench.py --no-stream --no-cpu --no-fhd > $O/bench_quick.json 2> $O/bench_quick.err \
    || { echo QUICK BENCH FAILED; tail -20 $O/bench_quick.err; exit 1; }
SLOW=$(python3 - $O/bench_quick.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d["config4_444"]
for n, x in (("420", d), ("444", c)):
    r = x["roofline"]
    print(n, x["value"], "frac", r["frac"], "ceiling", r.get("box_ceiling_GBps"), r.get("frac_of_box_ceiling"),
          "clock", (x.get("clock_under_load") or {}).get("sclk_GHz_median"), "launch", (x.get("launch") or {}).get("tasks_per_wave"),
          (x.get("launch") or {}).get("stores"), "memonly_ms", (x.get("stages") or {}).get("memory_only_ms"),
          "prod_ms", (x.get("stages") or {}).get("product_ms"), file=sys.stderr)
print("box", d["box"], file=sys.stderr)
print(1 if d["roofline"]["frac"] <= 0.79 else 0)
PY
)
if [ "$SLOW" = "1" ]; then
  echo "SLOW BOX: capturing"
  timeout -k 10 300 python -u tools/box_probe.py > $O/slow_box_probe.json 2> $O/slow_box_probe.err || { echo BOXPROBE FAILED; exit 1; }
  ( for i in $(seq 1 120); do date +%s.%N; rocm-smi --showclocks --showpower --showtemp --json 2>/dev/null; sleep 0.3; done ) > $O/slow_smi_under_load.txt 2>&1 &
  SMI=$!
  timeout -k 10 600 python -u tools/tune.py --workload 4k420 --frames 256 --rounds 3 --variants 0,1 \
      --grids 259200,129600,64800,32400 --stages 0,80 > $O/slow_tune_420.json 2> $O/slow_tune_420.err
  RC=$?
  kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
  [ $RC -eq 0 ] || { echo SLOW TUNE FAILED; tail $O/slow_tune_420.err; exit 1; }
  timeout -k 10 600 python -u tools/tune.py --workload 4k444 --frames 256 --rounds 2 --variants 0,1 \
      --grids 259200,129600,64800,32400 --stages 0,80 > $O/slow_tune_444.json 2> $O/slow_tune_444.err || { echo SLOW TUNE444 FAILED; exit 1; }
  python3 - $O <<'PY'
import json, sys
for wl in ("420", "444"):
    d = json.load(open(f"{sys.argv[1]}/slow_tune_{wl}.json"))
    for r in d["results"]:
        print("slow", wl, "var", r["variant"], "grid", r["grid"], "st", r["stages"], r["median_ms"], r["GBps_median"])
PY
  cd /tmp && export TMPDIR=/tmp
  timeout -s KILL 180 rocprofv3 -i $R/tools/pmc_tcc_write.txt --output-format csv -d $O/slow_tcc -o tcc -- \
      python3 $R/bench.py --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream --no-stages --no-fhd --no-autotune > $O/slow_tcc.json 2> $O/slow_tcc.err || { echo "TCC pass failed"; tail -5 $O/slow_tcc.err; }
  for p in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $p --output-format csv -d $O/slow_pmc_$p -o pmc -- \
        python3 $R/bench.py --frames 256 --steps 3 --warmup 1 --no-cpu --no-stream --no-stages --no-fhd --no-autotune > $O/slow_pmc_$p.json 2> $O/slow_pmc_$p.err || { echo "PMC $p failed"; tail -5 $O/slow_pmc_$p.err; }
  done
  timeout -k 10 300 rocprofv3 -i $R/tools/pmc_pixel.txt --output-format csv -d $O/slow_sq_4k420 -o px -- \
      python3 $R/bench.py --workload 4k420 --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream --no-stages --no-444 --no-fhd --no-autotune > $O/slow_sq_4k420.json 2> $O/slow_sq_4k420.err || { echo "SQ pass failed"; tail -5 $O/slow_sq_4k420.err; }
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/slow_kt -o bench -- \
      python3 $R/bench.py --no-stream --no-cpu --no-fhd > $O/slow_kt_bench.json 2> $O/slow_kt_bench.err || { echo KTRACE FAILED; exit 1; }
  cd $R
  echo "slow-box capture done"
fi
exit 0
