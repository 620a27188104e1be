#!/bin/bash
# Round-4 box survey (VERDICT r3 "Next" #1): on whatever box this call got,
# the pixel bench (same-run stages, ceiling, clock) and the L2 -> fabric write
# back-pressure of both product kernels at the default launch shape
# (--no-autotune, so boxes compare like for like), then the streaming probe.
# Usage: tools/gpu_r04_survey.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04s}
mkdir -p $O
cd $R
timeout -k 10 300 python -u bench.py --no-stream --no-cpu --no-fhd > $O/survey_bench.json 2> $O/survey_bench.err \
    || { echo QUICK BENCH FAILED; tail -20 $O/survey_bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
for wl in 4k420 4k444; do
  timeout -s KILL 180 rocprofv3 -i $R/tools/pmc_tcc_write.txt --output-format csv -d $O/tcc_$wl -o tcc -- \
      python3 $R/bench.py --workload $wl --frames 256 --steps 3 --warmup 1 --no-cpu --no-stream --no-stages --no-444 --no-fhd --no-autotune \
      > $O/tcc_$wl.json 2> $O/tcc_$wl.err || { echo "TCC $wl failed"; tail -5 $O/tcc_$wl.err; exit 1; }
done
cd $R
timeout -k 10 300 python -u tools/box_probe.py > $O/box_probe.json 2> $O/box_probe.err || { echo BOXPROBE FAILED; exit 1; }
python3 - $O <<'PY'
import json, sys, subprocess
o = sys.argv[1]
b = json.load(open(f"{o}/survey_bench.json"))
print("box", b["box"].get("serial"))
for wl, x, k, t in (("4k420", b, "decode_kernel<1,0,0>", 1036800), ("4k444", b["config4_444"], "decode_kernel<0,0,128>", 2073600)):
    s = x["stages"]
    d = json.loads(subprocess.run([sys.executable, "tools/sq_summary.py", f"{o}/tcc_{wl}", k, "--tasks-per-dispatch", str(t)],
                                  capture_output=True, text=True).stdout)
    dv = d["derived"]
    print(wl, "frac", x["roofline"]["frac"], "memonly", s["memory_only_ms"], "prod", s["product_ms"],
          "wr_credit_stall/cyc", dv.get("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_per_cycle"),
          "rd_credit_stall/cyc", dv.get("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_per_cycle"), "clk", dv.get("effective_clock_GHz"))
p = json.load(open(f"{o}/box_probe.json"))
print("probe", p.get("best_GBps_nt_xcd"))
PY
