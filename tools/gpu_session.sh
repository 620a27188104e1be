#!/bin/bash
# One GPU session on the gpurun box, as a list of steps (every GPU step under
# its own time limit; the session stops at the first failure):
#
#   tools/gpu_session.sh <tag> <step> [<step> ...]
#
# Output goes to gpurun_out/<tag>/ (merged back by gpurun).  Steps:
#   tests[:<pytest -k expr>]     the GPU suite (python -m pytest -m gpu), tests.log
#   smoke                        __graft_entry__.smoke(), smoke.log
#   bench[:<bench args>]         python bench.py <args> (default: the driver's
#                                command), bench.json + bench.err + bench_detail.json
#   ktrace:<workload>[:<args>]   rocprofv3 --kernel-trace --stats of bench.py
#                                --workload <workload> --no-cpu --no-stream <args>;
#                                ktrace:default traces the driver's own command (python bench.py)
#   pmc:<workload>               HBM bytes: FETCH_SIZE / WRITE_SIZE passes (tools/pmc/traffic.txt)
#   ent:<workload>[:<args>]      SQ counters of the entropy kernels (tools/pmc/entropy.txt)
#   htrace:<workload>[:<variant>]  HIP API + kernel + copy trace (no counters) of bench.py --workload
#   sq:<workload>[:<args>]       SQ counters of the fused kernel (tools/pmc/pixel.txt),
#                                256 frames at the default launch shape
#   ab:<variant>:<workload>:<rounds>[:<args>]
#                                same-box A/B: bench.py with the product library and with
#                                build/variants/<variant>/libhjd.so (HJD_LIB), interleaved
#   py:<script.py>[:<args>]      python <script.py> <args> (a tools/ measurement), py_<name>.json
# Arguments inside a step are separated by commas (e.g. bench:--steps,5).
set -u
TAG=${1:?usage: tools/gpu_session.sh <tag> <step> [<step> ...]}
shift
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/$TAG
mkdir -p "$O"
export TMPDIR=/tmp

fail() { echo "STEP FAILED: $1"; [ -f "$2" ] && tail -40 "$2"; exit 1; }

for step in "$@"; do
  IFS=: read -r kind a1 a2 a3 a4 <<< "$step"
  echo "== $step ($(date +%T))"
  case $kind in
    tests)
      K=()
      [ -n "${a1:-}" ] && K=(-k "$a1")
      (cd "$R" && timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests/ -x -m gpu \
          "${K[@]}" > "$O/tests.log" 2>&1) || fail tests "$O/tests.log"
      tail -1 "$O/tests.log" ;;
    smoke)
      (cd "$R" && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1) \
          || fail smoke "$O/smoke.log"
      tail -1 "$O/smoke.log" ;;
    bench)
      (cd "$R" && timeout -k 10 900 python -u bench.py ${a1//,/ } --detail-out "$O/bench_detail.json" \
          > "$O/bench.json" 2> "$O/bench.err") || fail bench "$O/bench.err"
      cat "$O/bench.json" ;;
    ktrace)
      # ktrace:default = the driver's own command (python bench.py), every leg
      if [ "$a1" = default ]; then BA=(); else BA=(--workload "$a1" --no-cpu --no-stream); fi
      (cd /tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/ktrace_$a1" -o bench -- \
          python3 "$R/bench.py" "${BA[@]}" ${a2//,/ } --detail-out "$O/ktrace_$a1.detail.json" \
          > "$O/ktrace_$a1.json" 2> "$O/ktrace_$a1.err") || fail ktrace "$O/ktrace_$a1.err"
      tail -c 400 "$O/ktrace_$a1.json" ;;
    pmc)
      (cd /tmp && timeout -k 10 900 rocprofv3 -i "$R/tools/pmc/traffic.txt" --output-format csv -d "$O/pmc_$a1" -o pmc -- \
          python3 "$R/bench.py" --workload "$a1" --steps 3 --warmup 1 --no-cpu --no-stream --no-stages --no-autotune \
          --no-444 --no-fhd --detail-out "$O/pmc_$a1.detail.json" > "$O/pmc_$a1.json" 2> "$O/pmc_$a1.err") \
          || fail pmc "$O/pmc_$a1.err"
      tail -c 300 "$O/pmc_$a1.json" ;;
    htrace)
      # HIP API + kernel trace of bench.py --workload <a1> (a2: a build/variants library, or product)
      if [ -n "${a2:-}" ] && [ "$a2" != product ]; then export HJD_LIB=$R/build/variants/$a2/libhjd.so; fi
      (cd /tmp && timeout -k 10 300 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --output-format csv \
          -d "$O/htrace_${a1}_${a2:-product}" -o ht -- python3 "$R/bench.py" --workload "$a1" --steps 40 --warmup 5 \
          --no-cpu > "$O/htrace_${a1}_${a2:-product}.json" 2> "$O/htrace_${a1}_${a2:-product}.err") \
          || fail htrace "$O/htrace_${a1}_${a2:-product}.err"
      unset HJD_LIB
      tail -c 300 "$O/htrace_${a1}_${a2:-product}.json" ;;
    ent)
      # SQ counters of the entropy kernels (tools/pmc/entropy.txt, two passes)
      (cd /tmp && timeout -k 10 300 rocprofv3 -i "$R/tools/pmc/entropy.txt" --output-format csv -d "$O/ent_$a1" -o ent -- \
          python3 "$R/bench.py" --workload "$a1" --steps 20 --warmup 3 --no-cpu ${a2//,/ } \
          --detail-out "$O/ent_$a1.detail.json" > "$O/ent_$a1.json" 2> "$O/ent_$a1.err") || fail ent "$O/ent_$a1.err"
      tail -c 300 "$O/ent_$a1.json" ;;
    sq)
      (cd /tmp && timeout -k 10 300 rocprofv3 -i "$R/tools/pmc/pixel.txt" --output-format csv -d "$O/sq_$a1" -o px -- \
          python3 "$R/bench.py" --workload "$a1" --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream --no-stages \
          --no-444 --no-fhd --no-autotune ${a2//,/ } --detail-out "$O/sq_$a1.detail.json" \
          > "$O/sq_$a1.json" 2> "$O/sq_$a1.err") || fail sq "$O/sq_$a1.err"
      tail -c 300 "$O/sq_$a1.json" ;;
    ab)
      V=$a1; WL=$a2; N=${a3:-3}
      for rep in $(seq 1 "$N"); do
        for lib in product "$V"; do
          if [ "$lib" = product ]; then unset HJD_LIB; else export HJD_LIB=$R/build/variants/$V/libhjd.so; fi
          (cd "$R" && timeout -k 10 600 python -u bench.py --workload "$WL" --no-cpu --no-stream --no-fhd --no-444 \
              ${a4//,/ } --detail-out "$O/ab_${WL}_${lib}_$rep.detail.json" \
              > "$O/ab_${WL}_${lib}_$rep.json" 2> "$O/ab_${WL}_${lib}_$rep.err") \
              || fail "ab $lib $rep" "$O/ab_${WL}_${lib}_$rep.err"
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], \
d['roofline']['frac'], d['roofline']['kernel_ms_per_launch'], d['output_checked_vs_oracle'])" \
              "$O/ab_${WL}_${lib}_$rep.json" "$lib" "$rep"
        done
      done
      unset HJD_LIB ;;
    py)
      NAME=$(basename "$a1" .py)
      (cd "$R" && timeout -k 10 600 python -u "$a1" ${a2//,/ } > "$O/py_$NAME.json" 2> "$O/py_$NAME.err") \
          || fail "py $a1" "$O/py_$NAME.err"
      tail -c 600 "$O/py_$NAME.json" ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done"
