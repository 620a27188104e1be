#!/bin/bash
# Round-4 box session (VERDICT r3 "Next" #1-#3): on one box, in one call --
#   box identity + d16 probe + rw-mix streaming sweep (tools/box_probe.py),
#   the pixel bench (4:2:0 + 4:4:4, same-run stages + box ceiling) with smi
#   sampled under load, its kernel trace, FETCH/WRITE PMC passes, SQ counters
#   of both kernels, and (last, may be refused by the counter set) TCC write
#   counters.  Usage: tools/gpu_r04_probe.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04a}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/box_probe.py > $O/box_probe.json 2> $O/box_probe.err \
    || { echo BOXPROBE FAILED; tail -20 $O/box_probe.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/box_probe.json'))
print('host', d['box']['hostname'], 'd16', d['d16_gather'], 'best', d['best_GBps_nt_xcd'])"
( for i in $(seq 1 200); do date +%s.%N; rocm-smi --showclocks --showpower --showtemp --json 2>/dev/null; sleep 0.5; done ) > $O/smi_under_load.txt 2>&1 &
SMI=$!
timeout -k 10 600 python -u bench.py --no-stream --no-cpu --no-fhd > $O/bench.json 2> $O/bench.err
RC=$?
kill $SMI 2>/dev/null; wait $SMI 2>/dev/null
[ $RC -eq 0 ] || { echo BENCH FAILED rc=$RC; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); c=d['config4_444']
for n, x in (('420', d), ('444', c)):
    r = x['roofline']; s = x['stages']
    print(n, x['value'], 'frac', r['frac'], 'box', r.get('box_ceiling_GBps'), r.get('frac_of_box_ceiling'),
          'memonly', s['memory_only_ms'], 'nostore', s['no_stores_ms'], 'prod', s['product_ms'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3-avail list > $O/counters_avail.txt 2>&1 || timeout -k 10 120 rocprofv3 -L > $O/counters_avail.txt 2>&1 || echo "counter list failed"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o bench -- \
    python3 $R/bench.py --no-stream --no-cpu --no-fhd > $O/kt_bench.json 2> $O/kt_bench.err || { echo KTRACE FAILED; tail -20 $O/kt_bench.err; exit 1; }
echo "ktrace done"
for p in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 600 rocprofv3 --pmc $p --output-format csv -d $O/pmc_$p -o pmc -- \
      python3 $R/bench.py --steps 3 --warmup 1 --no-cpu --no-stream --no-stages --no-fhd > $O/pmc_$p.json 2> $O/pmc_$p.err || { echo PMC $p FAILED; tail -20 $O/pmc_$p.err; exit 1; }
done
echo "pmc passes done"
for wl in 4k444 4k420; do
  timeout -k 10 600 rocprofv3 -i $R/tools/pmc_pixel.txt --output-format csv -d $O/sq_$wl -o px -- \
      python3 $R/bench.py --workload $wl --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream --no-stages --no-444 --no-fhd > $O/sq_$wl.json 2> $O/sq_$wl.err || { echo SQ $wl FAILED; tail $O/sq_$wl.err; exit 1; }
  echo "== $wl"; python3 $R/tools/pmc_pixel_summary.py $O/sq_$wl
done
timeout -s KILL 120 rocprofv3 -i $R/tools/pmc_tcc_write.txt --output-format csv -d $O/tcc -o tcc -- \
    python3 $R/bench.py --frames 256 --steps 2 --warmup 1 --no-cpu --no-stream --no-stages --no-fhd > $O/tcc.json 2> $O/tcc.err || { echo "TCC pass failed (counter names?)"; tail -5 $O/tcc.err; }
echo "session done"
