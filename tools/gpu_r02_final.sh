#!/bin/bash
# Round-2 closing run: full GPU suite, smoke, default bench (pixel line + config-5
# stream leg + CPU leg), then the entropy/stream profiles at the stream's S = 8192.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r02final}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest --timeout 300 --timeout-method thread tests/ -x -q -m gpu > $O/tests.log 2>&1 || { echo GPU TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH FAILED; tail $O/bench.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], d['roofline']['frac'], 'stream', d['config5_stream'].get('value'), d['config5_stream'].get('error'))"
timeout -k 10 600 python bench.py --workload 4k444 --no-cpu --no-stream > $O/bench444.json 2> $O/bench444.err || { echo BENCH444 FAILED; exit 1; }
python3 -c "import json; d=json.load(open('$O/bench444.json')); print('bench444', d['value'], d['roofline']['frac'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ent_kt -o ent -- \
    python3 $R/tools/entropy_bench.py --frames 48 --reps 5 --pinned --sub-bits 8192 > $O/ent_kt.json 2> $O/ent_kt.err || { echo ENT KT FAILED; tail $O/ent_kt.err; exit 1; }
timeout -k 10 600 rocprofv3 -i $R/tools/pmc_entropy.txt --output-format csv -d $O/ent_pmc -o ent -- \
    python3 $R/tools/entropy_bench.py --frames 48 --reps 1 --pinned --sub-bits 8192 > $O/ent_pmc.json 2> $O/ent_pmc.err || { echo ENT PMC FAILED; tail -20 $O/ent_pmc.err; exit 1; }
python3 $R/tools/pmc_entropy_summary.py $O/ent_pmc > $O/ent_pmc.txt; cat $O/ent_pmc.txt
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stream_kt -o stream -- \
    python3 $R/bench.py --workload stream4k420 --steps 3 --warmup 1 --no-cpu --no-stream > $O/stream_kt.json 2> $O/stream_kt.err || { echo STREAM KT FAILED; tail $O/stream_kt.err; exit 1; }
echo "final $1 done"
