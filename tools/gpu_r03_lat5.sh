#!/bin/bash
# Config-1 latency with the current defaults: bench line + kernel trace.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03lat5}
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/fhd.json 2> $O/fhd.err || { echo FHD FAILED; tail $O/fhd.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d.get('latency_ms_per_image'), d['output_checked_vs_oracle'], {k: v for k, v in d.items() if 'latency' in k or 'pinned' in k})" $O/fhd.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d $O/kt -o fhd -- \
    python3 $R/bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/kt.json 2> $O/kt.err || { echo KT FAILED; tail $O/kt.err; exit 1; }
echo done
