#!/bin/bash
# config-5 stream A/B: host destuff (pageable pool) vs GPU destuff (pinned pool), two rounds
set -e
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
for pin in 0 1; do
  HJD_STREAM_PINNED=$pin timeout -k 10 300 python bench.py --workload stream4k420 --steps 3 --warmup 1 > gpurun_out/ab.json 2> gpurun_out/ab.err
  python3 -c "import json; d=json.load(open('gpurun_out/ab.json')); print('pinned=$pin', d['value'], d['end_to_end']['output_checked_vs_oracle'])"
done
done
