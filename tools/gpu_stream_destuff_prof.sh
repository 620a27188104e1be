#!/bin/bash
# rocprof kernel + memory-copy trace of the config-5 stream, pinned pool (GPU destuff) vs pageable (host destuff)
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for pin in 1 0; do
  HJD_STREAM_PINNED=$pin timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_pin$pin -o run -- python3 bench.py --workload stream4k420 --steps 2 --warmup 1 --frames 480 > gpurun_out/prof_pin$pin.json 2> gpurun_out/prof_pin$pin.err
  find gpurun_out/prof_pin$pin -name "*stats.csv" | head
done
