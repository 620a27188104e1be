#!/bin/bash
# Isolated (one batch at a time) kernel times of the GPU-entropy decode of 48 4K
# frames, pinned inputs: GPU destuff vs host destuff (HJD_DESTUFF=host).
set -e
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for mode in auto host; do
  HJD_DESTUFF=$mode timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/iso_$mode -o run -- \
    python3 tools/entropy_bench.py --frames 48 --reps 10 --pixels --pinned > gpurun_out/iso_$mode.json 2> gpurun_out/iso_$mode.err
  cat gpurun_out/iso_$mode.json
done
