#!/bin/bash
# Tasks-per-wave sweep of the non-default samplings/formats (same box).
set -u
T=${1:-r03tpw}
for wl in 4kgray 4k422 4k440 4k411 4k420_i32 4k444_i32; do
  bash tools/gpu_tpw_sweep.sh $T $wl "1 2 4 8 16" 2 || exit 1
done
