#!/bin/bash
# HIP-graph probe of the launch-bound configs[1] (one FHD frame per launch).
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03graph}
mkdir -p $O
cd $R
for k in 200 20; do
  timeout -k 10 300 python tools/graph_probe.py --launches $k > $O/fhd420_k$k.json 2>> $O/probe.err \
      || { echo PROBE FAILED; tail $O/probe.err; exit 1; }
  cat $O/fhd420_k$k.json
done
