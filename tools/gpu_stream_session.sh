#!/bin/bash
# GPU session: entropy/stream parity tests, then the config-5 stream benches
# (GPU-entropy and host-Huffman) and a kernel trace of the GPU-entropy stream.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-gs}
mkdir -p $O
cd $R
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 600 python bench.py --workload stream4k420 --steps 4 --warmup 1 > $O/stream.json 2> $O/stream.err || { echo STREAM FAILED; tail -20 $O/stream.err; exit 1; }
cat $O/stream.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o stream -- python3 $R/bench.py --workload stream4k420 --steps 2 --warmup 1 > $O/kt.json 2> $O/kt.err || { echo PROF FAILED; tail $O/kt.err; exit 1; }
find $O/kt -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1,2,3,4 | grep -v fillBuffer
