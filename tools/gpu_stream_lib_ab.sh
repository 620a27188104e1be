#!/bin/bash
# Same-box A/B of libhjd.so builds on the config-5 stream and the entropy kernels:
#   tools/gpu_stream_lib_ab.sh TAG "NAME=LIB ..." [ROUNDS]
# LIB "intree" = the in-tree library.  The GPU entropy tests run on the in-tree
# library first; then per round and library: entropy_bench (48 pinned 4K frames,
# S = 8192) and one bench.py stream run.
set -u
TAG=$1; LIBS=$2; ROUNDS=${3:-2}
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests/test_gpu_entropy.py tests/test_stream.py tests/test_gpu_destuff.py -x -q \
    --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rnd in $(seq 1 $ROUNDS); do
  for nl in $LIBS; do
    n=${nl%%=*}; l=${nl#*=}
    if [ "$l" = intree ]; then unset HJD_LIB; else export HJD_LIB=$R/$l; fi
    timeout -k 10 300 python tools/entropy_bench.py --frames 48 --reps 5 --pinned --sub-bits 8192 \
        > $O/ent_${n}_$rnd.json 2> $O/ent_${n}_$rnd.err || { echo ENT $n FAILED; tail $O/ent_${n}_$rnd.err; exit 1; }
    timeout -k 10 300 python bench.py --workload stream4k420 --steps 3 --warmup 1 --no-cpu \
        > $O/st_${n}_$rnd.json 2> $O/st_${n}_$rnd.err || { echo STREAM $n FAILED; tail $O/st_${n}_$rnd.err; exit 1; }
    python3 -c "import json,sys; e=json.load(open(sys.argv[1])); s=json.load(open(sys.argv[2])); print(sys.argv[3], 'round', sys.argv[4], 'entropy ms/batch', e['device_ms_per_batch'], 'stream', s['value'])" \
        $O/ent_${n}_$rnd.json $O/st_${n}_$rnd.json $n $rnd
  done
done
unset HJD_LIB
