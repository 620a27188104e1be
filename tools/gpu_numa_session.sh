set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/numa1
mkdir -p $O
cd $R
cat /sys/bus/pci/devices/*/numa_node 2>/dev/null | sort | uniq -c | head; nproc; python3 -c "import os; print(len(os.sched_getaffinity(0)))"
timeout -k 10 900 python -m pytest tests/test_gpu_entropy.py tests/test_stream.py -x -q > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 600 python bench.py --workload stream4k420 --steps 3 --warmup 1 > $O/s_numa.json 2> $O/s_numa.err || { echo S1 FAILED; exit 1; }
HJD_NUMA=0 timeout -k 10 600 python bench.py --workload stream4k420 --steps 3 --warmup 1 > $O/s_nonuma.json 2> $O/s_nonuma.err || { echo S2 FAILED; exit 1; }
python3 -c "
import json
for f in ('s_numa', 's_nonuma'):
    d = json.load(open('$O/' + f + '.json')); print(f, d['value'], d['end_to_end'])"
