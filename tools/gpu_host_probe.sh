#!/bin/bash
# What host CPU share does a one-GPU box give us? (cpu_baseline core count, config-5 host ceiling)
echo "nproc: $(nproc)"
python3 -c "import os; print('affinity:', len(os.sched_getaffinity(0)), 'cpu_count:', os.cpu_count())"
echo "cgroup cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo n/a)"
echo "cgroup cpuset: $(cat /sys/fs/cgroup/cpuset.cpus.effective 2>/dev/null || echo n/a)"
echo "cgroup memory.max: $(cat /sys/fs/cgroup/memory.max 2>/dev/null || echo n/a)"
lscpu | grep -E "Model name|Socket|NUMA|Thread|Core"
for d in /sys/bus/pci/devices/*; do
  if [ -f $d/class ] && grep -q 0x1200 $d/class 2>/dev/null; then echo "accel $(basename $d) numa $(cat $d/numa_node)"; fi
done
free -g | head -2
