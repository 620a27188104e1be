#!/bin/bash
# Round 4: address-translation counters of the pixel kernels on buffers that
# run fast and slow (tools/alloc_var.py: fresh allocations in one process).
# Usage: tools/gpu_r04_tlb.sh <tag>
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r04v}
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/alloc_var.py --workload 4k444 --allocs 4 > $O/alloc_plain.json 2> $O/alloc_plain.err || { echo ALLOC FAILED; exit 1; }
cd /tmp && export TMPDIR=/tmp
for wl in 4k444 4k420; do
  timeout -s KILL 240 rocprofv3 -i $R/tools/pmc_tlb.txt --output-format csv -d $O/tlb_$wl -o tlb -- \
      python3 $R/tools/alloc_var.py --workload $wl --allocs 4 > $O/tlb_$wl.json 2> $O/tlb_$wl.err \
      || { echo "TLB pass $wl failed"; tail -5 $O/tlb_$wl.err; exit 1; }
done
echo done
