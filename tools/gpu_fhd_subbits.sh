set -u
O=$GRAFT_REPO_ROOT/gpurun_out/r02fhd2
mkdir -p $O
cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  for S in 512 1024 2048; do
    HJD_SUB_BITS=$S timeout -k 10 200 python bench.py --workload fhd420_jpeg --no-cpu --no-stream > $O/fhd_${S}_$rep.json 2> $O/fhd_${S}_$rep.err || { echo FHD $S FAILED; tail $O/fhd_${S}_$rep.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], {k: v for k, v in d.items() if 'latency' in k or 'ms' in k and k != 'ms_per_step'})" $O/fhd_${S}_$rep.json $S $rep
  done
done
