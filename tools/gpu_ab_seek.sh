set -u
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/ab_seek; mkdir -p $O; cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_kernels.py tests/test_gpu_extensions.py -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo TESTS FAILED; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in head new; do
    if [ $v = head ]; then export HJD_LIB=$R/build/variants/head/libhjd.so; else unset HJD_LIB; fi
    timeout -k 10 200 python tools/tune.py --workload 4k420 --frames 256 --variants 0 --rounds 5 --grids 0,518400,259200 > $O/${v}_420_$rep.json || exit 1
    timeout -k 10 200 python tools/tune.py --workload 4k444 --frames 256 --variants 0 --rounds 5 --grids 0,518400,259200,129600 > $O/${v}_444_$rep.json || exit 1
  done
done
unset HJD_LIB
python3 - $O <<'PY'
import glob, json, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*_4*_*.json"))):
    r = json.load(open(f))["results"]
    print(os.path.basename(f), [(x["grid"], x["GBps_median"]) for x in r])
PY
