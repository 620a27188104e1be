#!/bin/bash
# Round 3: the whole GPU suite once (verbose, per-test timeout), then smoke.
set -u
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r03tests}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -v --timeout 200 --timeout-method thread tests/ -x -m gpu > $O/tests.log 2>&1 || { echo GPU TESTS FAILED; tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE FAILED; tail $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
