#!/bin/bash
# Round 5: the GPU test suite + smoke
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5suite}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rs --maxfail=6 --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PERF|FUSED_STEP_WLO|ACCURACY|WOLFE|passed|failed|FAILED|ERROR" $O/pytest_gpu.log | cut -c1-250 | tail -40
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
