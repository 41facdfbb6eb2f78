#!/bin/bash
# round 6: new kernel unit tests + AC-baseline split sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6aj
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lay_reduce.py -m gpu -q -x --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
bash tools/gpu_runs/r6ai_acb_sweep.sh
