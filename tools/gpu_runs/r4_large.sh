#!/bin/bash
# Round 4: large-set fused-tail equivalence test
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4large
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -k "large_set or fused_step_tail" -m gpu -v --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "large_set|passed|failed" $O/pytest.log | tail -4
exit $rc
