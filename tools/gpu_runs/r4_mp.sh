#!/bin/bash
# Round 4: multi-process GPU tests after the port / fail-fast changes
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4mp
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests/test_peer_gpu.py tests/test_dist_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed" $O/pytest.log | tail -16
exit $rc
