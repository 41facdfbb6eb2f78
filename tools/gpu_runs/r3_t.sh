#!/bin/bash
# Round 3, pass t: one-shot peer all-reduce (2 ranks on one GPU) + DP tests incl. K-step DP graphs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3t}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_peer_gpu.py -x -v -s --timeout 300 --timeout-method thread > $O/pytest_peer.log 2>&1
rc=$?
tail -5 $O/pytest_peer.log; grep PEER $O/pytest_peer.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py -v -s --timeout 600 --timeout-method thread > $O/pytest_dist.log 2>&1
rc=$?
tail -3 $O/pytest_dist.log; grep -E "FAILED|ERROR|Error" $O/pytest_dist.log | head -20
exit $rc
