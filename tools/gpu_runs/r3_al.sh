#!/bin/bash
# Round 3, pass al: peer all-reduce tests incl. the bounded-wait timeout path.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3al}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_peer_gpu.py -v -s --timeout 200 --timeout-method thread > $O/pytest_peer.log 2>&1
rc=$?
tail -4 $O/pytest_peer.log
exit $rc
