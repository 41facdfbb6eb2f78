#!/bin/bash
# Round 3, pass aw: solver-level layered-engine runs (width 256 and 18 hidden layers) vs torch jet.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3aw}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_layered_jet.py -k trains > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
grep -E "passed|failed|LAYERED" $O/pytest.log
