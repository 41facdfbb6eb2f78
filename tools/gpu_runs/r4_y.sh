#!/bin/bash
# Round 4: examples at medium schedules (L2 + Adam ms/step)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4y
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_examples_gpu.py -k converges -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "EXAMPLE|passed|failed|Error" $O/pytest.log | head -20
exit $rc
