#!/bin/bash
# round 6: fused-kernel fp64 tests + fused-vs-separate tests, then the bench with the accuracy
# schedule on seed 0 (the L-BFGS phase now on the one-launch bf16x3 objective)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6b
timeout -k 10 900 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r6b/pytest.log 2>&1; rc=$?
grep -E "FUSED|passed|failed|Error" gpurun_out/r6b/pytest.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --acc-seeds 0 > gpurun_out/r6b/bench.log 2>&1 || { tail -20 gpurun_out/r6b/bench.log; exit 1; }
tail -1 gpurun_out/r6b/bench.log
