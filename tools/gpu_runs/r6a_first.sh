#!/bin/bash
# round 6, first GPU pass: smoke (fp64 checks of both fused kernels), the fused-kernel fp64 tests,
# the fused-vs-separate tests, then a throughput-only bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6a
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6a/smoke.log 2>&1 || { tail -30 gpurun_out/r6a/smoke.log; exit 1; }
tail -8 gpurun_out/r6a/smoke.log
timeout -k 10 900 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/r6a/pytest.log 2>&1; rc=$?
grep -E "FUSED|PASS|FAIL|passed|failed|Error" gpurun_out/r6a/pytest.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-l2 > gpurun_out/r6a/bench.log 2>&1 || { tail -20 gpurun_out/r6a/bench.log; exit 1; }
tail -2 gpurun_out/r6a/bench.log
