#!/bin/bash
# round 6: L-BFGS wall per iteration (pipelined polls), device L-BFGS GPU tests, bench with 3 seeds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6f
timeout -k 10 120 python -u tools/obj_bench.py --tag fused3 >> gpurun_out/r6f/obj.jsonl 2>/dev/null || exit 1
cat gpurun_out/r6f/obj.jsonl
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > gpurun_out/r6f/lbfgs.json 2>/dev/null || exit 1
cat gpurun_out/r6f/lbfgs.json
timeout -k 10 600 python -u -m pytest tests/test_lbfgs_device.py tests/test_lbfgs_wolfe.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r6f/pytest_lbfgs.log 2>&1; rc=$?
tail -3 gpurun_out/r6f/pytest_lbfgs.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6f/bench.log 2>&1 || { tail -20 gpurun_out/r6f/bench.log; exit 1; }
tail -1 gpurun_out/r6f/bench.log | cut -c1-200
