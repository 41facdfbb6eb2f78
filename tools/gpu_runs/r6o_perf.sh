#!/bin/bash
# round 6: perf guards (AC-SA / AC-baseline step, ratio) after the fused-kernel speedups
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6o
timeout -k 10 600 python -u -m pytest tests/test_perf_gpu.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r6o/perf.log 2>&1; rc=$?
grep -E "PERF|PASS|FAIL|passed|failed" gpurun_out/r6o/perf.log; exit $rc
