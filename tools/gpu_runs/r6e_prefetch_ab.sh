#!/bin/bash
# round 6: bf16x3 objective A/B - weight prefetch one phase ahead vs at the GEMM (FZ3_NO_PREFETCH);
# L-BFGS wall time per iteration with the pipelined host polls; device L-BFGS GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6e
for i in 1 2; do
timeout -k 10 120 python -u tools/obj_bench.py --tag prefetch >> gpurun_out/r6e/ab.jsonl 2>/dev/null || exit 1
TDQ_FUSED_STEP_DEFINES="-DFZ3_NO_PREFETCH" timeout -k 10 120 python -u tools/obj_bench.py --tag at_gemm >> gpurun_out/r6e/ab.jsonl 2>/dev/null || exit 1
done
TDQ_FUSED_STEP=0 timeout -k 10 120 python -u tools/obj_bench.py --tag separate >> gpurun_out/r6e/ab.jsonl 2>/dev/null || exit 1
cat gpurun_out/r6e/ab.jsonl
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > gpurun_out/r6e/lbfgs.json 2>/dev/null || exit 1
cat gpurun_out/r6e/lbfgs.json
timeout -k 10 600 python -u -m pytest tests/test_lbfgs_device.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r6e/pytest_lbfgs.log 2>&1; rc=$?
tail -3 gpurun_out/r6e/pytest_lbfgs.log; exit $rc
