#!/bin/bash
# round 6: line-search L-BFGS on the bf16x3 / fp32 objectives, approximate-Wolfe tolerance sweep
# (N_f 50k, Adam 10k start, seed 0), plus the fp32 objective's cost per evaluation
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6h
timeout -k 10 120 python -u tools/obj_bench.py --precision fp32 --tag fp32 > gpurun_out/r6h/obj_fp32.json 2>/dev/null || exit 1
cat gpurun_out/r6h/obj_fp32.json
timeout -k 10 600 python -u tools/wolfe_diag.py --npts 50000 --adam 10000 --iters 10000 --objectives bf16x3 --hz-eps 1e-6 1e-5 1e-4 1e-3 --out gpurun_out/r6h/diag.jsonl > gpurun_out/r6h/diag.log 2>&1 || { tail -20 gpurun_out/r6h/diag.log; exit 1; }
grep '^{' gpurun_out/r6h/diag.log
