#!/bin/bash
# bf16 derivative-stream storage: precision table, kernel tests, kernel-time A/B vs fp32 storage.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TDQ_RUN:-r2hs}
mkdir -p $O
timeout -k 10 300 python -u tools/precision_errors.py > $O/prec_err.txt 2>&1 || { tail -30 $O/prec_err.txt; exit 1; }
grep "128, 128, 128, 128, 1\|50, 50" $O/prec_err.txt
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
VARIANT=hs32 PREC=bf16 TDQ_RUN=${TDQ_RUN:-r2hs}/ab bash tools/gpu_runs/r2_ab_kern.sh
