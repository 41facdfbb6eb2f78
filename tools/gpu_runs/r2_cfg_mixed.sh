#!/bin/bash
# BASELINE configs with Adam in bf16 and L-BFGS in bf16x3 (the per-phase precision split).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r2cfgm}
mkdir -p $O
timeout -k 10 900 python -u tools/run_configs.py --precision ${PREC:-bf16+bf16x3} --which burgers helmholtz discovery poisson10m > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
grep "^{" $O/configs.log
