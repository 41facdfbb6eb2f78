#!/bin/bash
# accuracy probe: precision bf16 with bf16-rounded weights (variant library), Adam bf16 + L-BFGS bf16x3
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r2pw}
mkdir -p $O
export TDQ_LIB_PATH=$R/tensordiffeq_amd/csrc/build_purew/libtdq_hip.so
timeout -k 10 300 python -u tools/precision_errors.py > $O/prec_err.txt 2>&1 || { tail -30 $O/prec_err.txt; exit 1; }
grep "bf16 " $O/prec_err.txt
for s in 0 1 2; do
  timeout -k 10 240 python -u tools/accuracy_ac_sa.py --prec bf16+bf16x3 --seed $s >> $O/acc.jsonl 2>> $O/acc_err.log || { tail -20 $O/acc_err.log; exit 1; }
done
cat $O/acc.jsonl
timeout -k 10 600 python -u tools/run_configs.py --precision bf16+bf16x3 --which burgers discovery > $O/configs.log 2>&1 || { tail -30 $O/configs.log; exit 1; }
grep "^{" $O/configs.log
