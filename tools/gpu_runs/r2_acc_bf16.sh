#!/bin/bash
# AC-SA reference schedule (Adam 10k + L-BFGS 10k): L2 on the AC.mat grid, bf16 vs bf16x3, 2 seeds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TDQ_RUN:-r2accm}
mkdir -p $O
for s in 0 1 2; do
  timeout -k 10 240 python -u tools/accuracy_ac_sa.py --prec bf16+bf16x3 $( [ $s = 2 ] && echo bf16x3 ) --seed $s >> $O/acc.jsonl 2>> $O/acc_err.log || { tail -20 $O/acc_err.log; exit 1; }
done
cat $O/acc.jsonl
