#!/bin/bash
# AC-SA reference schedule (Adam 10k + L-BFGS 10k): device vs host-driven L-BFGS, two seeds.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r10
mkdir -p $O
for seed in 0 1; do
  for impl in device host; do
    TDQ_LBFGS=$impl timeout -k 10 300 python -u tools/accuracy_ac_sa.py --iters 10000 --newton 10000 --prec bf16x3 --seed $seed > $O/acc_${impl}_s$seed.jsonl 2> $O/acc.err || { tail -20 $O/acc.err; exit 1; }
    echo "$impl seed $seed: $(tail -1 $O/acc_${impl}_s$seed.jsonl)"
  done
done
