#!/bin/bash
# AC-SA reference schedule (Adam 10k + L-BFGS 10k) on the rebuilt library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r17
mkdir -p $O
timeout -k 10 400 python -u tools/accuracy_ac_sa.py --iters 10000 --newton 10000 --prec bf16x3 > $O/acc.jsonl 2> $O/acc.err || { tail -20 $O/acc.err; exit 1; }
cat $O/acc.jsonl
