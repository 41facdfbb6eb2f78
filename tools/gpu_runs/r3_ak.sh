#!/bin/bash
# Round 3, pass ak: BASELINE configurations on the current tree (Burgers, Helmholtz, discovery,
# 10M-point Poisson throughput) in bf16 (Adam) - one JSON line each.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ak}
mkdir -p $O
timeout -k 10 600 python -u tools/run_configs.py --which burgers helmholtz discovery poisson10m --precision bf16 > $O/configs_bf16.jsonl 2> $O/configs.err
rc=$?
cat $O/configs_bf16.jsonl | cut -c1-400
[ $rc -eq 0 ] || { tail -20 $O/configs.err; exit $rc; }
