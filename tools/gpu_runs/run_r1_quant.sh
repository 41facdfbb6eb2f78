#!/bin/bash
# Wave-quantization check: per-step time vs collocation points per GPU around the 256-CU round
# boundaries (64-point tiles, one workgroup per CU: 49152 = 3 rounds, 50000 = 3 rounds + 14 tiles,
# 65536 = 4 rounds).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r18
mkdir -p $O
for n in 49152 50000 65536 32768 16384; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --npts $n > $O/bench_$n.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "$n $(grep -o '"ms_per_step": [0-9.]*' $O/bench_$n.json)"
done
