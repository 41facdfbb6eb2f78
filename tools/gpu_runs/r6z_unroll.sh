#!/bin/bash
# round 6: steps per captured graph at the driver's shape (--steps 20 --warmup 5)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6z
mkdir -p $O
for rep in 1 2; do
  for U in 10 20 5 4; do
    TDQ_STEP_UNROLL=$U timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "unroll $U: $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
  done
done
