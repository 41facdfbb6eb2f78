#!/bin/bash
# round 6: AC-dist 500k - extra tile rounds for the side chain (TDQ_FS_SPLIT_ROUNDS) under the order rule
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ao
mkdir -p $O
for RD in 0 1 2 4 0 1; do
  TDQ_FS_SPLIT_ROUNDS=$RD timeout -k 10 300 python -u bench.py --problem ac-dist --steps 40 --warmup 5 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "ac-dist rounds+$RD $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
done
