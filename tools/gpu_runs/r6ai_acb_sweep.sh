#!/bin/bash
# round 6: AC-baseline split layout - launch order x extra tile rounds, and the AC-SA step in the same process family
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ai
mkdir -p $O
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
echo "ac-sa $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
for ORD in side_first fused_first; do
  for RD in 0 1 2; do
    TDQ_FS_SPLIT_ORDER=$ORD TDQ_FS_SPLIT_ROUNDS=$RD timeout -k 10 200 python -u bench.py --problem ac-baseline --steps 200 --warmup 20 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "ac-baseline $ORD rounds+$RD $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
  done
done
