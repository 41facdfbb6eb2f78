#!/bin/bash
# round 6: AC-dist / AC-baseline with the free-CU order rule, and both forced orders for AC-dist
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6an
mkdir -p $O
for ORD in auto side_first fused_first auto; do
  if [ $ORD = auto ]; then unset TDQ_FS_SPLIT_ORDER; else export TDQ_FS_SPLIT_ORDER=$ORD; fi
  timeout -k 10 300 python -u bench.py --problem ac-dist --steps 40 --warmup 5 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "ac-dist $ORD $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
done
unset TDQ_FS_SPLIT_ORDER
timeout -k 10 200 python -u bench.py --problem ac-baseline --steps 200 --warmup 20 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
echo "ac-baseline auto $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
