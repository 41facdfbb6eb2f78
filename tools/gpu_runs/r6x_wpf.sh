#!/bin/bash
# round 6: L2 warm-up of the weight images at kernel start (A/B) + first-tile phase stamps
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6x
mkdir -p $O
for D in "" "-DFZ_NO_WPREFETCH" "" "-DFZ_NO_WPREFETCH"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "[$D] $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
done
timeout -k 10 200 python -u tools/fused_step_timing.py > $O/phases_first.txt 2>&1 || { tail -5 $O/phases_first.txt; exit 1; }
grep -E "tile loads|gemm|all tiles|total" $O/phases_first.txt
