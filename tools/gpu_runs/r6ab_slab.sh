#!/bin/bash
# round 6: quad-transposed 8/16-byte slab stores vs 2/4-byte stores (FZ_SLAB_B16), same box
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ab
mkdir -p $O
for D in "" "-DFZ_SLAB_B16" "" "-DFZ_SLAB_B16"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { tail -5 $O/obj.log; exit 1; }
  echo "[$D] step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)  obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
done
