#!/bin/bash
# round 6: timing probe - the bf16 step without its dK slab stores (wrong gradients; timing only)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6au
mkdir -p $O
for D in "" "-DFZ_DBG_NO_SLAB" "" "-DFZ_DBG_NO_SLAB"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "[$D] step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
done
