#!/bin/bash
# round 6: more LLVM options for the bf16 step / bf16x3 objective
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6bc
mkdir -p $O
for D in "" "-mllvm -amdgpu-use-amdgpu-trackers=1" "-mllvm -amdgpu-disable-unclustered-high-rp-reschedule" "-mllvm -amdgpu-schedule-metric-bias=100" "-ffast-math" ""; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { echo "[$D] bench failed"; continue; }
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { echo "[$D] obj failed"; continue; }
  echo "[$D] step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)  obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
done
