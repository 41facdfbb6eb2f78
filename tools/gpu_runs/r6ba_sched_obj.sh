#!/bin/bash
# round 6: max-ilp scheduler for the bf16x3 objective only - repeat A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ba
mkdir -p $O
for D in "" "-mllvm -amdgpu-sched-strategy=max-ilp" "" "-mllvm -amdgpu-sched-strategy=max-ilp" "" "-mllvm -amdgpu-sched-strategy=max-ilp"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { tail -3 $O/obj.log; exit 1; }
  echo "[$D] obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
done
TDQ_FUSED_STEP_DEFINES="-mllvm -amdgpu-sched-strategy=max-ilp" timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/l1.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/l0.log 2>&1 || exit 1
echo "lbfgs max-ilp $(tail -1 $O/l1.log | grep -o "\"ms_per_iter\": [0-9.]*")  default $(tail -1 $O/l0.log | grep -o "\"ms_per_iter\": [0-9.]*")"
