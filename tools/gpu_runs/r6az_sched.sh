#!/bin/bash
# round 6: LLVM AMDGPU scheduler strategies for the run-time compiled fused kernels (hipRTC options)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6az
mkdir -p $O
for D in "" "-mllvm -amdgpu-sched-strategy=max-ilp" "-mllvm -amdgpu-sched-strategy=max-memory-clause" "-mllvm -amdgpu-sched-strategy=iterative-minreg" ""; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { echo "[$D] bench failed"; tail -3 $O/b.log; continue; }
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { echo "[$D] obj failed"; tail -3 $O/obj.log; continue; }
  echo "[$D] step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)  obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
done
