#!/bin/bash
# round 6: A/B of hipRTC defines on both fused kernels (step time 200 steps, objective us)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6n
for i in 1 2; do
for D in "" "-DFZ_GEMM_SB=0"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 120 python -u tools/obj_bench.py --tag "[$D]" >> gpurun_out/r6n/obj.jsonl 2>/dev/null || exit 1
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-l2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench200 [$D]', d['ms_per_step'])" >> gpurun_out/r6n/bench.txt || exit 1
done
done
cat gpurun_out/r6n/obj.jsonl gpurun_out/r6n/bench.txt
