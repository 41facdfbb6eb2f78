#!/bin/bash
# round 6: compile-time stream spec in the fused kernels - step / objective timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6k
for i in 1 2; do
timeout -k 10 120 python -u tools/obj_bench.py --tag spec_constexpr >> gpurun_out/r6k/obj.jsonl 2>/dev/null || exit 1
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-l2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench200', d['ms_per_step'])" >> gpurun_out/r6k/bench.txt || exit 1
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-l2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench20', d['ms_per_step'])" >> gpurun_out/r6k/bench.txt || exit 1
done
cat gpurun_out/r6k/obj.jsonl gpurun_out/r6k/bench.txt
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -x -q --timeout 200 --timeout-method thread 2>&1 | tail -2
