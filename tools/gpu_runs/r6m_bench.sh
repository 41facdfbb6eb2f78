#!/bin/bash
# round 6: driver-shape bench (throughput + AC-SA accuracy schedule on 3 seeds) + L-BFGS per iteration
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6m
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > gpurun_out/r6m/lbfgs.json 2>/dev/null || exit 1
cat gpurun_out/r6m/lbfgs.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6m/bench.log 2>&1 || { tail -20 gpurun_out/r6m/bench.log; exit 1; }
grep '^{' gpurun_out/r6m/bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['time_to_solution_s'], d['l2_full_schedule_seeds'])"
