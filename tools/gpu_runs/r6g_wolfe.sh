#!/bin/bash
# round 6: line-search L-BFGS (newton_eager=False) - algorithm vs objective precision (fp64 jet /
# bf16x3 / fp32 from the same Adam start, N_f 5k), then the reference schedule at 50k on 3 seeds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6g
timeout -k 10 500 python -u tools/wolfe_diag.py --npts 5000 --adam 10000 --iters 3000 --objectives bf16x3 fp32 fp64 --out gpurun_out/r6g/diag.jsonl > gpurun_out/r6g/diag.log 2>&1 || { tail -20 gpurun_out/r6g/diag.log; exit 1; }
grep '^{' gpurun_out/r6g/diag.log
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --newton-eager 0 > gpurun_out/r6g/bench_wolfe.log 2>&1 || { tail -20 gpurun_out/r6g/bench_wolfe.log; exit 1; }
grep '^{' gpurun_out/r6g/bench_wolfe.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['l2_full_schedule_seeds'], d['time_to_solution_s'], d['lbfgs'])"
