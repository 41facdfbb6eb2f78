#!/bin/bash
# round 6: L-BFGS with images written by the update (test + timing), Wolfe GPU test, bench 3 seeds
# with newton_eager=False (precision-aware line-search tolerance), default bench
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6i
timeout -k 10 600 python -u -m pytest tests/test_lbfgs_device.py tests/test_lbfgs_wolfe.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6i/pytest.log 2>&1; rc=$?
grep -E "WOLFE|PASS|FAIL|passed|failed|Error" gpurun_out/r6i/pytest.log | tail -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > gpurun_out/r6i/lbfgs.json 2>/dev/null || exit 1
cat gpurun_out/r6i/lbfgs.json
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6i/bench.log 2>&1 || { tail -20 gpurun_out/r6i/bench.log; exit 1; }
grep '^{' gpurun_out/r6i/bench.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['time_to_solution_s'], d['l2_full_schedule_seeds'])"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 1 --newton-eager 0 > gpurun_out/r6i/bench_wolfe.log 2>&1 || { tail -20 gpurun_out/r6i/bench_wolfe.log; exit 1; }
grep '^{' gpurun_out/r6i/bench_wolfe.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['l2_full_schedule_seeds'], d['time_to_solution_s'], d['lbfgs'])"
