#!/bin/bash
# round 6: bf16x3 objective - layer-0 adjoint from the rebuilt slot-0 image: fp64 tests, objective time, L-BFGS, accuracy
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ad
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -m gpu -q -x -s --timeout 300 --timeout-method thread -k "bf16x3" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|FUSED_FP64" $O/pytest.log | head -30; exit 1; }
grep -E "FUSED_FP64|passed" $O/pytest.log | cut -c1-200
for i in 1 2; do
timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { tail -5 $O/obj.log; exit 1; }
grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1
done
timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/lbfgs.log 2>&1 || { tail -5 $O/lbfgs.log; exit 1; }
tail -1 $O/lbfgs.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['value'], 'L2', d['l2_full_schedule'], d['l2_full_schedule_seeds'], d['time_to_solution_s'])"
