#!/bin/bash
# Round 5: weight-lo L-BFGS objective (bf16w) test + accuracy schedule (default bf16x3 vs bf16w),
# steps-per-graph sweep
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5wlo}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_step.py -x -v -s -m gpu -k "weight_lo" --timeout 250 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
grep -E "FUSED_STEP_WLO|passed|failed" $O/pytest.log
for u in 8 32; do
  TDQ_STEP_UNROLL=$u timeout -k 10 200 python bench.py --steps 1000 --warmup 20 --no-l2 > $O/b_u$u.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_u$u.json').read().splitlines()[-1]);print('unroll $u', round(d['ms_per_step'],5), round(d['value']/1e6,1))"
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/b_driver.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b_driver.json').read().splitlines()[-1]);print('driver', round(d['ms_per_step'],5), round(d['value']/1e6,1), d.get('l2_full_schedule'), d.get('l2_full_schedule_seeds'), d.get('time_to_solution_s'))"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --newton-precision bf16w > $O/b_bf16w.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b_bf16w.json').read().splitlines()[-1]);print('bf16w', round(d['ms_per_step'],5), d.get('l2_full_schedule'), d.get('l2_full_schedule_seeds'), d.get('time_to_solution_s'), d.get('lbfgs'))"
