#!/bin/bash
# Round 5: WLO dK fix check + bf16w L-BFGS accuracy + fused tests
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5wlo2}
mkdir -p $O
timeout -k 10 200 python -u tools/wlo_diag.py > $O/wlo_diag.txt 2>&1 || { tail -20 $O/wlo_diag.txt; exit 1; }
grep -E "rows|layer [1-3] K" $O/wlo_diag.txt
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|WLO" $O/pytest.log | head -20; exit 1; }
grep -E "WLO|passed" $O/pytest.log
timeout -k 10 500 python bench.py --steps 20 --warmup 5 --newton-precision bf16w > $O/bf16w.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bf16w.json').read().splitlines()[-1]);print('bf16w', round(d['ms_per_step'],5), [round(v,5) for v in d.get('l2_full_schedule_seeds')], d.get('time_to_solution_s'), [x['reason'] for x in d.get('lbfgs')])"
