#!/bin/bash
# Round 5: in-kernel bookkeeping + one-launch tail - tests and A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5book}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_step.py tests/test_hip_kernels.py -m gpu -q -x -s --timeout 300 --timeout-method thread -k "fused_step or tail" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -20; exit 1; }
grep -E "FUSED_STEP_TRAJ|passed" $O/pytest.log | cut -c1-250
for r in 1 2 3; do
for b in 1 0; do
TDQ_FS_BOOK=$b timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b_${b}_$r.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/b_${b}_$r.json').read().splitlines()[-1]);print('book $b', round(d['ms_per_step'],5), d['loss_after'])"
done
done
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/b_driver.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/b_driver.json').read().splitlines()[-1]);print('driver', round(d['ms_per_step'],5), round(d['value']/1e6,1), [round(v,5) for v in d.get('l2_full_schedule_seeds')], d.get('time_to_solution_s'))"
