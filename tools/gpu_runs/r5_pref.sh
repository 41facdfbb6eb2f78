#!/bin/bash
# Round 5: loss-input prefetch - tests, bench, steady-state phase stamps
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5pref}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_step.py tests/test_fused_kernels.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $O/pytest.log | head -20; exit 1; }
grep -E "FUSED_STEP |passed" $O/pytest.log | cut -c1-250
for r in 1 2; do
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-l2 > $O/b20_$r.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/b20_$r.json').read().splitlines()[-1]);print('driver shape', round(d['ms_per_step'],5), round(d['value']/1e6,1))"
timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b400_$r.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/b400_$r.json').read().splitlines()[-1]);print('400 steps', round(d['ms_per_step'],5), round(d['value']/1e6,1))"
done
TDQ_FUSED_STEP_DEFINES="-DFZ_TS_TILE=1" timeout -k 10 200 python -u tools/fused_step_timing.py > $O/timing_tile1.txt 2>&1 || { tail -10 $O/timing_tile1.txt; exit 1; }
grep -E "loss|layer 0|epi 3|tile loop" $O/timing_tile1.txt
