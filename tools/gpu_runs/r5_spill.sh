#!/bin/bash
# Round 5: fused step after the loss-section spill fix: tests + A/B bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5spill}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_step.py tests/test_fused_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -20; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
for rep in 1 2; do
timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b400_$rep.json 2>> $O/b.err || { tail -5 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b400_$rep.json').read().splitlines()[-1]);print('ac-sa 400 steps', round(d['ms_per_step'],5), round(d['value']/1e6,1))"
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-l2 > $O/b20_$rep.json 2>> $O/b.err || { tail -5 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b20_$rep.json').read().splitlines()[-1]);print('ac-sa driver shape', round(d['ms_per_step'],5), round(d['value']/1e6,1))"
done
