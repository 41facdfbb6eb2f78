#!/bin/bash
# Round 4: slab chunks scaled with the row count (large point sets) + batched second-pass loads
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4chunks
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_perf_gpu.py tests/test_lbfgs_device.py -m gpu -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; fi
for p in poisson ac-dist ac-sa; do
  timeout -k 10 300 python bench.py --problem $p --steps 20 --warmup 3 --no-l2 > $O/b_$p.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$p.json').read().splitlines()[-1]);print(json.dumps({'problem':'$p','ms':round(d['ms_per_step'],4),'value':d['value']}))" | tee -a $O/bench.jsonl
done
