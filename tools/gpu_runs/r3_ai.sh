#!/bin/bash
# Round 3, pass ai: pre-reduction in the DP / L-BFGS tails (dp_tail_a c_first): tests + L-BFGS A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ai}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_hip_kernels.py tests/test_dist_gpu.py tests/test_lbfgs_device.py tests/test_accuracy_gpu.py -q -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log; grep ACCURACY $O/pytest.log
for P in 1 0 1 0; do
  TDQ_PREREDUCE=$P timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 > $O/tmp.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/tmp.json').read().splitlines()[-1]);d['prereduce']='$P';print(json.dumps(d))" | tee -a $O/lbfgs.jsonl
done
