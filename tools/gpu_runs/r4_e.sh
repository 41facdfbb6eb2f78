#!/bin/bash
# Round 4: where the high-order kernels sit in the step graph (0 serial, 2 forward on a side branch, 1 both)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4e}
mkdir -p $O
for m in 0 2 1; do
  TDQ_HI_BRANCH=$m timeout -k 10 200 python -X faulthandler bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b400_acb_$m.json 2>> $O/b400_$m.err || { tail -30 $O/b400_$m.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400_acb_$m.json').read().splitlines()[-1]);print(json.dumps({'mode':'$m','ms':round(d['ms_per_step'],5),'value':d['value']}))"
done
