#!/bin/bash
# Round 4: AC-baseline cut sweep with the MFMA high-order kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4cut
mkdir -p $O
for rep in 1 2; do
for c in 0.50 0.56 0.62 0.68 0.74; do
  TDQ_SPLIT=$c timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b_$c.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$c.json').read().splitlines()[-1]);print(json.dumps({'problem':'ac-baseline','cut':$c,'rep':$rep,'ms':round(d['ms_per_step'],5)}))" | tee -a $O/sweep.jsonl
done
done
