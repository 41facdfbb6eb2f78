#!/bin/bash
# Round 4: AC-dist 500k cut sweep with the MFMA high-order kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4acdcut
mkdir -p $O
for rep in 1 2; do
for c in 0.38 0.44 0.50 0.56 0.62; do
  TDQ_SPLIT=$c timeout -k 10 200 python bench.py --problem ac-dist --steps 100 --warmup 5 --no-l2 > $O/b_$c.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$c.json').read().splitlines()[-1]);print(json.dumps({'problem':'ac-dist','cut':$c,'rep':$rep,'ms':round(d['ms_per_step'],5)}))" | tee -a $O/sweep.jsonl
done
done
