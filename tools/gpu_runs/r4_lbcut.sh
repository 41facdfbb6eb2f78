#!/bin/bash
# Round 4: bf16x3 (L-BFGS objective) range-cut sweep: L-BFGS wall time of 3000 iterations
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4lbcut
mkdir -p $O
for rep in 1 2; do
for c in 0.35 0.42 0.48 0.55; do
  TDQ_SPLIT=$c timeout -k 10 200 python bench.py --steps 5 --warmup 2 --min-warmup-s 0 --acc-seeds 0 --acc-iters 300 --acc-newton 3000 > $O/b_$c.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$c.json').read().splitlines()[-1]);print(json.dumps({'cut':$c,'rep':$rep,'lbfgs_s':d['time_to_solution_s'][0]['lbfgs_s'],'ms_per_iter':round(d['time_to_solution_s'][0]['lbfgs_s']/3000*1e3,4)}))" | tee -a $O/sweep.jsonl
done
done
