#!/bin/bash
# Round 3, pass y: point-range cut sweep with the JIT loss (bf16 and bf16x3), L-BFGS at its cut.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3y}
mkdir -p $O
bench() {  # $1 cut, $2 precision
  TDQ_SPLIT=$1 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'split':'$1','prec':'$2','ms':round(d['ms_per_step'],5)}))" | tee -a $O/sweep.jsonl
}
for r in 1 2; do
  for c in 0.40 0.45 0.50 0.55 0.60; do bench $c bf16 || exit 1; done
done
for c in 0.30 0.35 0.40 0.45 0.35 0.40; do bench $c bf16x3 || exit 1; done
for c in 0.35 0.40 0.30; do
  TDQ_SPLIT=$c timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 > $O/tmp.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/tmp.json').read().splitlines()[-1]);d['split']='$c';print(json.dumps(d))" | tee -a $O/lbfgs.jsonl
done
