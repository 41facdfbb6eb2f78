#!/bin/bash
# Round 3, pass z: finer bf16 cut sweep with the JIT loss.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3z}
mkdir -p $O
bench() {  # $1 cut, $2 precision
  TDQ_SPLIT=$1 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'split':'$1','prec':'$2','ms':round(d['ms_per_step'],5)}))" | tee -a $O/sweep.jsonl
}
for r in 1 2 3; do
  for c in 0.32 0.36 0.38 0.40 0.42 0.45; do bench $c bf16 || exit 1; done
done
