#!/bin/bash
# Round 3, pass ao: cut sweep with the pre-reduction (cuts on chunk boundaries 0.374 / 0.499 vs 0.45).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ao}
mkdir -p $O
bench() {  # $1 cut
  TDQ_SPLIT=$1 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'split':'$1','ms':round(d['ms_per_step'],5)}))" | tee -a $O/sweep.jsonl
}
for r in 1 2 3; do bench auto && bench 0.5 && bench 0.45 && bench 0.3 || exit 1; done
