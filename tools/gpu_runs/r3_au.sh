#!/bin/bash
# Round 3, pass au: the driver's bench shape (--steps 20 --warmup 5): 2 x 10-step graphs (old
# default) vs one 20-step graph (new default), alternating; then the GPU NaN-check test.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3au}
mkdir -p $O
bench() {  # $1 label, env in $2
  env $2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'case':'$1','ms':round(d['ms_per_step'],5),'k':d['steps_per_graph']}))" | tee -a $O/ab.jsonl
}
for r in 1 2 3; do
  bench k10 "TDQ_STEP_UNROLL=10" && bench auto "TDQ_X=1" || exit 1
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_config_metrics.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
