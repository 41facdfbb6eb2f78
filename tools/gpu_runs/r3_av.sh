#!/bin/bash
# Round 3, pass av: steps per graph at the driver's bench shape (--steps 20 --warmup 5): 4 / 5 / 10,
# alternating; then the full GPU suite and smoke() on the final tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3av}
mkdir -p $O
bench() {  # $1 label, env in $2
  env $2 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'case':'$1','ms':round(d['ms_per_step'],5),'k':d['steps_per_graph']}))" | tee -a $O/ab.jsonl
}
for r in 1 2 3; do
  bench k10 "TDQ_STEP_UNROLL=10" && bench k5 "TDQ_STEP_UNROLL=5" && bench k4 "TDQ_STEP_UNROLL=4" || exit 1
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
