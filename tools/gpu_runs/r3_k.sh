#!/bin/bash
# Round 3, pass k: point ranges on concurrent graph branches (TDQ_SPLIT): equivalence tests, the
# GPU suite, L-BFGS iteration time split vs single, Adam bf16x3 / bf16 bench split vs single.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3k}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep ACCURACY $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for SP in auto 0 auto 0; do
  TDQ_SPLIT=$SP timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 > $O/tmp.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/tmp.json').read().splitlines()[-1]);d['split']='$SP';print(json.dumps(d))" | tee -a $O/lbfgs.jsonl
done
for SP in 0.4 0 0.3 0.5; do
  TDQ_SPLIT=$SP timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision bf16x3 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'split':'$SP','prec':'bf16x3','ms':d['ms_per_step'],'value':d['value']}))" | tee -a $O/bench_split.jsonl
done
for SP in 0 0.5 0.4 0; do
  TDQ_SPLIT=$SP timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'split':'$SP','prec':'bf16','ms':d['ms_per_step'],'value':d['value']}))" | tee -a $O/bench_split.jsonl
done
