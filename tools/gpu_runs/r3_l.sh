#!/bin/bash
# Round 3, pass l: point-range tests (single-process + forced DP over RCCL), split-fraction sweep
# for the bf16 and bf16x3 Adam steps and the bf16x3 L-BFGS iteration.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3l}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_hip_kernels.py -k "range" -m gpu -v -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
grep -E "FAILED|ERROR" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
bench() {  # $1 split, $2 precision
  TDQ_SPLIT=$1 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'split':'$1','prec':'$2','ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/split_sweep.jsonl
}
for SP in 0 0.5 0.45 0.55 0.6 0.4 0.5 0; do bench $SP bf16 || exit 1; done
for SP in 0 0.4 0.35 0.45 0.3 0.4; do bench $SP bf16x3 || exit 1; done
for SP in 0.4 0 0.35 0.3 0.45; do
  TDQ_SPLIT=$SP timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 > $O/tmp.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/tmp.json').read().splitlines()[-1]);d['split']='$SP';print(json.dumps(d))" | tee -a $O/lbfgs.jsonl
done
