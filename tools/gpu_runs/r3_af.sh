#!/bin/bash
# Round 3, pass af: layered engine in bf16 / bf16x3 GEMM families: numerics + width-256 bench
# (layered fp32 / bf16x3 / bf16 vs the torch jet engine).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3af}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_layered_jet.py -v -s --timeout 300 --timeout-method thread > $O/pytest_layered.log 2>&1
rc=$?
tail -2 $O/pytest_layered.log; grep -E "KERNEL_ERR|FAILED" $O/pytest_layered.log | head -30
[ $rc -eq 0 ] || exit $rc
bench() {  # $1 backend, $2 precision
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --min-warmup-s 0.5 --no-l2 --layers 2,256,256,256,256,1 --backend $1 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'backend':'$1','prec':'$2','ms':round(d['ms_per_step'],4),'value':d['value'],'model':d['config']['model']}))" | tee -a $O/wide.jsonl
}
bench hip fp32 && bench hip bf16x3 && bench hip bf16
