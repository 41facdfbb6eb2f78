#!/bin/bash
# Round 3, pass v: specialized (hipRTC) fused-loss kernels - bitwise tests, bench A/B vs the
# interpreter, kernel timeline of the split step with the JIT loss.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3v}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_loss_jit.py tests/test_fusion.py -v -s --timeout 300 --timeout-method thread > $O/pytest_jit.log 2>&1
rc=$?
tail -3 $O/pytest_jit.log; grep -E "FAILED|Error|assert" $O/pytest_jit.log | head -20
[ $rc -eq 0 ] || exit $rc
bench() {  # $1 jit flag, $2 precision
  TDQ_LOSS_JIT=$1 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'jit':'$1','prec':'$2','ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/ab.jsonl
}
bench 1 bf16 && bench 0 bf16 && bench 1 bf16 && bench 0 bf16 && bench 1 bf16x3 && bench 0 bf16x3 || exit 1
for J in 1 0; do
  TDQ_LOSS_JIT=$J timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 > $O/tmp.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/tmp.json').read().splitlines()[-1]);d['jit']='$J';print(json.dumps(d))" | tee -a $O/lbfgs.jsonl
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 3 > $O/timeline.txt; tail -30 $O/timeline.txt
