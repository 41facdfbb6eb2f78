#!/bin/bash
# Round 3, pass x: bench A/B JIT loss vs interpreter (bf16, 600 timed steps, alternating x4).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3x}
mkdir -p $O
bench() {  # $1 jit flag, $2 precision
  TDQ_LOSS_JIT=$1 timeout -k 10 200 python bench.py --steps 600 --warmup 20 --no-l2 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'jit':'$1','prec':'$2','ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/ab.jsonl
}
for k in 1 2 3 4; do bench 1 bf16 && bench 0 bf16 || exit 1; done
grep -i warn $O/bench.err | head -3
