#!/bin/bash
# Round 5: accuracy of the reference schedule - separate launches vs fused step (cheap / accurate
# tanh) vs the bf16w L-BFGS objective
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5acc}
mkdir -p $O
run() {  # name, env..., -- bench args
  local name=$1; shift
  env "$@" timeout -k 10 400 python bench.py --steps 20 --warmup 5 $BARGS > $O/$name.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/$name.json').read().splitlines()[-1]);print('$name', round(d['ms_per_step'],5), [round(v,5) for v in d.get('l2_full_schedule_seeds') or []], d.get('time_to_solution_s'))"
}
BARGS="" run separate TDQ_FUSED_STEP=0
BARGS="" run fused_acc_tanh TDQ_FUSED_STEP_DEFINES=-DFZ_CHEAP_TANH=0
BARGS="--newton-precision bf16w" run fused_bf16w TDQ_FUSED_STEP=1
