#!/bin/bash
# Round 4: L-BFGS precision schedule sweep on the driver shape (3 seeds each): time to solution vs L2
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4j}
mkdir -p $O
for sch in bf16:6000 bf16:8000 bf16:9000; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --newton-schedule $sch > $O/sched_$sch.json 2> $O/sched_$sch.err || { tail -20 $O/sched_$sch.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/sched_$sch.json').read().splitlines()[-1]);print(json.dumps({'sched':'$sch','l2':d.get('l2_full_schedule_seeds'),'tts':d.get('time_to_solution_s')}))" | tee -a $O/sched.jsonl
done
