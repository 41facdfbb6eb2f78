#!/bin/bash
# Round 5: AC-SA accuracy schedule with the strong-Wolfe device L-BFGS (newton_eager=False)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5wacc}
mkdir -p $O
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --newton-eager 0 --acc-seeds 0 1 2 ${EXTRA} > $O/bench_wolfe.json 2> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_wolfe.json').read().splitlines()[-1]);print('wolfe', d.get('l2_full_schedule_seeds'), d.get('time_to_solution_s'), d.get('lbfgs'))"
