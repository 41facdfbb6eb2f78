#!/bin/bash
# Round 3, pass aj: driver-style bench (throughput + 3-seed full-schedule accuracy) on the current tree.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3aj}
mkdir -p $O
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','l2_full_schedule','l2_full_schedule_seeds','time_to_solution_s']})"
timeout -k 10 400 python bench.py --steps 20 --warmup 5 --acc-seeds 3 4 5 > $O/bench_seeds345.json 2> $O/bench_seeds345.err || { tail -20 $O/bench_seeds345.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_seeds345.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','l2_full_schedule','l2_full_schedule_seeds']})"
