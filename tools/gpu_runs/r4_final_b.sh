#!/bin/bash
# Round 4 final (b): per-problem bench records (ac-baseline with accuracy, discovery, poisson, ac-dist, width 256)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4fb}
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/bench_$tag.json 2> $O/bench_$tag.err || { tail -20 $O/bench_$tag.err; return 1; }
  python -c "import json;d=json.loads(open('$O/bench_$tag.json').read().splitlines()[-1]);print('$tag', json.dumps({k:d.get(k) for k in ['ms_per_step','value','l2_full_schedule_seeds','coefficients','time_to_solution_s','lbfgs']}))"
}
run acb --problem ac-baseline --steps 200 --warmup 20 --acc-seeds 0 && \
run disc --problem discovery --steps 20 --warmup 5 --acc-seeds 0 && \
run poisson --problem poisson --steps 20 --warmup 3 --no-l2 && \
run acdist --problem ac-dist --steps 100 --warmup 10 --no-l2 && \
run w256 --layers 2,256,256,256,256,1 --steps 100 --warmup 10 --no-l2
