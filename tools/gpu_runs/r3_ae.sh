#!/bin/bash
# Round 3, pass ae: capture order of the two point-range chains (TDQ_SPLIT_ORDER fwd | rev | main):
# which queue the graph runtime gives the tail, and the join latency before it.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ae}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -k "range" -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bench() {  # $1 order
  TDQ_SPLIT_ORDER=$1 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'order':'$1','ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
}
for r in 1 2; do bench fwd && bench rev && bench main || exit 1; done
for M in rev main; do
  (cd /tmp && export TMPDIR=/tmp && TDQ_SPLIT_ORDER=$M timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$M -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_$M.log 2>&1) || { tail -20 $O/prof_$M.log; exit 1; }
  python tools/timeline.py $O/prof_$M/run_kernel_trace.csv --anchor tail_adam --steps 1 > $O/timeline_$M.txt; tail -12 $O/timeline_$M.txt
done
