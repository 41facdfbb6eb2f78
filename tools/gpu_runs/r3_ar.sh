#!/bin/bash
# Round 3, pass ar: join order of the two point-range branches (TDQ_JOIN_ORDER fwd | rev): does the
# graph runtime put the tail behind the first-joined branch?
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ar}
mkdir -p $O
bench() {  # $1 label, env in $2
  env $2 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'case':'$1','ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
}
for r in 1 2; do
  bench fwd "TDQ_JOIN_ORDER=fwd" && bench rev "TDQ_JOIN_ORDER=rev" && bench rev_c62 "TDQ_JOIN_ORDER=rev TDQ_SPLIT=0.62 TDQ_PREREDUCE=0" || exit 1
done
(cd /tmp && export TMPDIR=/tmp && TDQ_JOIN_ORDER=rev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 48 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt; tail -24 $O/timeline.txt
