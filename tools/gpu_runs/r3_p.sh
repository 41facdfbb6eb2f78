#!/bin/bash
# Round 3, pass p: capture order of the point-range chains (TDQ_SPLIT_ORDER fwd | rev) x cut.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3p}
mkdir -p $O
bench() {  # $1 order, $2 split, $3 precision
  TDQ_SPLIT_ORDER=$1 TDQ_SPLIT=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $3 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'order':'$1','split':'$2','prec':'$3','ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
}
for r in 1 2; do
  for c in "fwd 0.45" "rev 0.45" "rev 0.55" "rev 0.5" "rev 0.6"; do bench $c bf16 || exit 1; done
done
for c in "fwd 0.35" "rev 0.35" "rev 0.45" "rev 0.55" "fwd 0.35" "rev 0.35"; do bench $c bf16x3 || exit 1; done
(cd /tmp && export TMPDIR=/tmp && TDQ_SPLIT_ORDER=rev timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt; tail -20 $O/timeline.txt
