#!/bin/bash
# Round 3, pass as: one-launch step tail (bookkeeping on the first range's branch, last-arriver
# theta Adam per column group) - bit-identity tests, A/B vs the two-launch tail, timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3as}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_hip_kernels.py -k "range or tail or one_launch" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bench() {  # $1 label, env in $2
  env $2 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'case':'$1','ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
}
for r in 1 2 3; do
  bench two "TDQ_TAIL_ONE=0" && bench one "TDQ_TAIL_ONE=1" || exit 1
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 48 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_one --steps 2 > $O/timeline.txt; tail -26 $O/timeline.txt
