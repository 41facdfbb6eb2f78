#!/bin/bash
# Round 3, pass q: step tail on the last range's stream (TDQ_SPLIT_TAIL last | cur).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3q}
mkdir -p $O
TDQ_SPLIT_TAIL=last timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -k "range" -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bench() {  # $1 tail, $2 precision
  TDQ_SPLIT_TAIL=$1 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'tail':'$1','prec':'$2','ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
}
for t in last cur last cur last cur; do bench $t bf16 || exit 1; done
for t in last cur last cur; do bench $t bf16x3 || exit 1; done
(cd /tmp && export TMPDIR=/tmp && TDQ_SPLIT_TAIL=last timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt; tail -20 $O/timeline.txt
