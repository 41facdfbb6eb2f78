#!/bin/bash
# Round 3, pass r: point-range topology (TDQ_SPLIT_MODE chain | fork) x cut.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3r}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py tests/test_dist_gpu.py -k "range" -m gpu -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bench() {  # $1 mode, $2 split, $3 precision
  TDQ_SPLIT_MODE=$1 TDQ_SPLIT=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $3 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'mode':'$1','split':'$2','prec':'$3','ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
}
for r in 1 2; do
  for c in "fork 0.45" "chain 0.45" "chain 0.35" "chain 0.55" "chain 0.25"; do bench $c bf16 || exit 1; done
done
for c in "fork 0.35" "chain 0.35" "chain 0.25" "chain 0.45" "fork 0.35" "chain 0.35"; do bench $c bf16x3 || exit 1; done
for M in chain fork chain fork; do
  TDQ_SPLIT_MODE=$M timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 > $O/tmp.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/tmp.json').read().splitlines()[-1]);d['mode']='$M';print(json.dumps(d))" | tee -a $O/lbfgs.jsonl
done
(cd /tmp && export TMPDIR=/tmp && TDQ_SPLIT_MODE=chain timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt; tail -20 $O/timeline.txt
