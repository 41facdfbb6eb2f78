#!/bin/bash
# Round 3, pass an: deferred join of the first point range (in-kernel signal wait instead of a graph
# join before the step tail): bitwise tests, bench A/B (TDQ_DEFER_JOIN), timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3an}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_hip_kernels.py tests/test_loss_jit.py tests/test_dist_gpu.py -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bench() {  # $1 defer flag, $2 precision
  TDQ_DEFER_JOIN=$1 timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 --precision $2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'defer':'$1','prec':'$2','ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
}
for r in 1 2 3; do bench 1 bf16 && bench 0 bf16 || exit 1; done
bench 1 bf16x3 && bench 0 bf16x3 || exit 1
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt; tail -24 $O/timeline.txt
