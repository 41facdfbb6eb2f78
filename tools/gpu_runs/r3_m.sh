#!/bin/bash
# Round 3, pass m: K-step graphs (Adam TDQ_STEP_UNROLL, L-BFGS TDQ_LBFGS_UNROLL) on top of the
# point ranges: GPU suite, bench A/B, L-BFGS A/B, kernel timeline of the split + unrolled step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3m}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep ACCURACY $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bench() {  # $1 unroll, $2 split
  TDQ_STEP_UNROLL=$1 TDQ_SPLIT=$2 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'unroll':'$1','split':'$2','ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/ab.jsonl
}
bench 8 auto && bench 1 auto && bench 8 auto && bench 1 auto && bench 16 auto && bench 8 0 || exit 1
for U in 8 1 8 1; do
  TDQ_LBFGS_UNROLL=$U timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 > $O/tmp.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/tmp.json').read().splitlines()[-1]);d['unroll']='$U';print(json.dumps(d))" | tee -a $O/lbfgs.jsonl
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
tail -1 $O/bench_driver.json | cut -c1-400
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 3 > $O/timeline.txt; tail -30 $O/timeline.txt
