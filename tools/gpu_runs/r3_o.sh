#!/bin/bash
# Round 3, pass o: fused loss with its global loads hoisted (LFGroup.ld_off / n_ld): GPU suite,
# bench, kernel table and timeline.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3o}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep ACCURACY $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/b.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b.json').read().splitlines()[-1]);print(json.dumps({'ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/bench.jsonl
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt; tail -20 $O/timeline.txt
(cd /tmp && export TMPDIR=/tmp && TDQ_SPLIT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof0 -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof0.log 2>&1) || { tail -20 $O/prof0.log; exit 1; }
python tools/timeline.py $O/prof0/run_kernel_trace.csv --anchor tail_adam --steps 1 > $O/timeline0.txt; tail -10 $O/timeline0.txt
