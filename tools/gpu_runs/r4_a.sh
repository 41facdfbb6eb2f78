#!/bin/bash
# Round 4, first run on the round-4 tree: GPU suite, smoke(), driver-style bench (throughput + 3-seed accuracy),
# kernel table of the bf16 step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4a}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "ACCURACY|PEER" $O/pytest_gpu.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','steps_per_graph','l2_full_schedule','l2_full_schedule_seeds','time_to_solution_s']})"
for k in 1 2; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b400.json 2>> $O/b400.err || { tail -20 $O/b400.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400.json').read().splitlines()[-1]);print(json.dumps({'steps':400,'ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/b400.jsonl
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 205 > $O/kernel_stats.txt 2>&1
head -12 $O/kernel_stats.txt | cut -c1-150
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt; tail -13 $O/timeline.txt
