#!/bin/bash
# Round 4 final (a): whole GPU suite, smoke, driver-shape bench with accuracy, AC-SA kernel table + timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4fa}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "ACCURACY|SELF_LAUNCH|PERF" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','steps_per_graph','l2_full_schedule','l2_full_schedule_seeds','time_to_solution_s']})"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_sa -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_sa.log 2>&1) || { tail -20 $O/prof_sa.log; exit 1; }
python tools/kernel_stats.py $O/prof_sa/run_kernel_stats.csv --steps 205 > $O/kernel_stats_sa.txt 2>&1
python tools/timeline.py $O/prof_sa/run_kernel_trace.csv --steps 2 > $O/timeline_sa.txt 2>&1
head -8 $O/kernel_stats_sa.txt | cut -c1-130
