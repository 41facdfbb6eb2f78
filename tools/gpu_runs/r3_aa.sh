#!/bin/bash
# Round 3, pass aa: full GPU suite on the current tree (peer all-reduce, layered engine, JIT loss),
# driver-style bench with the full-schedule accuracy, kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3aa}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "ACCURACY|PEER" $O/pytest_gpu.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
tail -1 $O/bench_driver.json | cut -c1-300
python -c "import json;d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','l2_full_schedule','l2_full_schedule_seeds','time_to_solution_s','lbfgs']})"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 205 > $O/kernel_stats.txt 2>&1 || head -5 $O/prof/run_kernel_stats.csv
cat $O/kernel_stats.txt | head -20
