#!/bin/bash
# Round 4: high-order jet kernels (jet_hi.hip) first, then the whole GPU suite, smoke, the driver
# bench (AC-SA) and the AC-baseline step (order-4 periodic BC on the fused path) + kernel table.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4b}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jet_hi.py -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_hi.log 2>&1
rc=$?
grep -E "HI |passed|failed|FAILED|Error" $O/pytest_hi.log | head -40
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "ACCURACY|SELF_LAUNCH" $O/pytest_gpu.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','steps_per_graph','l2_full_schedule','l2_full_schedule_seeds','time_to_solution_s']})"
for p in ac-sa ac-baseline; do
  timeout -k 10 200 python bench.py --problem $p --steps 400 --warmup 20 --no-l2 > $O/b400_$p.json 2>> $O/b400.err || { tail -20 $O/b400.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400_$p.json').read().splitlines()[-1]);print(json.dumps({'problem':'$p','steps':400,'ms':round(d['ms_per_step'],5),'value':d['value'],'spg':d['steps_per_graph']}))" | tee -a $O/b400.jsonl
done
timeout -k 10 300 python bench.py --problem ac-baseline --steps 20 --warmup 5 --acc-seeds 0 > $O/bench_acb.json 2> $O/bench_acb.err || { tail -20 $O/bench_acb.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_acb.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','l2_full_schedule_seeds','time_to_solution_s','lbfgs']})"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_acb -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_acb.log 2>&1) || { tail -20 $O/prof_acb.log; exit 1; }
python tools/kernel_stats.py $O/prof_acb/run_kernel_stats.csv --steps 205 > $O/kernel_stats_acb.txt 2>&1
head -14 $O/kernel_stats_acb.txt | cut -c1-150
timeout -k 10 400 python bench.py --problem discovery --steps 20 --warmup 5 --acc-seeds 0 > $O/bench_disc.json 2> $O/bench_disc.err || { tail -20 $O/bench_disc.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_disc.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','coefficients','time_to_solution_s','lbfgs']})"
timeout -k 10 300 python bench.py --problem poisson --steps 20 --warmup 3 --no-l2 > $O/bench_poisson.json 2> $O/bench_poisson.err || { tail -20 $O/bench_poisson.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_poisson.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','config']})"
