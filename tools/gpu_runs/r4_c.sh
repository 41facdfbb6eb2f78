#!/bin/bash
# Round 4: fast high-order kernels (1024-thread workgroups, chain jets) + recompute backward check.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4c}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_jet_hi.py tests/test_perf_gpu.py -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_hi.log 2>&1
rc=$?
grep -E "HI |BWDR|PERF|passed|failed|FAILED|Error" $O/pytest_hi.log | head -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for p in ac-sa ac-baseline; do
  timeout -k 10 200 python bench.py --problem $p --steps 400 --warmup 20 --no-l2 > $O/b400_$p.json 2>> $O/b400.err || { tail -20 $O/b400.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400_$p.json').read().splitlines()[-1]);print(json.dumps({'problem':'$p','steps':400,'ms':round(d['ms_per_step'],5),'value':d['value'],'spg':d['steps_per_graph']}))" | tee -a $O/b400.jsonl
done
timeout -k 10 200 python bench.py --problem ac-sa --steps 400 --warmup 20 --no-l2 > $O/b400_ac-sa_bwdr.json 2>> $O/b400.err || { tail -20 $O/b400.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b400_ac-sa_bwdr.json').read().splitlines()[-1]);print(json.dumps({'problem':'ac-sa bwdr','steps':400,'ms':round(d['ms_per_step'],5),'value':d['value'],'spg':d['steps_per_graph']}))" | tee -a $O/b400.jsonl
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_acb -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_acb.log 2>&1) || { tail -20 $O/prof_acb.log; exit 1; }
python tools/kernel_stats.py $O/prof_acb/run_kernel_stats.csv --steps 205 > $O/kernel_stats_acb.txt 2>&1
head -12 $O/kernel_stats_acb.txt | cut -c1-150
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_bwdr -o run --output-format csv -- python3 $R/bench.py --problem ac-sa --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_bwdr.log 2>&1) || { tail -20 $O/prof_bwdr.log; exit 1; }
python tools/kernel_stats.py $O/prof_bwdr/run_kernel_stats.csv --steps 205 > $O/kernel_stats_bwdr.txt 2>&1
head -10 $O/kernel_stats_bwdr.txt | cut -c1-150
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_bwdr.json 2> $O/bench_bwdr.err || { tail -20 $O/bench_bwdr.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_bwdr.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','l2_full_schedule_seeds','time_to_solution_s']})"
timeout -k 10 300 python bench.py --problem ac-baseline --steps 20 --warmup 5 --acc-seeds 0 > $O/bench_acb.json 2> $O/bench_acb.err || { tail -20 $O/bench_acb.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_acb.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','l2_full_schedule_seeds','time_to_solution_s','lbfgs']})"
