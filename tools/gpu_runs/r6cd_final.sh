#!/bin/bash
# round 6 final tree (last: shader-clock stamps behind TDQ_LBFGS_TS): smoke, GPU suite, driver-shape bench with
# accuracy, kernel table + timeline of the Adam step, L-BFGS ms/iteration
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6cd
mkdir -p $O
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['value'], 'L2', d['l2_full_schedule'], d['l2_full_schedule_seeds'], d['time_to_solution_s'])"
timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/lbfgs.log 2>&1 || { tail -5 $O/lbfgs.log; exit 1; }
tail -1 $O/lbfgs.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --min-warmup-s 0 --no-l2 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
cd $R
python tools/kernel_stats.py $O/kt/run_kernel_stats.csv --steps 221 > $O/kstats_step.txt
python tools/timeline.py $O/kt/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline_step.txt
head -6 $O/kstats_step.txt | cut -c1-110; tail -6 $O/timeline_step.txt | cut -c1-100
rm -rf $O/kt
