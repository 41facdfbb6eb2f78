#!/bin/bash
# round 6: slab pass 2 folded into tail_reduce1 (dp_tail_a: L-BFGS objective, DP step) - smoke, GPU
# suite, L-BFGS ms/iteration (fold on / off), driver-shape bench with accuracy, L-BFGS kernel table
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bq
mkdir -p $O
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log | tail -3
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
for F in 1 0 1; do
  TDQ_TAIL_FOLD=$F timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$F.log 2>&1 || { tail -5 $O/l$F.log; exit 1; }
  echo "fold $F $(tail -1 $O/l$F.log)"
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['value'], 'L2', d['l2_full_schedule'], d['l2_full_schedule_seeds'], d['time_to_solution_s'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 1000 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
cd $R
python tools/kernel_stats.py $O/kt/run_kernel_stats.csv --steps 1020 > $O/kstats_lbfgs.txt
python tools/timeline.py $O/kt/run_kernel_trace.csv --anchor lbfgs_dir_step --steps 2 > $O/timeline_lbfgs.txt
python tools/kdist.py $O/kt/run_kernel_trace.csv tdq_fused_step3 tail_reduce1 slab_reduce2 lbfgs_dots_logic lbfgs_dir_step > $O/kdist_lbfgs.txt
cat $O/kdist_lbfgs.txt; tail -8 $O/timeline_lbfgs.txt | cut -c1-100
rm -rf $O/kt
