#!/bin/bash
# round 6: L-BFGS direction kernels with the pair coefficients staged in LDS, the last block's
# coherent partial loads batched - device L-BFGS tests, ms/iteration, kernel durations, bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6br
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lbfgs_device.py tests/test_lbfgs_wolfe.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for F in 1 0 1; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$F.log 2>&1 || { tail -5 $O/l$F.log; exit 1; }
  echo "fused $F $(tail -1 $O/l$F.log)"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 1000 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
cd $R
python tools/kdist.py $O/kt/run_kernel_trace.csv tdq_fused_step3 tail_reduce1 slab_reduce2 lbfgs_dots_logic lbfgs_dir_step > $O/kdist_lbfgs.txt
cat $O/kdist_lbfgs.txt
rm -rf $O/kt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['value'], 'L2', d['l2_full_schedule'], d['l2_full_schedule_seeds'], d['time_to_solution_s'])"
