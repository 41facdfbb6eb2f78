#!/bin/bash
# round 6: L-BFGS update with the counter-tree hand-off - device L-BFGS tests, ms/iteration of the
# two- and five-launch updates, kernel table of the iteration
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bh
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lbfgs_device.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for F in 1 0 1; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$F.log 2>&1 || { tail -5 $O/l$F.log; exit 1; }
  tail -1 $O/l$F.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 1000 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
cd $R
python tools/kernel_stats.py $O/kt/run_kernel_stats.csv --steps 1020 > $O/kstats_lbfgs.txt
python tools/timeline.py $O/kt/run_kernel_trace.csv --anchor lbfgs_dir_step --steps 2 > $O/timeline_lbfgs.txt
head -10 $O/kstats_lbfgs.txt | cut -c1-110; tail -10 $O/timeline_lbfgs.txt | cut -c1-100
