#!/bin/bash
# round 6: shader clock during the L-BFGS update's logic (s_memtime cycles / s_memrealtime ticks,
# TDQ_LBFGS_TS=1), plain and under rocprofv3 --kernel-trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6cc
mkdir -p $O
timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 --ts > $O/plain.log 2>&1 || { tail -5 $O/plain.log; exit 1; }
tail -2 $O/plain.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 3000 --ts > $R/$O/prof.log 2>&1 || { tail -5 $R/$O/prof.log; exit 1; }
cd $R
grep -E "ts_iters|ms_per_iter" $O/prof.log | tail -2
rm -rf $O/kt
timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 --ts > $O/plain2.log 2>&1 || { tail -5 $O/plain2.log; exit 1; }
tail -2 $O/plain2.log
