#!/bin/bash
# round 6: is the L-BFGS loop host-bound?  host enqueue time of the graph replays vs time waiting on
# the GPU (TDQ_LBFGS_HOSTPROF=1), plain and under rocprofv3 --kernel-trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TDQ_LBFGS_HOSTPROF=1
O=gpurun_out/r6ca
mkdir -p $O
for K in a b; do
  timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$K.log 2>&1 || { tail -5 $O/l$K.log; exit 1; }
  tail -2 $O/l$K.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 3000 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
cd $R
grep -E "host_enqueue|ms_per_iter" $O/kt.log | tail -2
rm -rf $O/kt
