#!/bin/bash
# round 6: L-BFGS ms/iteration vs run length (1000 / 3000 / 6000 / 1000 iterations, no profiler)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bv
mkdir -p $O
for N in 1000 3000 6000 1000; do
  timeout -k 10 240 python -u tools/prof_lbfgs.py --iters $N > $O/l$N.log 2>&1 || { tail -5 $O/l$N.log; exit 1; }
  echo "iters $N $(tail -1 $O/l$N.log | grep -o '"ms_per_iter": [0-9.]*')" | tee -a $O/runlength.txt
done
