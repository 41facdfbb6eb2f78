#!/bin/bash
# round 6: L-BFGS iterations per captured graph (TDQ_LBFGS_UNROLL) and the image scatter vs a pack
# launch (TDQ_LBFGS_IMAGES=0) on the final update kernels - ms per iteration
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bt
mkdir -p $O
for U in 8 16 32 8 16 32; do
  TDQ_LBFGS_UNROLL=$U timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/u$U.log 2>&1 || { tail -5 $O/u$U.log; exit 1; }
  echo "unroll $U $(tail -1 $O/u$U.log | grep -o '"ms_per_iter": [0-9.]*')" | tee -a $O/sweep.txt
done
TDQ_LBFGS_IMAGES=0 timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 > $O/img0.log 2>&1 || { tail -5 $O/img0.log; exit 1; }
echo "images 0 $(tail -1 $O/img0.log | grep -o '"ms_per_iter": [0-9.]*')" | tee -a $O/sweep.txt
