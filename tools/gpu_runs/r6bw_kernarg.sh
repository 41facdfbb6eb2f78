#!/bin/bash
# round 6: kernel arguments in device memory (HIP_FORCE_DEV_KERNARG) - L-BFGS ms/iteration and the
# Adam step, default / 1 / 0
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bw
mkdir -p $O
for K in def 1 0 def 1; do
  if [ $K = def ]; then unset HIP_FORCE_DEV_KERNARG; else export HIP_FORCE_DEV_KERNARG=$K; fi
  timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$K.log 2>&1 || { tail -5 $O/l$K.log; exit 1; }
  timeout -k 10 240 python -u bench.py --steps 2000 --warmup 20 --min-warmup-s 0 --no-l2 > $O/b$K.log 2>&1 || { tail -5 $O/b$K.log; exit 1; }
  echo "kernarg $K lbfgs $(tail -1 $O/l$K.log | grep -o '"ms_per_iter": [0-9.]*') step $(tail -1 $O/b$K.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/kernarg.txt
done
