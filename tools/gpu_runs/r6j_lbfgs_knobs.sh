#!/bin/bash
# round 6: L-BFGS wall per iteration vs kernels per iteration / iterations per graph
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6j
for v in "TDQ_LBFGS_UNROLL=8" "TDQ_LBFGS_UNROLL=32" "TDQ_LBFGS_UNROLL=8 TDQ_LBFGS_FUSED=0" "TDQ_LBFGS_UNROLL=8 TDQ_LBFGS_IMAGES=0"; do
  env $v timeout -k 10 200 python -u tools/prof_lbfgs.py --iters 3000 2>/dev/null | sed "s/^/$v /" >> gpurun_out/r6j/knobs.txt || exit 1
done
cat gpurun_out/r6j/knobs.txt
