#!/bin/bash
# BASELINE.json configurations on the final round-1 build (device L-BFGS, v9 kernels).
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r16
mkdir -p $O
for c in poisson10m burgers helmholtz discovery; do
  timeout -k 10 400 python -u tools/run_configs.py --which $c > $O/cfg_$c.log 2>&1 || { tail -20 $O/cfg_$c.log; exit 1; }
  grep "^{" $O/cfg_$c.log | cut -c1-400
done
