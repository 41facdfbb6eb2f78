#!/bin/bash
# in-kernel phase stamps of the jet kernels (library prebuilt with tools/phase_timing.py's build())
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TDQ_RUN:-r2timing}
mkdir -p $O
for p in ${PRECS:-bf16 bf16x3}; do
  timeout -k 10 300 python tools/phase_timing.py --prec $p --lib tensordiffeq_amd/csrc/build_timing/libtdq_hip_timing.so > $O/timing_$p.log 2>&1 || { tail -20 $O/timing_$p.log; exit 1; }
  echo "#### $p"; cat $O/timing_$p.log
done
