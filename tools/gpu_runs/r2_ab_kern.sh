#!/bin/bash
# A/B of jet-kernel time (rocprofv3 kernel stats) between the production library and a variant
# (csrc/build_$VARIANT/libtdq_hip.so); no correctness check (timing variants may be wrong on purpose).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TDQ_RUN:-r2abk}
mkdir -p $O
VB=$R/tensordiffeq_amd/csrc/build_${VARIANT:?}/libtdq_hip.so
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/a$k -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 --precision ${PREC:-bf16x3} > $O/a$k.log 2>&1 || { tail -20 $O/a$k.log; exit 1; }
  TDQ_LIB_PATH=$VB timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/b$k -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 --precision ${PREC:-bf16x3} > $O/b$k.log 2>&1 || { tail -20 $O/b$k.log; exit 1; }
done
cd $R
for x in a1 b1 a2 b2; do echo "== $x"; python tools/kernel_stats.py $O/$x/run_kernel_stats.csv --steps 55 --top 3 | sed -n 2,4p | cut -c1-60; done
