#!/bin/bash
# Kernel-time A/B (rocprofv3 stats) + one LDS PMC pass, production library vs csrc/build_$VARIANT.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TDQ_RUN:-r2abp}
mkdir -p $O
VB=$R/tensordiffeq_amd/csrc/build_${VARIANT:?}/libtdq_hip.so
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --no-l2"
for x in a b; do
  if [ $x = b ]; then export TDQ_LIB_PATH=$VB; fi
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --kernel-include-regex "jet_" -d $O/pmc_$x --output-format csv -- $B > $O/pmc_$x.log 2>&1 || { echo "pmc fail $x"; tail -3 $O/pmc_$x.log; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/k_$x -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 > $O/k_$x.log 2>&1 || { tail -20 $O/k_$x.log; exit 1; }
done
unset TDQ_LIB_PATH
cd $R
for x in a b; do
  echo "== $x"; python tools/kernel_stats.py $O/k_$x/run_kernel_stats.csv --steps 55 --top 2 | sed -n 2,3p | cut -c1-60
  mkdir -p $O/s_$x/pmc1 && cp -r $O/pmc_$x/* $O/s_$x/pmc1/ && python tools/pmc_summary.py $O/s_$x | grep -A9 "bwd" | grep -v "^=="
done
