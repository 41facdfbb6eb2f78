#!/bin/bash
# Round 4: split timing of the weight-gradient pass of the high-order kernels
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4h}
mkdir -p $O
for p in 0 1 2; do
  (cd /tmp && export TMPDIR=/tmp && TDQ_HI_WGRAD_PART=$p timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_hi$p -o run --output-format csv -- python3 $R/tools/hi_bench.py > $R/$O/prof_hi$p.log 2>&1) || { tail -20 $O/prof_hi$p.log; exit 1; }
  python tools/kernel_stats.py $O/prof_hi$p/run_kernel_stats.csv --steps 400 > $O/kernel_stats_hi$p.txt 2>&1
  echo "part $p"; head -5 $O/kernel_stats_hi$p.txt | cut -c1-120
done
