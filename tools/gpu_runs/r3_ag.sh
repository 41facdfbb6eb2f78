#!/bin/bash
# Round 3, pass ag: kernel table of the width-256 layered step (bf16 and fp32).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ag}
mkdir -p $O
for P in bf16 fp32; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$P -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 3 --min-warmup-s 0 --no-l2 --layers 2,256,256,256,256,1 --precision $P > $R/$O/prof_$P.log 2>&1) || { tail -20 $O/prof_$P.log; exit 1; }
  python tools/kernel_stats.py $O/prof_$P/run_kernel_stats.csv --steps 24 > $O/kernels_$P.txt 2>&1
  head -25 $O/kernels_$P.txt | cut -c1-150
done
