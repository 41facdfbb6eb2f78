#!/bin/bash
# Round 3, pass w: kernel timeline + stats of the split bf16 step with the JIT loss (and the
# interpreter for comparison).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3w}
mkdir -p $O
for J in 1 0; do
  (cd /tmp && export TMPDIR=/tmp && TDQ_LOSS_JIT=$J timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof$J -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof$J.log 2>&1) || { tail -20 $O/prof$J.log; exit 1; }
  grep -i "warn" $O/prof$J.log | head -3
  python tools/timeline.py $O/prof$J/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline$J.txt; tail -20 $O/timeline$J.txt
  grep -i "loss" $O/prof$J/run_kernel_stats.csv | cut -c1-60,200-400
done
