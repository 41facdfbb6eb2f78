#!/bin/bash
# Round 6: L-BFGS iteration kernel table + timeline with the one-launch bf16x3 objective
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6c
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 5 --warmup 1 --min-warmup-s 0 --acc-seeds 0 --acc-iters 200 --acc-newton 1000 > $R/$O/bench.log 2>&1) || { tail -20 $O/bench.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 1000 > $O/kernel_stats.txt 2>&1
python tools/timeline.py $O/prof/run_kernel_trace.csv --anchor lbfgs_dir_step --steps 3 > $O/timeline.txt 2>&1
head -16 $O/kernel_stats.txt | cut -c1-120
tail -30 $O/timeline.txt | cut -c1-110
tail -1 $O/bench.log | cut -c1-300
