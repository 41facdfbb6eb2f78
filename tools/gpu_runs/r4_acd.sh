#!/bin/bash
# Round 4: AC-dist 500k kernel table
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4acd}
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --problem ac-dist --steps 20 --warmup 3 --min-warmup-s 0 --no-l2 > $R/$O/bench.log 2>&1) || { tail -20 $O/bench.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 23 > $O/kernel_stats.txt 2>&1
python tools/timeline.py $O/prof/run_kernel_trace.csv --steps 2 > $O/timeline.txt 2>&1
head -12 $O/kernel_stats.txt | cut -c1-150
tail -16 $O/timeline.txt | cut -c1-100
tail -1 $O/bench.log | cut -c1-300
