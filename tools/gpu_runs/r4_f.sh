#!/bin/bash
# Round 4: isolated high-order kernel timing (graph replays) + per-kernel table
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4f}
mkdir -p $O
timeout -k 10 120 python tools/hi_bench.py > $O/hi_bench.json 2> $O/hi_bench.err || { tail -20 $O/hi_bench.err; exit 1; }
cat $O/hi_bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_hi -o run --output-format csv -- python3 $R/tools/hi_bench.py > $R/$O/prof_hi.log 2>&1) || { tail -20 $O/prof_hi.log; exit 1; }
python tools/kernel_stats.py $O/prof_hi/run_kernel_stats.csv --steps 400 > $O/kernel_stats_hi.txt 2>&1
head -8 $O/kernel_stats_hi.txt | cut -c1-150
