#!/bin/bash
# round 6: one-launch step tail (tail1_kernel) A/B + kernel trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6u
mkdir -p $O
for T in 1 0 1 0; do
  TDQ_TAIL1=$T timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b$T.log 2>&1 || exit 1
  echo "TAIL1=$T $(grep -o "\"ms_per_step\": [0-9.]*" $O/b$T.log)"
done
cd /tmp && export TMPDIR=/tmp
TDQ_TAIL1=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --min-warmup-s 0 --no-l2 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
cd $R
python tools/kernel_stats.py $O/kt/run_kernel_stats.csv --steps 221 > $O/kstats_tail1.txt
python tools/timeline.py $O/kt/run_kernel_trace.csv --anchor tail1 --steps 2 > $O/timeline_tail1.txt
head -6 $O/kstats_tail1.txt | cut -c1-110; tail -8 $O/timeline_tail1.txt | cut -c1-100
