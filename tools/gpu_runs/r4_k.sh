#!/bin/bash
# Round 4: per-step timelines of AC-baseline (high-order branch) and AC-SA
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4k}
mkdir -p $O
for p in ac-baseline ac-sa; do
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$p -o run --output-format csv -- python3 $R/bench.py --problem $p --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_$p.log 2>&1) || { tail -20 $O/prof_$p.log; exit 1; }
  python tools/timeline.py $O/prof_$p/run_kernel_trace.csv --steps 2 > $O/timeline_$p.txt 2>&1
  cat $O/timeline_$p.txt | cut -c1-110
done
