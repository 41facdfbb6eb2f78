#!/bin/bash
# round 6: AC-baseline split layout kernel trace (rounds +0 and +1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6aa
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for RD in 1 0; do
  TDQ_FS_SPLIT_ROUNDS=$RD timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt$RD -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 100 --warmup 20 --min-warmup-s 0 --no-l2 > $R/$O/kt$RD.log 2>&1 || { tail -5 $R/$O/kt$RD.log; exit 1; }
  (cd $R && python tools/kernel_stats.py $O/kt$RD/run_kernel_stats.csv --steps 121 > $O/kstats$RD.txt && python tools/timeline.py $O/kt$RD/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline$RD.txt)
  echo "== rounds +$RD"; head -14 $R/$O/kstats$RD.txt | cut -c1-120; tail -16 $R/$O/timeline$RD.txt | cut -c1-110
done
