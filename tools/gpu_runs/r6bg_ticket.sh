#!/bin/bash
# round 6: cost of the last-block hand-off vs grid size (tools/microbench/ticket_cost.hip), and the
# L-BFGS ms/iteration of the two-launch (fused) and five-launch updates
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6bg
mkdir -p $O
timeout -k 10 60 tools/microbench/bin/ticket_cost > $O/ticket.txt 2>&1 || { cat $O/ticket.txt; exit 1; }
cat $O/ticket.txt
for F in 1 0; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$F.log 2>&1 || { tail -5 $O/l$F.log; exit 1; }
  tail -1 $O/l$F.log
done
