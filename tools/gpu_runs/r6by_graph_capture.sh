#!/bin/bash
# round 6: ROCclr graph packet capture on / off (DEBUG_CLR_GRAPH_PACKET_CAPTURE) - L-BFGS ms/iteration
# and the Adam step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6by
mkdir -p $O
for K in def 0 1 def 0; do
  if [ $K = def ]; then unset DEBUG_CLR_GRAPH_PACKET_CAPTURE; else export DEBUG_CLR_GRAPH_PACKET_CAPTURE=$K; fi
  timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$K.log 2>&1 || { tail -5 $O/l$K.log; exit 1; }
  timeout -k 10 240 python -u bench.py --steps 2000 --warmup 20 --min-warmup-s 0 --no-l2 > $O/b$K.log 2>&1 || { tail -5 $O/b$K.log; exit 1; }
  echo "capture $K lbfgs $(tail -1 $O/l$K.log | grep -o '"ms_per_iter": [0-9.]*') step $(tail -1 $O/b$K.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/capture.txt
done
