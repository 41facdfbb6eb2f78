#!/bin/bash
# Kernel table at 16384 points per GPU (one 256-tile round) to split the per-step intercept.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r19
mkdir -p $O
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-l2 --npts 16384 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
echo prof-ok
