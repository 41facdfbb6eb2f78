#!/bin/bash
# Round 4: width-256 fused kernels, then the high-order placement sweep
set -o pipefail
cd $GRAFT_REPO_ROOT
TDQ_RUN=r4m ./tools/gpu_runs/r4_m.sh || exit $?
TDQ_RUN=r4l ./tools/gpu_runs/r4_l.sh
