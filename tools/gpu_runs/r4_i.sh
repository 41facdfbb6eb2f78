#!/bin/bash
# Round 4: phase timestamps of the high-order forward kernel (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4i
timeout -k 10 60 ./tools/hi_stamps > gpurun_out/r4i/stamps.txt 2>&1
rc=$?
tail -12 gpurun_out/r4i/stamps.txt
exit $rc
