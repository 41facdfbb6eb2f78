#!/bin/bash
# Round 4: phase stamps of the high-order kernels (diagnostic build)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4r
timeout -k 10 60 ./tools/hi_stamps > gpurun_out/r4r/stamps.txt 2>&1
rc=$?
tail -14 gpurun_out/r4r/stamps.txt
exit $rc
