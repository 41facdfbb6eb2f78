#!/bin/bash
# round 6: the whole GPU suite + smoke
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6q
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6q/smoke.log 2>&1 || { tail -30 gpurun_out/r6q/smoke.log; exit 1; }
grep smoke gpurun_out/r6q/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6q/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r6q/pytest.log; exit $rc
