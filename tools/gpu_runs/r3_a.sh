#!/bin/bash
# Round 3, first GPU pass: full GPU suite (incl. the new RCCL forced-DP and torch.autograd.grad
# tests), the driver-shaped bench with the accuracy half + forced-DP timing, and the L-BFGS stop
# A/B (legacy = the reference's effective |f| < tolX) over the same 3 seeds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-dp > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lbfgs-stop legacy > $O/bench_legacy.json 2> $O/bench_legacy.err || { tail -20 $O/bench_legacy.err; exit 1; }
cat $O/bench_legacy.json
