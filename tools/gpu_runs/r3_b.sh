#!/bin/bash
# Round 3, second GPU pass: wide-plan kernels (S x WT > 32) numerics + the whole GPU suite,
# kernel error table, the bench with accuracy + forced-DP (RCCL), and the L-BFGS stop A/B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3b}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -m gpu -v -s --maxfail=20 --timeout 300 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?
tail -3 $O/pytest_kernels.log
grep -E "FAILED|ERROR" $O/pytest_kernels.log | head -30
grep KERNEL_ERR $O/pytest_kernels.log > $O/kernel_errors.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=10 --timeout 300 --timeout-method thread --deselect tests/test_hip_kernels.py > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-dp > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lbfgs-stop legacy > $O/bench_legacy.json 2> $O/bench_legacy.err || { tail -20 $O/bench_legacy.err; exit 1; }
cat $O/bench_legacy.json
