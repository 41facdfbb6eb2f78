#!/bin/bash
# Round 3, pass h: GPU suite (Burgers accuracy now bf16 Adam + bf16x3 L-BFGS), driver-shaped
# bench, L-BFGS fused vs five-launch update: wall time and kernel tables for both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3h}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "KERNEL_ERR|SOLVER_ERR|ACCURACY" $O/pytest_gpu.log > $O/kernel_errors.txt
grep ACCURACY $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
for F in 1 0 1 0; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 >> $O/lbfgs.jsonl 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  tail -1 $O/lbfgs.jsonl
done
for F in 1 0; do
  (cd /tmp && export TMPDIR=/tmp && TDQ_LBFGS_FUSED=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lb$F -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 300 > $R/$O/prof_lb$F.log 2>&1) || { tail -20 $O/prof_lb$F.log; exit 1; }
  python tools/kernel_stats.py $O/prof_lb$F/run_kernel_stats.csv --steps 320 --top 14 > $O/lbfgs_kernels_f$F.txt && head -14 $O/lbfgs_kernels_f$F.txt
done
