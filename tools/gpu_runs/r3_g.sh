#!/bin/bash
# Round 3, pass g: full GPU suite (incl. the accuracy regressions), the driver-shaped bench
# (accuracy half + forced DP), throughput repeats, kernel table, L-BFGS iteration profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3g}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "KERNEL_ERR|SOLVER_ERR|ACCURACY" $O/pytest_gpu.log > $O/kernel_errors.txt
grep ACCURACY $O/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-dp > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/bench_tp$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_tp$k.json').read().splitlines()[-1]);print('tp',d['value'],d['ms_per_step'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 57 --top 8 > $O/kernel_stats.txt && head -8 $O/kernel_stats.txt
for F in 1 0 1; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 >> $O/lbfgs.jsonl 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  tail -1 $O/lbfgs.jsonl
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lb -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 300 > $R/$O/prof_lb.log 2>&1) || { tail -20 $O/prof_lb.log; exit 1; }
python tools/kernel_stats.py $O/prof_lb/run_kernel_stats.csv --steps 320 --top 12 > $O/lbfgs_kernels.txt && head -12 $O/lbfgs_kernels.txt
