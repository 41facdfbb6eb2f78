#!/bin/bash
# Full verification of the current tree on one box: GPU test suite, smoke(), bench x3 and a
# rocprofv3 kernel-stats profile of the flagship step.  Outputs under gpurun_out/$TDQ_RUN/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
O=gpurun_out/${TDQ_RUN:-r2verify}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for k in 1 2 3; do
  timeout -k 10 200 python bench.py > $O/bench_$k.json 2>> $O/bench_err.log || { tail -20 $O/bench_err.log; exit 1; }
  cat $O/bench_$k.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 200 --warmup 20 --no-l2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $(find $O/prof -name '*kernel_stats.csv' | head -1) --steps 220 > $O/kernel_stats.txt 2>&1 || true
head -30 $O/kernel_stats.txt
