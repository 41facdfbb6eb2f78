#!/bin/bash
# Quick check of the current tree: the given test files ($TESTS), bench x3, and a rocprofv3
# kernel table of the flagship step.  Outputs under gpurun_out/$TDQ_RUN/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
O=gpurun_out/${TDQ_RUN:-r2quick}
mkdir -p $O
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_hip_kernels.py} -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/bench_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "bench $(python -c "import json;print(json.load(open('$O/bench_$k.json'))['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 200 --warmup 20 --no-l2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $(find $O/prof -name '*kernel_stats.csv' | head -1) --steps 220 > $O/kernel_stats.txt 2>&1 || true
head -8 $O/kernel_stats.txt
