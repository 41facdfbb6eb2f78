#!/bin/bash
# Fused step tail: kernel tests (incl. fused vs unfused bit-equality), then bench A/B on one box
# (A = fused tail, B = TDQ_FUSED_TAIL=0) and a kernel-stats profile of the fused step.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
O=gpurun_out/${TDQ_RUN:-r2tail}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/a_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  TDQ_FUSED_TAIL=0 timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/b_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "A(fused tail) $(python -c "import json;print(json.load(open('$O/a_$k.json'))['ms_per_step'])")  B(unfused) $(python -c "import json;print(json.load(open('$O/b_$k.json'))['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python bench.py --steps 200 --warmup 20 --no-l2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $(find $O/prof -name '*kernel_stats.csv' | head -1) --steps 220 > $O/kernel_stats.txt 2>&1 || true
head -14 $O/kernel_stats.txt
