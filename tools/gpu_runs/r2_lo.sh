#!/bin/bash
# bf16-activation mode + buffer-resource addressing: numerics of every precision, kernel tests,
# then bench A/B on one box: HEAD snapshot (ab_prev/) vs working tree bf16x3 vs working tree bf16.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TDQ_RUN:-r2lo}
mkdir -p $O
[ -n "$PREC_ERR" ] && { timeout -k 10 300 python -u tools/precision_errors.py > $O/prec_err.txt 2>&1 || exit 1; }

timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
for k in 1 2 3; do
  (cd ab_prev && timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2) > $O/prev_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/x3_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision bf16 > $O/b16_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "prev $(python -c "import json;print(json.load(open('$O/prev_$k.json'))['ms_per_step'])")  x3 $(python -c "import json;print(json.load(open('$O/x3_$k.json'))['ms_per_step'])")  bf16 $(python -c "import json;print(json.load(open('$O/b16_$k.json'))['ms_per_step'])")"
done
cd /tmp && export TMPDIR=/tmp
for p in bf16x3 bf16; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/k_$p -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 --precision $p > $R/$O/k_$p.log 2>&1 || { tail -20 $R/$O/k_$p.log; exit 1; }
done
cd $R
for p in bf16x3 bf16; do echo "== $p"; python tools/kernel_stats.py $O/k_$p/run_kernel_stats.csv --steps 55 --top 4; done
