#!/bin/bash
# Kernel-time + bench A/B, production library (a) vs csrc/build_$VARIANT (b), for each precision
# in $PRECS; kernel tests on the production build first.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TDQ_RUN:-r2ab2}
mkdir -p $O
VB=$R/tensordiffeq_amd/csrc/build_${VARIANT:?}/libtdq_hip.so
[ -n "$PREC_ERR" ] && { timeout -k 10 300 python -u tools/precision_errors.py > $O/prec_err.txt 2>&1 || { tail -20 $O/prec_err.txt; exit 1; }; grep "bf16 " $O/prec_err.txt; }
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
for p in ${PRECS:-bf16 bf16x3}; do
  for k in 1 2; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $p > $O/a_${p}_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
    TDQ_LIB_PATH=$VB timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $p > $O/b_${p}_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
    echo "$p A $(python -c "import json;print(round(json.load(open('$O/a_${p}_$k.json'))['ms_per_step'],4))")  B($VARIANT) $(python -c "import json;print(round(json.load(open('$O/b_${p}_$k.json'))['ms_per_step'],4))")"
  done
done
cd /tmp && export TMPDIR=/tmp
for p in ${PRECS:-bf16 bf16x3}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/k_$p -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 --precision $p > $R/$O/k_$p.log 2>&1 || { tail -20 $R/$O/k_$p.log; exit 1; }
  (cd $R && python tools/kernel_stats.py $O/k_$p/run_kernel_stats.csv --steps 55 --top 3 | cut -c1-70)
done
