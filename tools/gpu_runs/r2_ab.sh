#!/bin/bash
# A/B of the production library against a variant build (csrc/build_$VARIANT/libtdq_hip.so) on one
# box: kernel tests on the production build, then bench.py alternating A, B, A, B, A, B.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r2ab}
mkdir -p $O
VB=$R/tensordiffeq_amd/csrc/build_${VARIANT:?}/libtdq_hip.so
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/a_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  TDQ_LIB_PATH=$VB timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/b_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "A $(python -c "import json;print(json.load(open('$O/a_$k.json'))['ms_per_step'])")  B($VARIANT) $(python -c "import json;print(json.load(open('$O/b_$k.json'))['ms_per_step'])")"
done
