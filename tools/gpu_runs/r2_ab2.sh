#!/bin/bash
# A/B of the production library against csrc/build_$VARIANT on one box, both bench precisions:
# GPU kernel tests first, then bench.py bf16 and bf16x3 alternating A, B three times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r2ab2}
mkdir -p $O
VB=$R/tensordiffeq_amd/csrc/build_${VARIANT:?}/libtdq_hip.so
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_fusion.py tests/test_dist_gpu.py tests/test_lbfgs_device.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for p in bf16 bf16x3; do
  for k in 1 2 3; do
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $p > $O/a_${p}_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
    TDQ_LIB_PATH=$VB timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $p > $O/b_${p}_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
    echo "$p A $(python -c "import json;print(json.load(open('$O/a_${p}_$k.json'))['ms_per_step'])")  B($VARIANT) $(python -c "import json;print(json.load(open('$O/b_${p}_$k.json'))['ms_per_step'])")"
  done
done
