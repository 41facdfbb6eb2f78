#!/bin/bash
# bf16 gradient slabs (precision bf16): GPU tests, kernel errors vs fp64 for both slab types,
# bench A/B (A = bf16 slabs, B = fp32 slabs variant), AC-SA accuracy seeds 0-4 (Adam bf16 +
# L-BFGS bf16x3).  Outputs under gpurun_out/$TDQ_RUN/.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
O=gpurun_out/${TDQ_RUN:-r2slab}
mkdir -p $O
VB=$R/tensordiffeq_amd/csrc/build_${VARIANT:-slab32}/libtdq_hip.so
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_fusion.py tests/test_dist_gpu.py tests/test_lbfgs_device.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python tools/precision_errors.py > $O/precision_errors_a.txt 2>&1 || { tail -20 $O/precision_errors_a.txt; exit 1; }
TDQ_LIB_PATH=$VB timeout -k 10 300 python tools/precision_errors.py > $O/precision_errors_b.txt 2>&1 || { tail -20 $O/precision_errors_b.txt; exit 1; }
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/a_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  TDQ_LIB_PATH=$VB timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/b_$k.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "A(bf16 slabs) $(python -c "import json;print(json.load(open('$O/a_$k.json'))['ms_per_step'])")  B(fp32 slabs) $(python -c "import json;print(json.load(open('$O/b_$k.json'))['ms_per_step'])")"
done
for s in 0 1 2 3 4; do
  timeout -k 10 200 python tools/accuracy_ac_sa.py --prec bf16+bf16x3 --seed $s >> $O/accuracy.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  tail -1 $O/accuracy.jsonl | cut -c1-90
done
