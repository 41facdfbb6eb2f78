#!/bin/bash
# Fused L-BFGS objective: kernel tests, then the AC-SA schedule (seed 0) with the fused tail and
# with TDQ_FUSED_TAIL=0, interleaved twice (same trajectory: compare the phase wall times).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
export TMPDIR=/tmp
O=gpurun_out/${TDQ_RUN:-r2lbfgs}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_lbfgs_device.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for k in 1 2; do
  timeout -k 10 200 python tools/accuracy_ac_sa.py --prec bf16+bf16x3 --seed 0 >> $O/fused.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  TDQ_FUSED_TAIL=0 timeout -k 10 200 python tools/accuracy_ac_sa.py --prec bf16+bf16x3 --seed 0 >> $O/unfused.jsonl 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "fused: $(tail -1 $O/fused.jsonl | cut -c1-200)"
  echo "unfused: $(tail -1 $O/unfused.jsonl | cut -c1-200)"
done
