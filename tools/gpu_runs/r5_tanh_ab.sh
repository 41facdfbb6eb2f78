#!/bin/bash
# Round 5: fused kernels with the cheap tanh vs the saved-activation kernels' tanh (variant build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5tanh
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_fused_kernels.py -v -s -k saved --timeout 120 --timeout-method thread > $O/cheap.log 2>&1
grep -E "FUSED_VS|passed|failed" $O/cheap.log
TDQ_LIB_PATH=$R/tensordiffeq_amd/csrc/build_acc/libtdq_hip.so timeout -k 10 200 python -u -m pytest tests/test_fused_kernels.py -v -s --timeout 120 --timeout-method thread > $O/acc.log 2>&1
grep -E "FUSED|passed|failed" $O/acc.log
