#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/acc_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/acc_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|assert" gpurun_out/acc_pytest.log | head -60; exit 1; }
timeout -k 10 1200 python tools/accuracy_ac_sa.py --iters 10000 --newton 10000 --prec bf16x3 fp32 > gpurun_out/acc_ac_sa.log 2>&1; rc=$?; tail -3 gpurun_out/acc_ac_sa.log; exit $rc
