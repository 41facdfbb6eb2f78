#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 1500 python tools/run_configs.py --which poisson10m burgers helmholtz discovery > gpurun_out/configs.log 2>&1; rc=$?
grep "^{" gpurun_out/configs.log; tail -3 gpurun_out/configs.log; exit $rc
