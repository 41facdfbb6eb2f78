#!/bin/bash
# layered-engine envelope routing (d_in > 8, d_out > 4, > 16 hidden layers, fp32 wide plans)
set -o pipefail
mkdir -p gpurun_out/r3ap
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread -m gpu \
  tests/test_layered_jet.py tests/test_hip_kernels.py > gpurun_out/r3ap/tests.log 2>&1
