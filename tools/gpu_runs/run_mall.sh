#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
python tools/phase_timing.py --npts 12544 > gpurun_out/timing_12k.log 2>&1 || exit 1
python tools/phase_timing.py --lib tensordiffeq_amd/csrc/build_timing/libtdq_hip_timing.so --npts 50000 > gpurun_out/timing_50k.log 2>&1 || exit 1
grep -A30 "== fwd" gpurun_out/timing_12k.log | head -32; echo ======; grep -A30 "== fwd" gpurun_out/timing_50k.log | head -32
