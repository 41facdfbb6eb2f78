#!/bin/bash
# Round 5: fused-step phase stamps of a steady-state tile (the second of each workgroup)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5ts2}
mkdir -p $O
TDQ_FUSED_STEP_DEFINES="-DFZ_TS_TILE=1" timeout -k 10 200 python -u tools/fused_step_timing.py > $O/timing_tile1.txt 2>&1 || { tail -10 $O/timing_tile1.txt; exit 1; }
grep -v Warn $O/timing_tile1.txt | grep -v "model.compile\|amdgpu.ids"
