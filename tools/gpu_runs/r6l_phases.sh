#!/bin/bash
# round 6: phase stamps of both fused kernels after the compile-time spec / offsets (steady tile)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6l
TDQ_FUSED_STEP_DEFINES="-DFZ_TS_TILE=1" timeout -k 10 200 python -u tools/fused_step_timing.py --precision bf16 > gpurun_out/r6l/phase_bf16.txt 2>&1 || { tail -20 gpurun_out/r6l/phase_bf16.txt; exit 1; }
TDQ_FUSED_STEP_DEFINES="-DFZ_TS_TILE=1" timeout -k 10 200 python -u tools/fused_step_timing.py --precision bf16x3 > gpurun_out/r6l/phase_bf16x3.txt 2>&1 || { tail -20 gpurun_out/r6l/phase_bf16x3.txt; exit 1; }
grep -v "Warn\|amdgpu.ids" gpurun_out/r6l/phase_bf16.txt gpurun_out/r6l/phase_bf16x3.txt
