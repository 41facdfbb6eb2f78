#!/bin/bash
# round 6: bf16x3 fused objective phase stamps (first tile, steady tile), op build time, bench 3 seeds
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6d
timeout -k 10 200 python -u tools/fused_step_timing.py --precision bf16x3 > gpurun_out/r6d/phase_first.txt 2>&1 || { tail -20 gpurun_out/r6d/phase_first.txt; exit 1; }
cat gpurun_out/r6d/phase_first.txt | grep -v Warn
TDQ_FUSED_STEP_DEFINES="-DFZ_TS_TILE=1" timeout -k 10 200 python -u tools/fused_step_timing.py --precision bf16x3 > gpurun_out/r6d/phase_steady.txt 2>&1 || { tail -20 gpurun_out/r6d/phase_steady.txt; exit 1; }
grep -v Warn gpurun_out/r6d/phase_steady.txt
timeout -k 10 200 python -u -c "
import time, torch, bench
from tensordiffeq_amd.ops import fused_step
for prec in ('bf16', 'bf16x3', 'bf16x3'):
    m = bench.build_problem(50000, 1, 'hip', torch.device('cuda', 0), False, prec)
    t0 = time.perf_counter(); p = m.program(); t1 = time.perf_counter(); fs = fused_step.for_program(p); t2 = time.perf_counter()
    print(prec, 'program', round(t1 - t0, 3), 's, fused op build', round(t2 - t1, 3), 's')
" > gpurun_out/r6d/build_time.txt 2>&1; cat gpurun_out/r6d/build_time.txt | grep -v Warn
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r6d/bench.log 2>&1 || { tail -20 gpurun_out/r6d/bench.log; exit 1; }
tail -1 gpurun_out/r6d/bench.log
