#!/bin/bash
# round 6: the loss's first per-point input prefetched one tile ahead into LDS (GenLoss::pre) - tests + A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ae
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py tests/test_hip_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for NP in 0 1 0 1; do
  TDQ_FS_NO_PRE=$NP timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  TDQ_FS_NO_PRE=$NP timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { tail -5 $O/obj.log; exit 1; }
  echo "NO_PRE=$NP step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)  obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
done
