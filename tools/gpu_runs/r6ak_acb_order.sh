#!/bin/bash
# round 6: AC-baseline split layout, fused-first default - tests, perf guards, order A/B repeat
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ak
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_perf_gpu.py tests/test_fused_step.py tests/test_jet_hi.py tests/test_fused_kernels.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|PERF" $O/pytest.log | head -30; exit 1; }
grep -E "PERF|passed" $O/pytest.log | cut -c1-160
for rep in 1 2; do
  for ORD in fused_first side_first; do
    TDQ_FS_SPLIT_ORDER=$ORD timeout -k 10 200 python -u bench.py --problem ac-baseline --steps 200 --warmup 20 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    echo "ac-baseline $ORD $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
  done
done
