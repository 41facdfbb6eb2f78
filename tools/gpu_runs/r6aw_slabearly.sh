#!/bin/bash
# round 6: final dK layers stored inside the last tile vs all at the end (-DFZ_SLAB_AT_END)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6aw
mkdir -p $O
timeout -k 10 200 python -u tools/det_check.py bf16 > $O/det.log 2>&1 || { tail -5 $O/det.log; exit 1; }
grep distinct $O/det.log | cut -c1-120
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for D in "" "-DFZ_SLAB_AT_END" "" "-DFZ_SLAB_AT_END"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "[$D] step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
done
