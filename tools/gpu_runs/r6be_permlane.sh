#!/bin/bash
# round 6: col4_sum on v_permlane16/32_swap vs ds_bpermute (-DTDQ_COL4_BPERMUTE): bitwise check + A/B
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6be
mkdir -p $O
timeout -k 10 200 python -u tools/det_check.py > $O/det.log 2>&1 || { tail -5 $O/det.log; exit 1; }
grep distinct $O/det.log | cut -c1-90
timeout -k 10 500 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py tests/test_hip_kernels.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for D in "" "-DTDQ_COL4_BPERMUTE" "" "-DTDQ_COL4_BPERMUTE"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || exit 1
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || exit 1
  echo "[$D] step $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)  obj $(grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1)"
done
