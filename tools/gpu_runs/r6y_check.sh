#!/bin/bash
# round 6: tree check after the early x fetch: determinism, fp64 tests, step time, obj time
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 200 python -u tools/det_check.py > $O/det.log 2>&1 || { tail -5 $O/det.log; exit 1; }
grep distinct $O/det.log | cut -c1-150
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py tests/test_fused_step.py -m gpu -q -x --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error" $O/pytest.log | head -30; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "2000 steps: $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
done
timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-l2 > $O/b20.log 2>&1 || { tail -5 $O/b20.log; exit 1; }
echo "20 steps: $(grep -o "\"ms_per_step\": [0-9.]*" $O/b20.log)"
timeout -k 10 200 python -u tools/obj_bench.py --reps 300 > $O/obj.log 2>&1 || { tail -5 $O/obj.log; exit 1; }
grep -o "\"us_per_eval\": [0-9.]*" $O/obj.log | tail -1
