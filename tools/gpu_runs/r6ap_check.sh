#!/bin/bash
# round 6: split-layout rules - tests + AC-dist / AC-baseline steps
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ap
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_perf_gpu.py tests/test_fused_step.py tests/test_jet_hi.py tests/test_dist_gpu.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|PERF" $O/pytest.log | head -30; exit 1; }
grep -E "PERF|passed" $O/pytest.log | cut -c1-160
timeout -k 10 300 python -u bench.py --problem ac-dist --steps 40 --warmup 5 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
echo "ac-dist $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
