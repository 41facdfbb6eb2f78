#!/bin/bash
# Round 4: after removing the float4 tail-Adam variant: fused-tail GPU tests + short bench
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4tail
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py tests/test_perf_gpu.py -m gpu -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-l2 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-200
