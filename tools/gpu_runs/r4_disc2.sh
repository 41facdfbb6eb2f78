#!/bin/bash
# Round 4: discovery with the log c1 parametrization: GPU test + bench record
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4disc2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_accuracy_gpu.py -k discovery -m gpu -q -s --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "ACCURACY|passed|failed" $O/pytest.log
if [ $rc -ne 0 ]; then tail -20 $O/pytest.log; exit $rc; fi
timeout -k 10 300 python bench.py --problem discovery --steps 20 --warmup 5 --acc-seeds 0 > $O/bench_disc.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench_disc.json | cut -c1-400
