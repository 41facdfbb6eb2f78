#!/bin/bash
# Round 5 baseline: GPU suite, driver-shape bench, kernel table of the AC-SA step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5base
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -5 $O/pytest.log
if [ $rc -ne 0 ]; then tail -40 $O/pytest.log; exit $rc; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python $R/bench.py --steps 200 --warmup 20 --no-l2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
find $R/$O/prof -name '*kernel_stats.csv' | head -3
