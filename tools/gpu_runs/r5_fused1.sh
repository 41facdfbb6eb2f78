#!/bin/bash
# Round 5: first GPU run of the persistent point-tile kernels (csrc/jet_fused.h)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r5f1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -x -v -s --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1
rc=$?
grep -E "FUSED|passed|failed|Error" $O/pytest_fused.log | head -30
if [ $rc -ne 0 ]; then tail -40 $O/pytest_fused.log; exit $rc; fi
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/bench_fused.json 2> $O/bench_fused.err || { tail -20 $O/bench_fused.err; exit 1; }
tail -1 $O/bench_fused.json
TDQ_FUSED=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/bench_saved.json 2> $O/bench_saved.err || { tail -20 $O/bench_saved.err; exit 1; }
tail -1 $O/bench_saved.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python $R/bench.py --steps 50 --warmup 10 --no-l2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
find $R/$O/prof -name '*kernel_stats.csv' | head -3
