#!/bin/bash
# k-block-outer jet kernels (2 workgroups per CU): kernel tests, bench, kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r2kb}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_hip_kernels.py -x -v --timeout 120 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -40 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
timeout -k 10 200 python bench.py --steps 300 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
cd $R && python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 55 --top 8
