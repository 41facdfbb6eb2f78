#!/bin/bash
# A/B of the layer-0 recompute: kernel tests, bench with and without it, kernel profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r9
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for k in 1 2; do
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/bench_h0_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench_h0_$k.json | cut -c1-200
TDQ_H0_RECOMPUTE=0 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/bench_noh0_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench_noh0_$k.json | cut -c1-200
done
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/bench.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-l2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
echo prof-ok
