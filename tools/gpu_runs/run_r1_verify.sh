#!/bin/bash
# Re-verification of the rebuilt in-tree library: GPU tests, smoke, flagship bench x2, kernel profile.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r16
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for k in 1 2; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 > $O/bench_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  cat $O/bench_$k.json
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-l2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
echo prof-ok
