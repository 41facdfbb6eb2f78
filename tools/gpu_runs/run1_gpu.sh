#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/r3_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r3_pytest.log
tail -5 gpurun_out/r3_pytest.log
grep -q "rc=0" gpurun_out/r3_pytest.log || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3_smoke.log 2>&1 || { tail -20 gpurun_out/r3_smoke.log; exit 1; }
tail -2 gpurun_out/r3_smoke.log
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/r3_bench.log 2>&1 || { tail -20 gpurun_out/r3_bench.log; exit 1; }
tail -1 gpurun_out/r3_bench.log
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof3 -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-l2 > $GRAFT_REPO_ROOT/gpurun_out/r3_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/r3_prof.log; exit 1; }
tail -1 $GRAFT_REPO_ROOT/gpurun_out/r3_prof.log
cd $GRAFT_REPO_ROOT && timeout -k 10 300 python bench.py --steps 100 --warmup 10 --precision fp32 > gpurun_out/r3_bench_fp32.log 2>&1; tail -1 gpurun_out/r3_bench_fp32.log
