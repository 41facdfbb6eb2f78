#!/bin/bash
# GPU iteration: kernel tests, bench, rocprof stats, phase timing
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/it_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/it_pytest.log; [ $rc -eq 0 ] || exit 1
timeout -k 10 300 python bench.py --steps 100 --warmup 10 > gpurun_out/it_bench.log 2>&1 || { tail -20 gpurun_out/it_bench.log; exit 1; }
tail -1 gpurun_out/it_bench.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_it -o run --output-format csv -- python $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-l2 > $GRAFT_REPO_ROOT/gpurun_out/it_prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/it_prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && timeout -k 10 600 python tools/phase_timing.py > gpurun_out/timing.log 2>&1; grep -A40 "== fwd" gpurun_out/timing.log
