#!/bin/bash
# then the GPU kernel tests on the default library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r14
mkdir -p $O
L=$GRAFT_REPO_ROOT/tensordiffeq_amd/csrc
for k in 1 2 3; do
  for v in def prev; do
    if [ $v = def ]; then unset TDQ_LIB_PATH; else export TDQ_LIB_PATH=$L/build_$v/libtdq_hip.so; fi
    timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/bench_${v}_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
    echo "$v $(grep -o '"ms_per_step": [0-9.]*' $O/bench_${v}_$k.json)"
  done
done
unset TDQ_LIB_PATH
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
