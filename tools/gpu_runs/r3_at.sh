#!/bin/bash
# Round 3, pass at: peer all-reduce with 4 ranks sharing the GPU (tests + a 4-rank bench rehearsal;
# the driver's real N=4/8 runs use one GPU per rank).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3at}
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu tests/test_peer_gpu.py > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
[ -n "$SKIP_TESTS" ] || grep -E "PEER|passed|failed" $O/pytest.log
TDQ_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 4 --steps 40 --warmup 5 --no-l2 > $O/bench_n4.json 2> $O/bench_n4.err || { tail -30 $O/bench_n4.err; exit 1; }
tail -1 $O/bench_n4.json
