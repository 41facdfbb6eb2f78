#!/bin/bash
# Round 3, pass ad: debug the 2-rank torchrun rehearsal (peer setup stages logged, short timeouts).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ad}
mkdir -p $O
TDQ_PEER_DEBUG=1 TDQ_PEER_TIMEOUT_S=5 TDQ_DIST_BACKEND=gloo TDQ_PEER_ALLREDUCE=auto timeout -k 10 150 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29521 bench.py --gpus 2 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "rc $?"
grep -v amdgpu.ids $O/bench.err | tail -30
cat $O/bench.json | cut -c1-300
