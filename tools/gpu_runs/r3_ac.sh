#!/bin/bash
# Round 3, pass ac: rehearsal of the driver's multi-rank bench on the one-GPU box - torchrun with 2
# and 4 ranks sharing cuda:0 over gloo (TDQ_DIST_BACKEND; RCCL refuses ranks sharing a device): peer
# all-reduce setup / self-test / timing / selection, DP step graphs, JSON line.  Per-rank GPU time
# is shared, so the numbers are not a scaling measurement.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ac}
mkdir -p $O
run() {  # $1 ranks, $2 peer mode, $3 port
  TDQ_PEER_TIMEOUT_S=20 TDQ_DIST_BACKEND=gloo TDQ_PEER_ALLREDUCE=$2 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 \
    --master-addr 127.0.0.1 --master-port $3 bench.py --gpus $1 --steps 20 --warmup 5 > $O/bench_n$1_p$2.json 2> $O/bench_n$1_p$2.err || { tail -30 $O/bench_n$1_p$2.err; return 1; }
  python -c "import json;d=json.loads(open('$O/bench_n$1_p$2.json').read().splitlines()[-1]);print(json.dumps({k:d.get(k) for k in ['n_gpus','ms_per_step','value','steps_per_graph','allreduce']}))"
}
run 2 auto 29511 && run 2 0 29512 && run 4 auto 29513 && run 2 1 29514
