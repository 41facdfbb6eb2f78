#!/bin/bash
# Round 3, pass j: do point subsets on separate graph branches fill the jet kernels' wave-slot
# quantisation holes?  (tools/concurrency_probe.py, bf16 and bf16x3)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3j}
mkdir -p $O
timeout -k 10 240 python tools/concurrency_probe.py --prec bf16 > $O/probe_bf16.jsonl 2> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe_bf16.jsonl
timeout -k 10 240 python tools/concurrency_probe.py --prec bf16x3 > $O/probe_bf16x3.jsonl 2>> $O/probe.err || { tail -20 $O/probe.err; exit 1; }
cat $O/probe_bf16x3.jsonl
