#!/bin/bash
# A/B: non-temporal saved-activation stores (csrc/build_nt, -DTDQ_NT_STORES) vs the default library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r11
mkdir -p $O
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/bench_def_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "default $(grep -o '"ms_per_step": [0-9.]*' $O/bench_def_$k.json)"
  TDQ_LIB_PATH=$GRAFT_REPO_ROOT/tensordiffeq_amd/csrc/build_nt/libtdq_hip.so timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/bench_nt_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "nt      $(grep -o '"ms_per_step": [0-9.]*' $O/bench_nt_$k.json)"
done
