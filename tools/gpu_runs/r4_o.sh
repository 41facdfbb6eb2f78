#!/bin/bash
# Round 4: AC-discovery coefficient recovery - precision / schedule variants (one process each)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R:$R/examples
O=gpurun_out/${TDQ_RUN:-r4o}
mkdir -p $O
run() {
  tag=$1; shift
  timeout -k 10 240 python examples/AC-discovery.py --device cuda "$@" > $O/disc_$tag.log 2>&1 || { tail -20 $O/disc_$tag.log; return 1; }
  echo "$tag: $(grep AC-discovery $O/disc_$tag.log | tail -1 | cut -c1-400)"
}
run default --newton 5000 && \
run fp32 --newton 5000 --precision fp32 && \
run newton15k --newton 15000 && \
run adam20k --iters 20000 --newton 5000 && \
run bf16adam --newton 5000 --precision bf16 --newton-precision bf16x3
