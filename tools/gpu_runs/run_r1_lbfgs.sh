#!/bin/bash
# GPU validation: kernel/solver tests, flagship bench (+ backward tile-order A/B), kernel profile,
# full AC-SA schedule with the device L-BFGS.  Every GPU step has its own time limit; stop at the
# first failure.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r7
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 200 python bench.py --steps 200 --warmup 20 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
TDQ_BWD_ORDER=forward timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/bench_fwdorder.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench_fwdorder.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-l2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
echo prof-ok
timeout -k 10 400 python -u tools/accuracy_ac_sa.py --iters 10000 --newton 10000 --prec bf16x3 > $O/acc.jsonl 2> $O/acc.err || { tail -20 $O/acc.err; exit 1; }
cat $O/acc.jsonl
