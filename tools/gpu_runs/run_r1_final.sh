#!/bin/bash
# Final round-1 evidence on the committed tree: GPU tests, smoke, flagship bench x3, kernel profile,
# AC-SA reference schedule with the device L-BFGS.
set -o pipefail
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
O=gpurun_out/r15
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 > $O/bench_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  echo "$(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"l2_rel_error_after_steps": [0-9.]*' $O/bench_$k.json | tr '\n' ' ')"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 50 --warmup 5 --no-l2 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
echo prof-ok
timeout -k 10 400 python -u tools/accuracy_ac_sa.py --iters 10000 --newton 10000 --prec bf16x3 > $O/acc.jsonl 2> $O/acc.err || { tail -20 $O/acc.err; exit 1; }
tail -1 $O/acc.jsonl
