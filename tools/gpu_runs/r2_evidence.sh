#!/bin/bash
# Round-2 evidence on the committed tree: GPU tests, smoke, flagship bench x3, kernel table,
# AC-SA reference schedule (Adam 10k + device L-BFGS 10k), BASELINE configs.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r2e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 > $O/bench_$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json;d=json.load(open('$O/bench_$k.json'));print('bench',d['value'],d['ms_per_step'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 55 --top 10 > $O/kernel_stats.txt && head -6 $O/kernel_stats.txt
timeout -k 10 400 python -u tools/accuracy_ac_sa.py --iters 10000 --newton 10000 --prec bf16x3 > $O/acc.jsonl 2> $O/acc.err || { tail -20 $O/acc.err; exit 1; }
tail -1 $O/acc.jsonl
timeout -k 10 600 python -u tools/run_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cat $O/configs.jsonl
