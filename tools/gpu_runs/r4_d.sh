#!/bin/bash
# Round 4: high-order kernels as adjoint chain + weight-gradient GEMM pass; forward save flag at compile time.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4d}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_jet_hi.py tests/test_perf_gpu.py -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_hi.log 2>&1
rc=$?
grep -E "HI |BWDR|PERF|passed|failed|FAILED|Error" $O/pytest_hi.log | head -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for p in ac-sa ac-baseline; do
  timeout -k 10 200 python bench.py --problem $p --steps 400 --warmup 20 --no-l2 > $O/b400_$p.json 2>> $O/b400.err || { tail -20 $O/b400.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400_$p.json').read().splitlines()[-1]);print(json.dumps({'problem':'$p','steps':400,'ms':round(d['ms_per_step'],5),'value':d['value'],'spg':d['steps_per_graph']}))" | tee -a $O/b400.jsonl
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_acb -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_acb.log 2>&1) || { tail -20 $O/prof_acb.log; exit 1; }
python tools/kernel_stats.py $O/prof_acb/run_kernel_stats.csv --steps 205 > $O/kernel_stats_acb.txt 2>&1
head -14 $O/kernel_stats_acb.txt | cut -c1-150
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_sa -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_sa.log 2>&1) || { tail -20 $O/prof_sa.log; exit 1; }
python tools/kernel_stats.py $O/prof_sa/run_kernel_stats.csv --steps 205 > $O/kernel_stats_sa.txt 2>&1
head -10 $O/kernel_stats_sa.txt | cut -c1-150
