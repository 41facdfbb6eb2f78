#!/bin/bash
# Round 4: high-order kernels with register-prefetched weights; placement in the step graph
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4g}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jet_hi.py -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_hi.log 2>&1
rc=$?
grep -E "HI |passed|failed|FAILED|Error" $O/pytest_hi.log | grep -v "HI fwd" | head -30
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python tools/hi_bench.py > $O/hi_bench.json 2> $O/hi_bench.err || { tail -20 $O/hi_bench.err; exit 1; }
cat $O/hi_bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_hi -o run --output-format csv -- python3 $R/tools/hi_bench.py > $R/$O/prof_hi.log 2>&1) || { tail -20 $O/prof_hi.log; exit 1; }
python tools/kernel_stats.py $O/prof_hi/run_kernel_stats.csv --steps 400 > $O/kernel_stats_hi.txt 2>&1
head -6 $O/kernel_stats_hi.txt | cut -c1-150
for m in 1; do
  TDQ_HI_BRANCH=$m timeout -k 10 200 python -X faulthandler bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b400_acb_$m.json 2>> $O/b400_$m.err || { tail -30 $O/b400_$m.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400_acb_$m.json').read().splitlines()[-1]);print(json.dumps({'mode':'$m','ms':round(d['ms_per_step'],5),'value':d['value']}))"
done
timeout -k 10 200 python -u -m pytest tests/test_perf_gpu.py -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_perf.log 2>&1
grep -E "PERF|passed|failed" $O/pytest_perf.log
timeout -k 10 60 ./tools/hi_stamps > $O/stamps.txt 2>&1 && tail -3 $O/stamps.txt
