#!/bin/bash
# Round 4: bf16x3 MFMA GEMMs in the high-order forward and adjoint chain
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4x}
mkdir -p $O
timeout -k 10 60 ./tools/hi_stamps > $O/stamps.txt 2>&1 || { tail -8 $O/stamps.txt; exit 1; }
tail -6 $O/stamps.txt
timeout -k 10 300 python -u -m pytest tests/test_jet_hi.py tests/test_perf_gpu.py -m gpu -q -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "HI grad|PERF|passed|failed|FAILED|Error" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then tail -30 $O/pytest.log; exit $rc; fi
for p in ac-baseline ac-sa ac-baseline ac-sa; do
  timeout -k 10 200 python bench.py --problem $p --steps 400 --warmup 20 --no-l2 > $O/b400_$p.json 2>> $O/b400.err || { tail -20 $O/b400.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400_$p.json').read().splitlines()[-1]);print(json.dumps({'problem':'$p','ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/b400.jsonl
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_acb -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_acb.log 2>&1) || { tail -20 $O/prof_acb.log; exit 1; }
python tools/kernel_stats.py $O/prof_acb/run_kernel_stats.csv --steps 205 > $O/kernel_stats_acb.txt 2>&1
python tools/timeline.py $O/prof_acb/run_kernel_trace.csv --steps 2 > $O/timeline_acb.txt 2>&1
tail -18 $O/timeline_acb.txt | cut -c1-100
