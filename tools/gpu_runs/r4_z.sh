#!/bin/bash
# Round 4: weight gradient fused into the high-order adjoint chain (REJECTED: A/B 0.2222/0.2233 vs 0.2205/0.2199 ms,
# profiles/r4z_hi_fused_dk_ab_REJECTED.jsonl; the code is not in the tree)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4z}
mkdir -p $O
timeout -k 10 60 ./tools/hi_stamps > $O/stamps.txt 2>&1 || { tail -8 $O/stamps.txt; exit 1; }
tail -6 $O/stamps.txt
TDQ_HI_KF=0 timeout -k 10 200 python -u -m pytest tests/test_jet_hi.py -m gpu -q -s --timeout 120 --timeout-method thread -k fp64 > $O/pytest_kf0.log 2>&1 || { tail -30 $O/pytest_kf0.log; exit 1; }
grep -E "HI grad|HI time|passed" $O/pytest_kf0.log
timeout -k 10 300 python -u -m pytest tests/test_jet_hi.py tests/test_perf_gpu.py -m gpu -q -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "HI grad|PERF|passed|failed|FAILED|Error" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then tail -30 $O/pytest.log; exit $rc; fi
for v in kf kf0 kf kf0; do
  if [ $v = kf0 ]; then export TDQ_HI_KF=0; else unset TDQ_HI_KF; fi
  timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b400_$v.json 2>> $O/b400.err || { tail -20 $O/b400.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b400_$v.json').read().splitlines()[-1]);print(json.dumps({'problem':'ac-baseline','variant':'$v','ms':round(d['ms_per_step'],5),'value':d['value']}))" | tee -a $O/b400.jsonl
done
unset TDQ_HI_KF
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_acb -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_acb.log 2>&1) || { tail -20 $O/prof_acb.log; exit 1; }
python tools/kernel_stats.py $O/prof_acb/run_kernel_stats.csv --steps 205 > $O/kernel_stats_acb.txt 2>&1
python tools/timeline.py $O/prof_acb/run_kernel_trace.csv --steps 2 > $O/timeline_acb.txt 2>&1
tail -18 $O/timeline_acb.txt | cut -c1-100
