#!/bin/bash
# Round 4: high-order forward on the second range's branch ("cross") x cut
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4u}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jet_hi.py -m gpu -q --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for sp in 0.40 0.50 0.56 0.62; do
  TDQ_HI_PLACE=cross TDQ_SPLIT=$sp timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b_$sp.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$sp.json').read().splitlines()[-1]);print(json.dumps({'place':'cross','split':'$sp','ms':round(d['ms_per_step'],5)}))" | tee -a $O/place.jsonl
done
timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b_default.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b_default.json').read().splitlines()[-1]);print(json.dumps({'place':'default','ms':round(d['ms_per_step'],5)}))" | tee -a $O/place.jsonl
(cd /tmp && export TMPDIR=/tmp && TDQ_HI_PLACE=cross TDQ_SPLIT=0.50 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_acb -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_acb.log 2>&1) || { tail -20 $O/prof_acb.log; exit 1; }
python tools/timeline.py $O/prof_acb/run_kernel_trace.csv --steps 2 > $O/timeline_acb.txt 2>&1
tail -17 $O/timeline_acb.txt | cut -c1-100
