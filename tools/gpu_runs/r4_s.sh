#!/bin/bash
# Round 4: AC-baseline, high-order gradient before range 0's backward x larger first ranges (repeat)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4s}
mkdir -p $O
for rep in 1 2; do
  for sp in 0.58 0.62 0.66 0.70; do
    TDQ_HI_PLACE=serial_before TDQ_SPLIT=$sp timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b_${sp}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_${sp}_$rep.json').read().splitlines()[-1]);print(json.dumps({'place':'serial_before','split':'$sp','rep':$rep,'ms':round(d['ms_per_step'],5)}))" | tee -a $O/place.jsonl
  done
done
(cd /tmp && export TMPDIR=/tmp && TDQ_HI_PLACE=serial_before TDQ_SPLIT=0.62 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_acb -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_acb.log 2>&1) || { tail -20 $O/prof_acb.log; exit 1; }
python tools/timeline.py $O/prof_acb/run_kernel_trace.csv --steps 2 > $O/timeline_acb.txt 2>&1
tail -18 $O/timeline_acb.txt | cut -c1-100
