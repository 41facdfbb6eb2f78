#!/bin/bash
# Round 5: AC-baseline step layouts (point ranges vs residual-fused + side chain) + timelines
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5acb}
mkdir -p $O
for m in 0 1; do
  TDQ_FUSED_STEP_MIXED=$m timeout -k 10 200 python bench.py --problem ac-baseline --steps 200 --warmup 20 --no-l2 > $O/b_mixed$m.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_mixed$m.json').read().splitlines()[-1]);print('ac-baseline MIXED=$m', round(d['ms_per_step'],5))"
done
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/b_acsa.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b_acsa.json').read().splitlines()[-1]);print('ac-sa', round(d['ms_per_step'],5))"
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-1 0}; do
TDQ_FUSED_STEP_MIXED=$m timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$O/prof_$m -o run -- python3 $R/bench.py --problem ac-baseline --steps 50 --warmup 10 --no-l2 > $R/$O/prof_$m.log 2>&1 || { tail -20 $R/$O/prof_$m.log; exit 1; }
(cd $R && python tools/timeline_db.py $O/prof_$m/run_results.db --steps 2 > $O/timeline_mixed$m.txt; cat $O/timeline_mixed$m.txt | head -40)
done
