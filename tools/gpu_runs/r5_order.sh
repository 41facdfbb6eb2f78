#!/bin/bash
# Round 5: fused step launch order A/B (side_first vs fused_first) + timelines
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5ord}
mkdir -p $O
for rep in 1 2; do
for ord in side_first fused_first; do
  TDQ_FS_ORDER=$ord timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b_${ord}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_${ord}_$rep.json').read().splitlines()[-1]);print('$ord', round(d['ms_per_step'],5), round(d['value']/1e6,1))"
done
done
cd /tmp && export TMPDIR=/tmp
for ord in side_first fused_first; do
TDQ_FS_ORDER=$ord timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$O/prof_$ord -o run -- python3 $R/bench.py --steps 50 --warmup 10 --no-l2 > $R/$O/prof_$ord.log 2>&1 || { tail -20 $R/$O/prof_$ord.log; exit 1; }
(cd $R && python tools/timeline_db.py $O/prof_$ord/run_results.db --steps 2)
done
