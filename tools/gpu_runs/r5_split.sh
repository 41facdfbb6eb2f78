#!/bin/bash
# Round 5: AC-baseline split layout (main-plan outputs fused, high-order outputs on the jet_hi side chain)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5split}
mkdir -p $O
[ -n "$SKIP_TESTS" ] || timeout -k 10 400 python -u -m pytest tests/test_fused_step.py tests/test_jet_hi.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|FUSED_STEP" $O/pytest.log | head -30; exit 1; }
grep -E "FUSED_STEP|passed" $O/pytest.log | cut -c1-250
for cfg in ${CFGS:-split:side_first:1:1 split:side_first:1:0 split:fused_first:1:1 0:side_first:0:0}; do
  m=${cfg%%:*}; rest=${cfg#*:}; ord=${rest%%:*}; rest=${rest#*:}; r=${rest%%:*}; dy=${rest#*:}
  TDQ_FS_DYN_RESERVE=${RES:-32} TDQ_FS_DYNAMIC=$dy TDQ_FS_SPLIT_ROUNDS=$r TDQ_FS_SPLIT_ORDER=$ord TDQ_FUSED_STEP_MIXED=$m timeout -k 10 200 python bench.py --problem ac-baseline --steps 200 --warmup 20 --no-l2 > $O/b_${m}_${ord}_${r}_$dy.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_${m}_${ord}_${r}_$dy.json').read().splitlines()[-1]);print('ac-baseline MIXED=$m $ord rounds+$r dyn=$dy', round(d['ms_per_step'],5))"
done
TDQ_FS_DYNAMIC=1 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/b_acsa_dyn.json 2>> $O/b.err && python -c "import json;d=json.loads(open('$O/b_acsa_dyn.json').read().splitlines()[-1]);print('ac-sa dyn', round(d['ms_per_step'],5))" || exit 1
timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/b_acsa.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b_acsa.json').read().splitlines()[-1]);print('ac-sa', round(d['ms_per_step'],5))"
cd /tmp && export TMPDIR=/tmp
TDQ_FUSED_STEP_MIXED=split timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/bench.py --problem ac-baseline --steps 50 --warmup 10 --no-l2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
cd $R && python tools/timeline_db.py $O/prof/run_results.db --steps 2 > $O/timeline_split.txt; head -30 $O/timeline_split.txt; rm -rf $O/prof
