#!/bin/bash
# Round 5: fused training step (MODE 2) - persistent-kernel tests, fused-step tests, bench A/B,
# kernel times of the default step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5st3}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_fused_step.py -x -v -s -m gpu --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "FUSED_ERR.*N=20000|FUSED_VS.*20000|FUSED_STEP|passed|failed|Error" $O/pytest.log | cut -c1-220 | head -14
if [ $rc -ne 0 ]; then tail -40 $O/pytest.log; exit $rc; fi
for f in 1 0 1; do
  TDQ_FUSED_STEP=$f timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/bench_$f.json 2> $O/bench_$f.err || { tail -20 $O/bench_$f.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$f.json').read().splitlines()[-1]);print('TDQ_FUSED_STEP=$f ms/step',round(d['ms_per_step'],5), d['value'])"
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python $R/bench.py --steps 50 --warmup 10 --no-l2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
cd $R && python tools/kstats_db.py $O/prof/run_results.db --steps 60 > $O/kstats.txt; head -12 $O/kstats.txt
python tools/timeline_db.py $O/prof/run_results.db --steps 2
