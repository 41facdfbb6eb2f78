#!/bin/bash
# Round 5: GPU suite + smoke + driver-shape bench + kernel table
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5f1}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rs --maxfail=6 --timeout 300 --timeout-method thread -s > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PERF|ACCURACY|WOLFE|FUSED_STEP_WLO|passed|failed|^FAILED|^ERROR" $O/pytest_gpu.log | cut -c1-250 | tail -30
[ $rc -ne 0 ] && { grep -E "^_____|^E  " $O/pytest_gpu.log | head -30 | cut -c1-250; exit $rc; }
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_driver.json').read().splitlines()[-1]);print('driver', round(d['ms_per_step'],5), round(d['value']/1e6,1), [round(v,5) for v in d.get('l2_full_schedule_seeds')], d.get('time_to_solution_s'))"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python3 $R/bench.py --steps 100 --warmup 10 --no-l2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
cd $R && python tools/kstats_db.py $O/prof/run_results.db --steps 110 > $O/kstats.txt; head -8 $O/kstats.txt
python tools/timeline_db.py $O/prof/run_results.db --steps 2
