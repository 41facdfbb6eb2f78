#!/bin/bash
# round 6: tree validation - smoke, the whole GPU suite, driver-shape bench with the accuracy runs
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6ac
mkdir -p $O
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['value'], 'L2', d['l2_full_schedule'], d['l2_full_schedule_seeds'], d['time_to_solution_s'])"
