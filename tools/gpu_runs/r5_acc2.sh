#!/bin/bash
# Round 5: L2 over seeds 0-5 for the fused step's layer-0 tanh variants; WLO diagnostic; fixed tests
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5acc2}
mkdir -p $O
timeout -k 10 200 python -u tools/wlo_diag.py > $O/wlo_diag.txt 2>&1 || { tail -20 $O/wlo_diag.txt; exit 1; }
cat $O/wlo_diag.txt | grep -v Warning
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_fused_kernels.py tests/test_dist_gpu.py -m gpu -q -x --timeout 300 --timeout-method thread -k "tail_matches_unfused or lbfgs_objective_matches or point_ranges_match or saved_activation or forced_dp" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $O/pytest.log | head -20; exit 1; }
tail -2 $O/pytest.log
for v in "acc_h0:" "cheap_h0:-DFZ_CHEAP_H0=1"; do
  name=${v%%:*}; def=${v#*:}
  TDQ_FUSED_STEP_DEFINES="$def" timeout -k 10 500 python bench.py --steps 20 --warmup 5 --acc-seeds 0 1 2 3 4 5 > $O/$name.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/$name.json').read().splitlines()[-1]);s=d.get('l2_full_schedule_seeds');import statistics as st;print('$name', round(d['ms_per_step'],5), [round(v,5) for v in s], 'median6', round(st.median(s),5), 'median012', round(st.median(s[:3]),5))"
done
