#!/bin/bash
# Round 5: fused step - steps per graph and timed-step count sweep (host launch vs GPU time)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5unr}
mkdir -p $O
for u in 8 16 32; do
for st in 200 1000; do
  TDQ_STEP_UNROLL=$u timeout -k 10 200 python bench.py --steps $st --warmup 20 --no-l2 > $O/b_${u}_$st.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_${u}_$st.json').read().splitlines()[-1]);print('unroll $u steps $st', round(d['ms_per_step'],5), round(d['value']/1e6,1))"
done
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/b_driver.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b_driver.json').read().splitlines()[-1]);print('driver shape', round(d['ms_per_step'],5), round(d['value']/1e6,1), d.get('l2_full_schedule'), d.get('time_to_solution_s'))"
