#!/bin/bash
# round 6: L-BFGS logic with R^{-1} kept current, matrix-vector products split over 4 waves, R^{-1} packed into Y^T Y's unused triangle, 1 slot per dots block
# - device L-BFGS tests, ms/iteration, phase stamps, AC-SA accuracy at 3 seeds
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bp
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lbfgs_device.py tests/test_lbfgs_wolfe.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for F in 1 1; do
  timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 > $O/l$F.log 2>&1 || { tail -5 $O/l$F.log; exit 1; }
  tail -1 $O/l$F.log
done
timeout -k 10 240 python -u tools/prof_lbfgs.py --iters 3000 --ts > $O/ts.log 2>&1 || { tail -5 $O/ts.log; exit 1; }
tail -2 $O/ts.log
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-200
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r6bp/bench.log").read().strip().splitlines()[-1])
print("ms", d["ms_per_step"], "L2", d["l2_full_schedule_seeds"], "TTS", d["time_to_solution_s"], [x["n_iter"] for x in d["lbfgs"]])
PY
