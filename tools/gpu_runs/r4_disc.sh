#!/bin/bash
# Round 4: AC-discovery c1 parametrization A/B (Adam 10k + L-BFGS 15k, full AC.mat field)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4disc
mkdir -p $O
while read -r tag args; do
  timeout -k 10 200 python -c "
import sys, json, time; sys.path.insert(0, 'examples')
import importlib.util
spec = importlib.util.spec_from_file_location('d', 'examples/AC-discovery.py'); m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
t0 = time.perf_counter()
r = m.main(['--device', 'cuda', '--quiet'] + '$args'.split())
print(json.dumps({'run': '$tag', 'args': '$args', 'backend': r['backend'], 'c1': r['c1'], 'c2': r['c2'], 'c1_rel_err': r['c1_rel_err'], 'c2_rel_err': r['c2_rel_err'], 'wall_s': round(time.perf_counter() - t0, 1), 'phases': r.get('wall_s'), 'lbfgs': r.get('lbfgs')}))
" 2>> $O/err.log | tee -a $O/disc.jsonl || { tail -20 $O/err.log; exit 1; }
done < ${DISC_RUNS:-tools/gpu_runs/r4_disc_runs.txt}
