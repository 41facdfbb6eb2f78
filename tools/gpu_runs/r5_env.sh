#!/bin/bash
# Round 5: graph-launch runtime knobs vs the fused step's wall-clock step time
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5env}
mkdir -p $O
i=0
for e in "HIP_FORCE_QUEUE_PROFILING=1" "AMD_DIRECT_DISPATCH=0" "AMD_DIRECT_DISPATCH=1" "GPU_FLUSH_ON_EXECUTION=0" "ROC_ACTIVE_WAIT_TIMEOUT=0" "X=2"; do
  i=$((i+1))
  env $e timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/b_$i.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$i.json').read().splitlines()[-1]);print('$e', round(d['ms_per_step'],5))"
done
