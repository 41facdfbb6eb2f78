#!/bin/bash
# Round 5: loss-input prefetch A/B on one box (alternating)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5prefab}
mkdir -p $O
for r in 1 2 3; do
for p in 1 0; do
TDQ_FS_PREFETCH=$p timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b_${p}_$r.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
python -c "import json;d=json.loads(open('$O/b_${p}_$r.json').read().splitlines()[-1]);print('prefetch $p', round(d['ms_per_step'],5))"
done
done
