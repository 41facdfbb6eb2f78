#!/bin/bash
# Round 4: AC-baseline range cut x high-order placement (serial), after the reduction split
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4q}
mkdir -p $O
timeout -k 10 60 ./tools/hi_stamps > $O/stamps.txt 2>&1 || { tail -8 $O/stamps.txt; exit 1; }
tail -8 $O/stamps.txt
for pl in serial_after serial_before; do
  for sp in 0.30 0.45 0.55 0.62; do
    TDQ_HI_PLACE=$pl TDQ_SPLIT=$sp timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b_${pl}_$sp.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_${pl}_$sp.json').read().splitlines()[-1]);print(json.dumps({'place':'$pl','split':'$sp','ms':round(d['ms_per_step'],5)}))" | tee -a $O/place.jsonl
  done
done
