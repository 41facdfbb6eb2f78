#!/bin/bash
# Round 4: high-order gradient split across the two graph branches (TDQ_HI_PLACE=split) vs serial_before
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4split}
mkdir -p $O
timeout -k 10 300 python - > $O/bitwise.log 2>&1 <<'PY' || { tail -20 $O/bitwise.log; exit 1; }
import os, sys, torch
sys.path.insert(0, "tests")
import bench
res = {}
for place in ("serial_before", "split"):
    os.environ["TDQ_HI_PLACE"] = place
    m = bench.PROBLEMS["ac-baseline"]["build"](50000, 1, "hip", torch.device("cuda", 0), False, "bf16")
    m.fit(tf_iter=30)
    res[place] = (m.u_model.flat.detach().clone(), [r["Total Loss"] for r in m.losses])
a, b = res["serial_before"], res["split"]
print("BITWISE params", torch.equal(a[0], b[0]), "losses", a[1] == b[1], a[1][-1], b[1][-1])
assert torch.equal(a[0], b[0]) and a[1] == b[1]
PY
cat $O/bitwise.log | tail -1
for rep in 1 2 3; do
for pl in split serial_before; do
  TDQ_HI_PLACE=$pl timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b_$pl.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$pl.json').read().splitlines()[-1]);print(json.dumps({'place':'$pl','rep':$rep,'ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
done
done
(cd /tmp && export TMPDIR=/tmp && TDQ_HI_PLACE=split timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --problem ac-baseline --steps 100 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/timeline.py $O/prof/run_kernel_trace.csv --steps 2 > $O/timeline.txt 2>&1
tail -17 $O/timeline.txt | cut -c1-100
