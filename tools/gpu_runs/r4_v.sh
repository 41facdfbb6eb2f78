#!/bin/bash
# Round 4: width-256 dK column passes A/B (TDQ_W16_NCP 2 = default library vs 4 = variant build)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4v}
mkdir -p $O
for rep in 1 2; do
  for v in default ncp4; do
    if [ $v = ncp4 ]; then export TDQ_LIB_PATH=$R/tensordiffeq_amd/csrc/build_ncp4/libtdq_hip.so; else unset TDQ_LIB_PATH; fi
    timeout -k 10 300 python bench.py --layers 2,256,256,256,256,1 --steps 100 --warmup 10 --no-l2 > $O/b_${v}_$rep.json 2>> $O/b.err || { tail -20 $O/b.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/b_${v}_$rep.json').read().splitlines()[-1]);print(json.dumps({'variant':'$v','rep':$rep,'ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
  done
done
