#!/bin/bash
# points-per-GPU sweep of the AC-SA step (workgroup-quantization check), precision $PREC
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TDQ_RUN:-r2sweep}
mkdir -p $O
for n in ${NPTS:-16384 32768 40960 49152 50000 57344 65536}; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-l2 --npts $n --precision ${PREC:-bf16} > $O/n$n.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.load(open('$O/n$n.json'));print($n, (($n+63)//64), round(d['ms_per_step'],4), round(d['value']/1e6,1))"
done
