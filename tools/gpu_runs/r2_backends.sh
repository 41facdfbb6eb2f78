#!/bin/bash
# Same AC-SA training step through every backend on one MI355X: nested torch.autograd (the
# reference's formulation), the torch jet engine, and the HIP kernels (bf16x3 / bf16).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/${TDQ_RUN:-r2be}
mkdir -p $O
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-l2 --backend autograd --precision fp32 > $O/autograd.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --no-l2 --backend jet --precision fp32 > $O/jet.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-l2 --precision fp32 > $O/hip_fp32.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 20 --no-l2 --precision bf16x3 > $O/hip_bf16x3.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 20 > $O/hip_bf16.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
for f in autograd jet hip_fp32 hip_bf16x3 hip_bf16; do python -c "import json;d=json.load(open('$O/$f.json'));print('$f', d['config']['backend'], round(d['ms_per_step'],4), 'ms', round(d['value']/1e6,2), 'M pts/s')"; done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/k -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --no-l2 > $R/$O/k.log 2>&1 || { tail -20 $R/$O/k.log; exit 1; }
cd $R && python tools/kernel_stats.py $O/k/run_kernel_stats.csv --steps 55 --top 10 | cut -c1-100
