#!/bin/bash
# Round 3, pass d: store-bandwidth probe (is the jet forward write-bound?), and the L-BFGS
# iteration (bf16x3 objective) with the fused two-launch update vs the five-launch one.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3d}
mkdir -p $O
timeout -k 10 120 ./tools/microbench/store_bw > $O/store_bw.jsonl 2>&1 || { cat $O/store_bw.jsonl; exit 1; }
cat $O/store_bw.jsonl
for F in 1 0; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 200 python tools/prof_lbfgs.py --iters 1000 > $O/lbfgs_$F.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  tail -1 $O/lbfgs_$F.json
  (cd /tmp && export TMPDIR=/tmp && TDQ_LBFGS_FUSED=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lb$F -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 300 > $R/$O/prof_lb$F.log 2>&1) || { tail -20 $O/prof_lb$F.log; exit 1; }
  python tools/kernel_stats.py $O/prof_lb$F/run_kernel_stats.csv --steps 340 --top 14 > $O/lbfgs_kernels_$F.txt && head -14 $O/lbfgs_kernels_$F.txt
done
