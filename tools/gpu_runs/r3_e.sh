#!/bin/bash
# Round 3, pass e: saved-activation cache-policy A/B (the store probe showed non-temporal 16-B
# stores at 3.8 TB/s vs 5.9 TB/s default-policy for the forward's 217 MB), then the L-BFGS
# iteration with the fused two-launch update vs the five-launch one.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3e}
mkdir -p $O
for rep in 1 2; do
  for V in default ts tsl tl; do
    if [ $V = default ]; then L=""; else L=$R/tensordiffeq_amd/csrc/build_$V/libtdq_hip.so; fi
    TDQ_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/ab_$V.$rep.json 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
    python -c "import json;d=json.loads(open('$O/ab_$V.$rep.json').read().splitlines()[-1]);print('$V',$rep,round(d['ms_per_step'],4))"
  done
done
for V in default ts; do
  if [ $V = default ]; then L=""; else L=$R/tensordiffeq_amd/csrc/build_$V/libtdq_hip.so; fi
  (cd /tmp && export TMPDIR=/tmp && TDQ_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$V -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_$V.log 2>&1) || { tail -20 $O/prof_$V.log; exit 1; }
  python tools/kernel_stats.py $O/prof_$V/run_kernel_stats.csv --steps 57 --top 6 > $O/kernels_$V.txt && head -6 $O/kernels_$V.txt
done
for F in 1 0; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 200 python tools/prof_lbfgs.py --iters 1000 > $O/lbfgs_$F.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  tail -1 $O/lbfgs_$F.json
  (cd /tmp && export TMPDIR=/tmp && TDQ_LBFGS_FUSED=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lb$F -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 300 > $R/$O/prof_lb$F.log 2>&1) || { tail -20 $O/prof_lb$F.log; exit 1; }
  python tools/kernel_stats.py $O/prof_lb$F/run_kernel_stats.csv --steps 340 --top 14 > $O/lbfgs_kernels_$F.txt && head -14 $O/lbfgs_kernels_$F.txt
done
