#!/bin/bash
# Round 3, pass e: kernel numerics with the top-layer rebuild (TDQ_RECOMPUTE_TOP), then step A/B:
# default (rebuild + non-temporal saved-activation stores), ts (temporal stores), tsl (temporal
# stores + loads), r0 (no rebuild); then the L-BFGS iteration, fused vs five-launch update.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3e}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py tests/test_lbfgs_device.py tests/test_dist_gpu.py -m gpu -q --maxfail=5 --timeout 300 --timeout-method thread > $O/pytest_kernels.log 2>&1
rc=$?
tail -2 $O/pytest_kernels.log
grep -E "FAILED|ERROR" $O/pytest_kernels.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for rep in 1 2; do
  for V in default ts tsl r0; do
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
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-l2 --force-dp > $O/bench_dp.json 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
tail -1 $O/bench_dp.json
for F in 1 0; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 200 python tools/prof_lbfgs.py --iters 1000 > $O/lbfgs_$F.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  tail -1 $O/lbfgs_$F.json
  (cd /tmp && export TMPDIR=/tmp && TDQ_LBFGS_FUSED=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lb$F -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 300 > $R/$O/prof_lb$F.log 2>&1) || { tail -20 $O/prof_lb$F.log; exit 1; }
  python tools/kernel_stats.py $O/prof_lb$F/run_kernel_stats.csv --steps 340 --top 14 > $O/lbfgs_kernels_$F.txt && head -14 $O/lbfgs_kernels_$F.txt
done
