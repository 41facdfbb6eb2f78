#!/bin/bash
# Round 3, pass f: full GPU suite (unequal widths, wide plans, fused L-BFGS), then the saved-
# activation cache-policy A/B on the round-2 kernel structure (nt = default, ts, tsl) for bf16
# and bf16x3, then the L-BFGS iteration profile (fused vs five-launch update).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3f}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "KERNEL_ERR|SOLVER_ERR" $O/pytest_gpu.log > $O/kernel_errors.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for P in bf16 bf16x3; do
  for rep in 1 2; do
    for V in default ts tsl; do
      if [ $V = default ]; then L=""; else L=$R/tensordiffeq_amd/csrc/build_$V/libtdq_hip.so; fi
      TDQ_LIB_PATH=$L timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 --precision $P > $O/ab_${P}_$V.$rep.json 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
      python -c "import json;d=json.loads(open('$O/ab_${P}_$V.$rep.json').read().splitlines()[-1]);print('$P $V',$rep,round(d['ms_per_step'],4))"
    done
  done
done
for F in 1 0; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 200 python tools/prof_lbfgs.py --iters 1000 > $O/lbfgs_$F.json 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  tail -1 $O/lbfgs_$F.json
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lb -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 300 > $R/$O/prof_lb.log 2>&1) || { tail -20 $O/prof_lb.log; exit 1; }
python tools/kernel_stats.py $O/prof_lb/run_kernel_stats.csv --steps 320 --top 12 > $O/lbfgs_kernels.txt && head -12 $O/lbfgs_kernels.txt
