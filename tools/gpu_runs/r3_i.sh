#!/bin/bash
# Round 3, pass i: L-BFGS update rework (grouped dots, wave-0 logic with register rows, direction
# sum split over 4 waves): GPU L-BFGS tests, iteration timing fused / five-launch, kernel tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3i}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_lbfgs_device.py tests/test_accuracy_gpu.py -m gpu -v -s --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -3 $O/pytest.log
grep -E "FAILED|ERROR|ACCURACY" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then exit $rc; fi
for F in 1 0 1 0; do
  TDQ_LBFGS_FUSED=$F timeout -k 10 200 python tools/prof_lbfgs.py --iters 2000 >> $O/lbfgs.jsonl 2>> $O/lbfgs.err || { tail -20 $O/lbfgs.err; exit 1; }
  tail -1 $O/lbfgs.jsonl
done
for F in 1 0; do
  (cd /tmp && export TMPDIR=/tmp && TDQ_LBFGS_FUSED=$F timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_lb$F -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 300 > $R/$O/prof_lb$F.log 2>&1) || { tail -20 $O/prof_lb$F.log; exit 1; }
  python tools/kernel_stats.py $O/prof_lb$F/run_kernel_stats.csv --steps 320 --top 14 | grep -E "lbfgs|pack|slab|total" > $O/lbfgs_kernels_f$F.txt; cat $O/lbfgs_kernels_f$F.txt
done
