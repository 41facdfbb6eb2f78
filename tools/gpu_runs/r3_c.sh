#!/bin/bash
# Round 3, pass c: GPU suite, the driver-shaped bench (accuracy half + forced-DP), throughput
# repeats, kernel table, and PMC passes over the jet kernels incl. HBM bytes (FETCH/WRITE_SIZE).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3c}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --maxfail=10 --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -2 $O/pytest_gpu.log
grep -E "FAILED|ERROR" $O/pytest_gpu.log | head -20
grep -E "KERNEL_ERR|SOLVER_ERR" $O/pytest_gpu.log > $O/kernel_errors.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-dp > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 300 --warmup 20 --no-l2 > $O/bench_tp$k.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_tp$k.json').read().splitlines()[-1]);print('tp',d['value'],d['ms_per_step'])"
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 57 --top 12 > $O/kernel_stats.txt && head -8 $O/kernel_stats.txt
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 10 --warmup 2 --min-warmup-s 0 --no-l2 --precision ${PREC:-bf16}"
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "jet_|loss_fused|tail_" -d $R/$O/pmc$i --output-format csv -- $B > $R/$O/pmc$i.log 2>&1 || { echo "pmc fail $i"; tail -3 $R/$O/pmc$i.log; exit 1; }
done
cd $R && python tools/pmc_summary.py $O > $O/pmc_summary.txt && head -60 $O/pmc_summary.txt
