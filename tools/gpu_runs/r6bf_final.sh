#!/bin/bash
# round 6 final tree: smoke, GPU suite, driver-shape bench with accuracy, kernel table + timeline, PMC of the step
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6bf
mkdir -p $O
timeout -k 10 400 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
grep smoke $O/smoke.log
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('bench', d['ms_per_step'], d['value'], 'L2', d['l2_full_schedule'], d['l2_full_schedule_seeds'], d['time_to_solution_s'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --min-warmup-s 0 --no-l2 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
i=0
for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
         "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "tdq_fused_step$" -d $R/$O/step/pmc$i --output-format csv -- python3 $R/bench.py --steps 10 --warmup 2 --min-warmup-s 0 --no-l2 > $R/$O/pmc$i.log 2>&1 || { echo "pmc fail $i"; tail -3 $R/$O/pmc$i.log; exit 1; }
done
cd $R
python tools/pmc_summary.py $O/step > $O/pmc_summary_step.txt
python tools/kernel_stats.py $O/kt/run_kernel_stats.csv --steps 221 > $O/kstats_step.txt
python tools/timeline.py $O/kt/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline_step.txt
head -6 $O/kstats_step.txt | cut -c1-110; tail -6 $O/timeline_step.txt | cut -c1-100
rm -rf $O/step $O/kt
