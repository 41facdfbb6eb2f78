#!/bin/bash
# round 6: PMC of both fused kernels (bf16 Adam step, bf16x3 objective) + kernel tables / timelines
# of the Adam step and the L-BFGS iteration
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6r
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
i=0
for W in step obj; do
  if [ $W = step ]; then B="python3 $R/bench.py --steps 10 --warmup 2 --min-warmup-s 0 --no-l2"; RX="tdq_fused_step$"; else B="python3 $R/tools/obj_bench.py --reps 20"; RX="tdq_fused_step3"; fi
  for G in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES" \
           "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $G --kernel-include-regex "$RX" -d $R/$O/$W/pmc$i --output-format csv -- $B > $R/$O/$W.pmc$i.log 2>&1 || { echo "pmc fail $W $i"; tail -3 $R/$O/$W.pmc$i.log; exit 1; }
  done
  (cd $R && python tools/pmc_summary.py $O/$W > $O/pmc_summary_$W.txt && cat $O/pmc_summary_$W.txt)
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt_step -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 20 --min-warmup-s 0 --no-l2 > $R/$O/kt_step.log 2>&1 || { tail -5 $R/$O/kt_step.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt_lbfgs -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 1000 > $R/$O/kt_lbfgs.log 2>&1 || { tail -5 $R/$O/kt_lbfgs.log; exit 1; }
cd $R
python tools/kernel_stats.py $O/kt_step/run_kernel_stats.csv --steps 221 > $O/kstats_step.txt
python tools/timeline.py $O/kt_step/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline_step.txt
python tools/kernel_stats.py $O/kt_lbfgs/run_kernel_stats.csv --steps 1020 > $O/kstats_lbfgs.txt
python tools/timeline.py $O/kt_lbfgs/run_kernel_trace.csv --anchor lbfgs_dir_step --steps 2 > $O/timeline_lbfgs.txt
head -8 $O/kstats_step.txt | cut -c1-110; tail -12 $O/timeline_step.txt | cut -c1-100; head -10 $O/kstats_lbfgs.txt | cut -c1-110; tail -10 $O/timeline_lbfgs.txt | cut -c1-100
rm -rf $O/step $O/obj
