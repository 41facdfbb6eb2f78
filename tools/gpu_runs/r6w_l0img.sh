#!/bin/bash
# round 6: layer-0 adjoint reading h_0 from the slot-0 image (hi + lo value, bf16 derivative streams)
# instead of recomputing layer 0: fp64 oracle, determinism, step A/B, accuracy
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6w
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -m gpu -q -x -s --timeout 300 --timeout-method thread -k "bf16 and not bf16x3" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|FUSED_FP64" $O/pytest.log | head -30; exit 1; }
grep -E "FUSED_FP64|passed" $O/pytest.log | cut -c1-200
for D in "" "-DFZ_L0_RECOMPUTE" "" "-DFZ_L0_RECOMPUTE"; do
  TDQ_FUSED_STEP_DEFINES="$D" timeout -k 10 200 python -u bench.py --steps 2000 --warmup 200 --no-l2 > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
  echo "[$D] $(grep -o "\"ms_per_step\": [0-9.]*" $O/b.log)"
done
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench_l2.json 2> $O/bench_l2.err || { tail -5 $O/bench_l2.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_l2.json').read().splitlines()[-1]);print('driver shape', d['ms_per_step'], d['value'], 'L2', d['l2_full_schedule'], d['l2_full_schedule_seeds'], d['time_to_solution_s'])"
