#!/bin/bash
# round 6: layered engine with the HIP column sums / weight planes (no torch.sum, no bf16 cast kernels)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_lay_gemm.py tests/test_layered_jet.py -m gpu -q -x -s --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "^E |FAILED|passed|failed|Error|LAY_|KERNEL_ERR" $O/pytest.log | head -30; exit 1; }
grep -E "LAY_|KERNEL_ERR|passed" $O/pytest.log | cut -c1-200
for cfg in "bf16:2,512,512,512,512,1" "bf16x3:2,256,256,256,256,1" "fp32:2,256,256,256,256,1"; do
  pr=${cfg%%:*}; ly=${cfg#*:}
  timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-l2 --precision $pr --layers $ly > $O/b_${pr}.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_${pr}.json').read().splitlines()[-1]);print('$pr $ly', round(d['ms_per_step'],4))"
done
cd /tmp && export TMPDIR=/tmp
for cfg in "bf16:2,512,512,512,512,1" "bf16x3:2,256,256,256,256,1"; do
  pr=${cfg%%:*}; ly=${cfg#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_$pr -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-l2 --precision $pr --layers $ly > $R/$O/prof_$pr.log 2>&1 || { tail -20 $R/$O/prof_$pr.log; exit 1; }
  (cd $R && python tools/kstats_db.py $O/prof_$pr/run_results.db --steps 25 > $O/kstats_$pr.txt && head -16 $O/kstats_$pr.txt | cut -c1-140 && echo "Cijk kernels: $(grep -c Cijk $O/kstats_$pr.txt)  at::native kernels: $(grep -c at::native $O/kstats_$pr.txt)")
done
