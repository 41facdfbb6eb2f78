#!/bin/bash
# Round 5: persistent-kernel iteration - tests, fused bench, kernel times, phase stamps
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5it}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_fused_kernels.py -x -q -s --timeout 120 --timeout-method thread > $O/pytest_fused.log 2>&1
rc=$?
grep -E "FUSED_ERR.*N=20000|FUSED_VS.*20000|passed|failed|Error" $O/pytest_fused.log | cut -c1-200 | head -8
if [ $rc -ne 0 ]; then tail -30 $O/pytest_fused.log; exit $rc; fi
TDQ_FUSED=1 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-l2 > $O/bench_fused.json 2> $O/bench_fused.err || { tail -20 $O/bench_fused.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_fused.json').read().splitlines()[-1]);print('fused ms/step',round(d['ms_per_step'],5))"
cd /tmp && export TMPDIR=/tmp && export TDQ_FUSED=1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run -- python $R/bench.py --steps 50 --warmup 10 --no-l2 > $R/$O/prof.log 2>&1 || { tail -20 $R/$O/prof.log; exit 1; }
cd $R && python tools/kstats_db.py $O/prof/run_results.db --steps 60 | head -7
timeout -k 10 300 python tools/fused_timing.py > $O/timing.txt 2>&1 || { tail -5 $O/timing.txt; exit 1; }
tail -28 $O/timing.txt
rm -rf $R/tensordiffeq_amd/csrc/build_timing_fz
