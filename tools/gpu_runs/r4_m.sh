#!/bin/bash
# Round 4: width-256 fused kernels (WT = 16, bf16): numerics vs fp64, AC-SA step at width 256, kernel table
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4m}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jet_hi.py -m gpu -v -s --timeout 240 --timeout-method thread > $O/pytest_hi.log 2>&1
rc=$?
grep -E "HI time|HI ac|HI grad|passed|failed|FAILED|Error" $O/pytest_hi.log | head -20
if [ $rc -ne 0 ]; then tail -30 $O/pytest_hi.log; exit $rc; fi
timeout -k 10 120 python tools/hi_bench.py > $O/hi_bench.json 2> $O/hi_bench.err || { tail -20 $O/hi_bench.err; exit 1; }
cat $O/hi_bench.json
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$O/prof_hi -o run --output-format csv -- python3 $R/tools/hi_bench.py > $R/$O/prof_hi.log 2>&1) || { tail -20 $O/prof_hi.log; exit 1; }
python tools/kernel_stats.py $O/prof_hi/run_kernel_stats.csv --steps 400 > $O/kernel_stats_hi.txt 2>&1
head -6 $O/kernel_stats_hi.txt | cut -c1-150
timeout -k 10 300 python -u -m pytest tests/test_hip_kernels.py -m gpu -v -s -k "wide256" --timeout 240 --timeout-method thread > $O/pytest_w256.log 2>&1
rc=$?
grep -E "KERNEL_ERR|passed|failed|FAILED|Error" $O/pytest_w256.log | head -30
if [ $rc -ne 0 ]; then tail -30 $O/pytest_w256.log; exit $rc; fi
timeout -k 10 300 python bench.py --layers 2,256,256,256,256,1 --steps 100 --warmup 10 --no-l2 > $O/b256.json 2> $O/b256.err || { tail -20 $O/b256.err; exit 1; }
python -c "import json;d=json.loads(open('$O/b256.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','value','config']})"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_w256 -o run --output-format csv -- python3 $R/bench.py --layers 2,256,256,256,256,1 --steps 50 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof_w256.log 2>&1) || { tail -20 $O/prof_w256.log; exit 1; }
python tools/kernel_stats.py $O/prof_w256/run_kernel_stats.csv --steps 55 > $O/kernel_stats_w256.txt 2>&1
head -12 $O/kernel_stats_w256.txt | cut -c1-150
timeout -k 10 600 python -u -m pytest tests/test_layered_jet.py tests/test_hip_kernels.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_kern.log 2>&1
tail -3 $O/pytest_kern.log
