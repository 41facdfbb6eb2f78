#!/bin/bash
# Round 4: high-order kernels with the A rows split into bf16 hi/lo once at the LDS store (vs per wave)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r4asplit
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_jet_hi.py tests/test_perf_gpu.py -m gpu -q -s --timeout 240 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "HI grad|HI time|HI fwd.*(0, 0, 0, 0)|PERF|passed|failed" $O/pytest.log | head -20
if [ $rc -ne 0 ]; then tail -30 $O/pytest.log; exit $rc; fi
for rep in 1 2 3; do
for v in new old; do
  if [ $v = old ]; then export TDQ_LIB_PATH=$R/tensordiffeq_amd/csrc/build_old/libtdq_hip.so TDQ_SKIP_HASH_CHECK=1; else unset TDQ_LIB_PATH TDQ_SKIP_HASH_CHECK; fi
  timeout -k 10 200 python bench.py --problem ac-baseline --steps 400 --warmup 20 --no-l2 > $O/b_$v.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/b_$v.json').read().splitlines()[-1]);print(json.dumps({'variant':'$v','rep':$rep,'ms':round(d['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
done
done
unset TDQ_LIB_PATH TDQ_SKIP_HASH_CHECK
timeout -k 10 60 ./tools/hi_stamps > $O/stamps.txt 2>&1 && tail -4 $O/stamps.txt
