#!/bin/bash
# Round 3, pass ab: 16-byte bf16 slab reduction (stride rounded to 8): bitwise tail tests, bench A/B
# against the previous commit's library (TDQ_LIB_PATH, hash check off for the variant).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3ab}
mkdir -p $O
VB=$R/tensordiffeq_amd/csrc/build_prev/libtdq_hip.so
timeout -k 10 600 python -u -m pytest tests/test_hip_kernels.py -k "tail or range or lbfgs" -q --timeout 300 --timeout-method thread > $O/pytest_k.log 2>&1 || { tail -30 $O/pytest_k.log; exit 1; }
tail -1 $O/pytest_k.log
for k in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/a.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  TDQ_SKIP_HASH_CHECK=1 TDQ_LIB_PATH=$VB timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b.json 2>> $O/err.log || { tail -20 $O/err.log; exit 1; }
  echo "{\"new\": $(python -c "import json;print(json.loads(open('$O/a.json').read().splitlines()[-1])['ms_per_step'])"), \"prev\": $(python -c "import json;print(json.loads(open('$O/b.json').read().splitlines()[-1])['ms_per_step'])")}" | tee -a $O/ab.jsonl
done
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 200 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
grep -E "tail_|loss" $O/prof/run_kernel_stats.csv | cut -c1-40,150-260
