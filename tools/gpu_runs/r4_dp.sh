#!/bin/bash
# Round 4: DP step at world 1 (RCCL in the graph): A/B of the bookkeeping fused into the Adam launch (REJECTED:
# no gain, profiles/r4dp_book_fused_ab_REJECTED.jsonl, tools/patches/dp_book_fused_into_adam_REJECTED.patch) + kernel table + timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r4dp}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_hip_kernels.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -2 $O/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $O/pytest.log | head; exit $rc; fi
for v in 1 0 1 0 1 0; do
  TDQ_DP_BOOK_FUSED=$v timeout -k 10 300 python bench.py --steps 400 --warmup 5 --no-l2 --force-dp > $O/ab_$v.json 2>> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/ab_$v.json').read().splitlines()[-1]);print(json.dumps({'dp_book_fused':$v,'plain_ms':round(d['ms_per_step'],5),'dp_ms':round(d['forced_dp']['ms_per_step'],5)}))" | tee -a $O/ab.jsonl
done
timeout -k 10 300 python bench.py --steps 200 --warmup 5 --no-l2 --force-dp > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print({k:d.get(k) for k in ['ms_per_step','forced_dp']})"
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o run --output-format csv -- python3 $R/bench.py --steps 100 --warmup 5 --min-warmup-s 0 --no-l2 --force-dp > $R/$O/prof.log 2>&1) || { tail -20 $O/prof.log; exit 1; }
python tools/kernel_stats.py $O/prof/run_kernel_stats.csv --steps 210 > $O/kernel_stats.txt 2>&1
python tools/timeline.py $O/prof/run_kernel_trace.csv --steps 3 > $O/timeline.txt 2>&1
head -14 $O/kernel_stats.txt | cut -c1-130
tail -32 $O/timeline.txt | cut -c1-100
