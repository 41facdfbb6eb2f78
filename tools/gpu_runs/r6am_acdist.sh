#!/bin/bash
# round 6: AC-dist-new program (BASELINE's multi-GPU config) at world 1, 500k points: step time, kernel table, timeline
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
O=gpurun_out/r6am
mkdir -p $O
timeout -k 10 300 python -u bench.py --problem ac-dist --steps 40 --warmup 5 --no-l2 > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench.json').read().splitlines()[-1]);print('ac-dist', d['ms_per_step'], d['value'], d['config'])" | cut -c1-400
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/kt -o run --output-format csv -- python3 $R/bench.py --problem ac-dist --steps 40 --warmup 5 --min-warmup-s 0 --no-l2 > $R/$O/kt.log 2>&1 || { tail -5 $R/$O/kt.log; exit 1; }
cd $R
python tools/kernel_stats.py $O/kt/run_kernel_stats.csv --steps 45 > $O/kstats.txt
python tools/timeline.py $O/kt/run_kernel_trace.csv --anchor tail_adam --steps 2 > $O/timeline.txt
head -12 $O/kstats.txt | cut -c1-120; tail -12 $O/timeline.txt | cut -c1-100
rm -rf $O/kt
