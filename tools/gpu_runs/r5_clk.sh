#!/bin/bash
# Round 5: shader clock / power during a sustained fused-step run, with and without rocprofv3
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5clk}
mkdir -p $O
sample() { for i in $(seq 1 40); do rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Power|Socket" | head -4 | tr '\n' ' '; echo; sleep 0.25; done > $1; }
sample $O/smi_plain.txt &
SP=$!
timeout -k 10 200 python bench.py --steps 20000 --warmup 20 --no-l2 > $O/b_plain.json 2>> $O/err.log || { kill $SP; tail -20 $O/err.log; exit 1; }
wait $SP
python -c "import json;d=json.loads(open('$O/b_plain.json').read().splitlines()[-1]);print('plain', round(d['ms_per_step'],5))"
sort $O/smi_plain.txt | uniq -c | sort -rn | head -5
cd /tmp && export TMPDIR=/tmp
(cd $R && sample $O/smi_prof.txt) &
SP=$!
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/prof -o run -- python3 $R/bench.py --steps 20000 --warmup 20 --no-l2 > $R/$O/prof.log 2>&1 || { kill $SP; tail -20 $R/$O/prof.log; exit 1; }
wait $SP
cd $R
grep -o '"ms_per_step": [0-9.]*' $O/prof.log
sort $O/smi_prof.txt | uniq -c | sort -rn | head -5
rm -rf $O/prof
