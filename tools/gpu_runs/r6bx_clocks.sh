#!/bin/bash
# round 6: shader clock / power while the L-BFGS phase and the Adam step run (rocm-smi samples), plain
# and under rocprofv3 --kernel-trace
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/r6bx
mkdir -p $O
sample() {  # $1: tag
  for i in 1 2 3 4 5 6; do
    sleep 2
    timeout 20 rocm-smi --showclocks --showpower 2>/dev/null | grep -E "sclk|Power|power" | head -4 | sed "s/^/$1 /" >> $O/clocks.txt || true
  done
}
timeout -k 10 20 rocm-smi --showclocks --showpower > $O/idle.txt 2>&1 || true
grep -E "sclk|ower" $O/idle.txt | head -4 | sed "s/^/idle /" >> $O/clocks.txt || true
timeout -k 10 300 python -u tools/prof_lbfgs.py --iters 40000 > $O/l.log 2>&1 &
P=$!
sleep 25
sample lbfgs
wait $P || { tail -5 $O/l.log; exit 1; }
tail -1 $O/l.log
timeout -k 10 300 python -u bench.py --steps 60000 --warmup 20 --min-warmup-s 0 --no-l2 > $O/b.log 2>&1 &
P=$!
sleep 25
sample adam
wait $P || { tail -5 $O/b.log; exit 1; }
tail -1 $O/b.log | cut -c1-200
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$O/kt -o run --output-format csv -- python3 $R/tools/prof_lbfgs.py --iters 40000 > $R/$O/kt.log 2>&1 &
P=$!
sleep 30
cd $R
sample lbfgs_prof
wait $P || { tail -5 $O/kt.log; exit 1; }
grep ms_per_iter $O/kt.log | tail -1
rm -rf $O/kt
cat $O/clocks.txt
