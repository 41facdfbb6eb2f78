#!/bin/bash
# Round 5: why is the AC-SA step faster under rocprofv3?  graph modes and profiler variants
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TAG:-r5gap}
mkdir -p $O
run() { # name, env..., then bench
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 400 --warmup 20 --no-l2 > $O/b_$name.json 2>> $O/b.err || { tail -5 $O/b.err; return 1; }
  python -c "import json;d=json.loads(open('$O/b_$name.json').read().splitlines()[-1]);print('$name', round(d['ms_per_step'],5))"
}
run default X=1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$O/p1 -o run -- python3 $R/bench.py --steps 400 --warmup 20 --no-l2 > $R/$O/p1.log 2>&1 || { tail -5 $R/$O/p1.log; exit 1; }
grep '^{' $R/$O/p1.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('rocprof kernel-trace', round(d['ms_per_step'],5))"; rm -rf $R/$O/p1
timeout -k 10 200 rocprofv3 --memory-copy-trace -d $R/$O/p2 -o run -- python3 $R/bench.py --steps 400 --warmup 20 --no-l2 > $R/$O/p2.log 2>&1 || { tail -5 $R/$O/p2.log; exit 1; }
grep '^{' $R/$O/p2.log | tail -1 | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('rocprof memcopy-trace only', round(d['ms_per_step'],5))"; rm -rf $R/$O/p2
