export SKIP_TESTS=1
for res in 24 32 48 64; do RES=$res CFGS="split:side_first:1:1" TAG=r5split5_$res bash tools/gpu_runs/r5_split.sh 2>&1 | grep "ac-baseline" | sed "s/^/reserve $res: /" || exit 1; done
