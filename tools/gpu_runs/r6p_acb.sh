#!/bin/bash
# round 6: AC-baseline split layout - extra fused rounds left to the jet_hi side chain (A/B)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r6p
for i in 1 2; do
for R in 0 1 2; do
  TDQ_FS_SPLIT_ROUNDS=$R timeout -k 10 200 python -u bench.py --problem ac-baseline --steps 200 --warmup 20 --no-l2 2>/dev/null | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('acb rounds+$R', d['ms_per_step'])" >> gpurun_out/r6p/acb.txt || exit 1
done
done
cat gpurun_out/r6p/acb.txt
