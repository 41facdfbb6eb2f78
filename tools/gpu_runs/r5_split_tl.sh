#!/bin/bash
# Round 5: AC-baseline split layout timelines at +1 / +2 fused rounds (CUs left to the jet_hi side chain)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=gpurun_out/${TAG:-r5splittl}
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
export PYTHONPATH=$R
for r in 1 2; do
TDQ_FS_SPLIT_ROUNDS=$r timeout -k 10 200 rocprofv3 --kernel-trace -d $R/$O/p$r -o run -- python3 $R/bench.py --problem ac-baseline --steps 50 --warmup 10 --no-l2 > $R/$O/p$r.log 2>&1 || { tail -5 $R/$O/p$r.log; exit 1; }
(cd $R && python tools/timeline_db.py $O/p$r/run_results.db --steps 1 > $O/timeline_rounds$r.txt; echo "== rounds +$r"; cat $O/timeline_rounds$r.txt; rm -rf $O/p$r)
done
