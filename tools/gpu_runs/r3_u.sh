#!/bin/bash
# Round 3, pass u: layer-wise jet engine (hidden widths > 128) numerics + wide solver, kernel tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
export PYTHONPATH=$R
O=gpurun_out/${TDQ_RUN:-r3u}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_layered_jet.py -v -s --timeout 300 --timeout-method thread > $O/pytest_layered.log 2>&1
rc=$?
tail -3 $O/pytest_layered.log; grep -E "KERNEL_ERR|FAILED|Error" $O/pytest_layered.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python - > $O/mm_dtype.txt 2>&1 <<'PY'
import torch, time
a = torch.randn(200000, 256, device="cuda").bfloat16(); b = torch.randn(256, 256, device="cuda").bfloat16()
try:
    c = torch.mm(a, b, out_dtype=torch.float32); print("mm out_dtype ok", c.dtype)
except Exception as e:
    print("mm out_dtype failed", e)
af = a.float(); bf = b.float()
for name, fn in [("fp32", lambda: torch.mm(af, bf)), ("bf16", lambda: torch.mm(a, b))]:
    for _ in range(3): fn()
    torch.cuda.synchronize(); t = time.perf_counter()
    for _ in range(20): fn()
    torch.cuda.synchronize(); dt = (time.perf_counter() - t) / 20
    print(name, f"{dt*1e6:.1f} us", f"{2*200000*256*256/dt/1e12:.1f} TF/s")
PY
cat $O/mm_dtype.txt
