#!/bin/bash
cd $GRAFT_REPO_ROOT
export PYTHONPATH=$GRAFT_REPO_ROOT
timeout -k 10 900 python -m pytest tests/test_hip_kernels.py -q -x > gpurun_out/mixed_pytest.log 2>&1; rc=$?; tail -3 gpurun_out/mixed_pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\|assert" gpurun_out/mixed_pytest.log | head -80; exit 1; }
timeout -k 10 600 python - <<'PY'
import sys, time, importlib.util, torch
sys.path.insert(0, "examples")
spec = importlib.util.spec_from_file_location("acb", "examples/AC-baseline.py"); m = importlib.util.module_from_spec(spec); spec.loader.exec_module(m)
for be in ("auto", "jet"):
    t0 = time.perf_counter(); r = m.main(["--iters", "500", "--newton", "0", "--quiet", "--backend", be]); dt = time.perf_counter() - t0
    print(be, r, f"{dt:.2f}s for 500 Adam steps (incl. compile/capture)", flush=True)
PY
