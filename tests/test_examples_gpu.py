"""Every ported example on the MI355X (a few iterations each): the run finishes with finite
numbers and its loss ran on the HIP kernels (every example reports its backend; none uses a
custom network, so "hip" is required everywhere - incl. the 3-D testing.py plan with 7 jet
streams, a "wide" kernel plan)."""
import importlib.util
import math
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")

SMALL = ["--iters", "20", "--newton", "5", "--n-f", "2000", "--device", "cuda", "--quiet"]
CASES = {
    "AC-SA": SMALL, "AC-baseline": SMALL, "burgers-new": SMALL, "burgers-assimilate": SMALL,
    "steady-state": SMALL, "steady-state-poisson": SMALL, "testing": SMALL, "testing1D": SMALL,
    "testing1D-AC": SMALL, "transfer-learn": ["--iters", "20", "--n-f", "2000", "--device", "cuda", "--quiet"],
    "AC-discovery": ["--iters", "20", "--n-data", "4000", "--device", "cuda", "--quiet"],
    "AC-inference": ["--iters", "20", "--device", "cuda", "--quiet"],
    "AC-dist": ["--iters", "20", "--n-f", "2000", "--device", "cuda", "--quiet", "--passes", "2"],
    "AC-dist-new": ["--iters", "20", "--n-f", "2000", "--device", "cuda", "--quiet"],
}


def _load(name):
    if EX not in sys.path:
        sys.path.insert(0, EX)
    spec = importlib.util.spec_from_file_location(name.replace("-", "_") + "_gpu", os.path.join(EX, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("name", sorted(CASES))
def test_example_runs_on_gpu(name, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    res = _load(name).main(CASES[name])
    assert isinstance(res, dict) and res
    for k, v in res.items():
        if isinstance(v, float):
            assert math.isfinite(v), (name, k, v)
    assert res.get("backend") == "hip", (name, res.get("backend"))


# medium schedules (Adam + L-BFGS, the examples' default point counts): the L2 against each
# example's ground truth and the Adam phase's wall time per step (graph capture included, so the
# bound is loose; a fall back to the torch / autograd engines costs 10-100x) - values measured on
# MI355X in profiles/r4y_examples_converge.txt (the Allen-Cahn examples need the full 10k + 10k schedule:
# tests/test_accuracy_gpu.py)
CONVERGE = {
    "burgers-new": (["--iters", "2000", "--newton", "2000"], 5e-3, 0.5),
    "steady-state": (["--iters", "2000", "--newton", "2000"], 6e-2, 0.5),
    "steady-state-poisson": (["--iters", "2000", "--newton", "2000"], 6e-2, 0.5),
    "burgers-assimilate": (["--iters", "2000", "--newton", "2000"], 0.25, 0.5),
}


@pytest.mark.parametrize("name", sorted(CONVERGE))
def test_example_converges(name, monkeypatch):
    argv, l2_max, ms_max = CONVERGE[name]
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    res = _load(name).main(argv + ["--device", "cuda", "--quiet"])
    print(f"EXAMPLE {name} l2 {res['l2_error']:.3e} adam {res['adam_ms_per_step']:.4f} ms/step "
          f"lbfgs {res.get('lbfgs_iters')} backend {res['backend']}")
    assert res["backend"] == "hip"
    assert res["l2_error"] < l2_max, (name, res["l2_error"])
    assert res["adam_ms_per_step"] < ms_max, (name, res["adam_ms_per_step"])
