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
