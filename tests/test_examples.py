"""Every ported example runs end to end (CPU, a few iterations, tiny point sets).

The reference ships 14 driver scripts and no tests; half of them target a removed API
(§2.4 B23).  Each port exposes ``main(argv) -> dict``; here each one trains for 2 Adam steps (+1
L-BFGS step where the reference runs L-BFGS) and must return finite numbers.
"""
import importlib.util
import math
import os
import sys

import pytest

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")

SMALL = ["--iters", "2", "--newton", "1", "--n-f", "300", "--device", "cpu", "--quiet"]
CASES = {
    "AC-SA": SMALL, "AC-baseline": SMALL, "burgers-new": SMALL, "burgers-assimilate": SMALL,
    "steady-state": SMALL, "steady-state-poisson": SMALL, "testing": SMALL, "testing1D": SMALL,
    "testing1D-AC": SMALL, "transfer-learn": ["--iters", "2", "--n-f", "300", "--device", "cpu", "--quiet"],
    "AC-discovery": ["--iters", "2", "--n-data", "1000", "--device", "cpu", "--quiet"],
    "AC-inference": ["--iters", "2", "--device", "cpu", "--quiet", "--no-sa"],
    "AC-dist": ["--iters", "2", "--n-f", "500", "--device", "cpu", "--quiet", "--passes", "2"],
    "AC-dist-new": ["--iters", "2", "--n-f", "500", "--device", "cpu", "--quiet"],
}


def _load(name):
    if EX not in sys.path:
        sys.path.insert(0, EX)
    spec = importlib.util.spec_from_file_location(name.replace("-", "_"), os.path.join(EX, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.parametrize("name", sorted(CASES))
def test_example_runs(name, monkeypatch):
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    res = _load(name).main(CASES[name])
    assert isinstance(res, dict) and res
    for k, v in res.items():
        if isinstance(v, float):
            assert math.isfinite(v), (name, k, v)


def test_every_reference_example_has_a_port():
    ref = {"AC-SA", "AC-baseline", "AC-discovery", "AC-dist-new", "AC-dist", "AC-inference",
           "burgers-assimilate", "burgers-new", "steady-state-poisson", "steady-state", "testing",
           "testing1D-AC", "testing1D", "transfer-learn"}
    assert ref <= set(CASES) and all(os.path.exists(os.path.join(EX, n + ".py")) for n in ref)
