"""Accuracy regression on MI355X: the reference's own schedules reach the reference-level L2 on
the ground-truth .mat grids (the accuracy half of the BASELINE metric; reference
examples/burgers-new.py:40-41 "train for 10k newton and 10k adam", examples/AC-SA.py:64-88).

Bounds are ~1.5-2.5x the values measured on MI355X (profiles/r3_lbfgs_stop_ab.jsonl, BENCH JSON):
AC-SA seed 0 2.18e-2 (Adam 10k bf16 + L-BFGS 10k bf16x3, legacy stop); Burgers 3.9e-4 in the same
precisions (round 2; all-bf16x3 1.1-1.5e-3).
"""
import importlib.util
import os
import sys

import pytest

pytestmark = pytest.mark.gpu

EX = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "examples")


def _example(name):
    if EX not in sys.path:
        sys.path.insert(0, EX)
    spec = importlib.util.spec_from_file_location(name.replace("-", "_") + "_acc", os.path.join(EX, name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


@pytest.mark.timeout(300)
def test_burgers_reference_schedule_l2():
    """Burgers [2,20x8,1], N_f 10k, Adam 10k (bf16) + L-BFGS 10k (bf16x3) - the reference protocol
    in the bench precisions: L2 < 1e-3."""
    res = _example("burgers-new").main(["--device", "cuda", "--quiet", "--precision", "bf16",
                                        "--newton-precision", "bf16x3"])
    print(f"ACCURACY burgers l2 {res['l2_error']:.3e}")
    assert res["backend"] == "hip"
    assert res["l2_error"] < 1e-3, res


@pytest.mark.timeout(300)
def test_ac_sa_reference_schedule_l2():
    """Allen-Cahn SA-PINN [2,128x4,1], N_f 50k, Adam 10k (bf16) + L-BFGS 10k (bf16x3), seed 0:
    L2 < 3e-2 (SA-PINN paper: 2.1e-2), and L-BFGS ran the reference's full 10k iterations."""
    res = _example("AC-SA").main(["--device", "cuda", "--quiet", "--precision", "bf16",
                                  "--newton-precision", "bf16x3", "--seed", "0"])
    print(f"ACCURACY ac-sa l2 {res['l2_error']:.3e} lbfgs {res['lbfgs_n_iter']} {res['lbfgs_reason']}")
    assert res["backend"] == "hip"
    assert res["l2_error"] < 3e-2, res
    assert res["lbfgs_n_iter"] == 10000
