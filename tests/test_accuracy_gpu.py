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
    """Allen-Cahn SA-PINN [2,128x4,1], N_f 50k, Adam 10k (bf16) + L-BFGS 10k (bf16x3), seeds 0-2:
    the MEDIAN L2 < 3e-2 (SA-PINN paper: 2.1e-2; measured 2.04-2.54e-2 over seeds 0-2, up to 3.2e-2
    over seeds 3-5 - a single-seed bound would fit one seed rather than the method), every seed
    < 4.5e-2, and L-BFGS ran the reference's full 10k iterations (~7 s per seed)."""
    l2s = []
    for seed in (0, 1, 2):
        res = _example("AC-SA").main(["--device", "cuda", "--quiet", "--precision", "bf16",
                                      "--newton-precision", "bf16x3", "--seed", str(seed)])
        print(f"ACCURACY ac-sa seed {seed} l2 {res['l2_error']:.3e} lbfgs {res['lbfgs_n_iter']} "
              f"{res['lbfgs_reason']}", flush=True)
        assert res["backend"] == "hip"
        assert res["lbfgs_n_iter"] == 10000
        l2s.append(res["l2_error"])
    med = sorted(l2s)[1]
    print(f"ACCURACY ac-sa median l2 {med:.3e}")
    assert med < 3e-2, l2s
    assert max(l2s) < 4.5e-2, l2s


@pytest.mark.timeout(300)
def test_helmholtz_steady_state_reference_schedule_l2():
    """2-D steady state (examples/steady-state.py: u_xx + u_yy + u = q, exact sin(pi x) sin(4 pi y)),
    [2,50x4,1], N_f 10k, Adam 10k + L-BFGS 10k in bf16x3: L2 < 2e-2 (measured 7.9e-3)."""
    res = _example("steady-state").main(["--device", "cuda", "--quiet", "--precision", "bf16x3"])
    print(f"ACCURACY helmholtz l2 {res['l2_error']:.3e}")
    assert res["backend"] == "hip"
    assert res["l2_error"] < 2e-2, res


@pytest.mark.timeout(300)
def test_ac_discovery_recovers_coefficients():
    """AC-discovery (examples/AC-discovery.py) on the full AC.mat field: Adam 10k (the reference
    schedule, SA collocation weights) + 15k L-BFGS over network and coefficients (truth c1 = 1e-4,
    c2 = 5; the reference marks its Adam-only version "doesnt work quite yet", so parity is unpinned),
    with c1 = exp(v) from v = -6 (Raissi et al.'s parametrization of a small positive coefficient;
    the reference's raw c1 = v ends 5-11x too large: 6.1e-4, profiles/r4o_discovery_variants.txt).

    c2 comes out within 1 % on every seed.  c1 with the log parametrization, seeds 0-4: 4.9e-5,
    1.31e-4, 4.2e-5, 4.5e-5, 9.1e-5 (median 51 % off, profiles/r4disc_c1_param_ab.jsonl) - the
    data's x-grid (512 points, spacing 3.9e-3) is coarser than the interface width
    sqrt(c1 / c2) = 4.5e-3, so u_xx at the fronts is weakly pinned by the data; the bound below is
    the measured spread (a factor 3), a regression guard rather than the 30 % target."""
    import time
    t0 = time.perf_counter()
    res = _example("AC-discovery").main(["--device", "cuda", "--quiet", "--newton", "15000", "--c1-param", "log"])
    dt = time.perf_counter() - t0
    print(f"ACCURACY discovery c1 {res['c1']:.4e} ({res['c1_rel_err']:.3f}) c2 {res['c2']:.4f} "
          f"({res['c2_rel_err']:.4f}) wall {dt:.1f} s {res.get('wall_s')} lbfgs {res.get('lbfgs')}")
    assert res["backend"] == "hip"
    assert res["c2_rel_err"] < 0.02, res
    assert 3.3e-5 < res["c1"] < 3e-4, res   # factor 3 around the truth (see docstring)