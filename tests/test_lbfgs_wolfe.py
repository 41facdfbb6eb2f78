"""Line-search L-BFGS (optimizers/lbfgs_wolfe.py): the ``newton_eager=False`` optimizer.

CPU: convergence on a quadratic and on Rosenbrock, agreement with ``torch.optim.LBFGS``
(strong-Wolfe) on the reached minimum, the stopping rules, and a solver run through
``fit(newton_eager=False)``.  GPU: the graph-replayed run (fused objective) decreases the AC-SA
loss with at most a few trials per iteration and one host read per trial.
"""
import math

import pytest
import torch

from tensordiffeq_amd.optimizers import lbfgs_wolfe


def _quadratic(p=40, seed=0):
    g = torch.Generator().manual_seed(seed)
    Q = torch.randn(p, p, generator=g, dtype=torch.float64)
    A = (Q @ Q.T / p + 0.1 * torch.eye(p, dtype=torch.float64)).float()
    b = torch.randn(p, generator=g).float()
    x = torch.zeros(p)

    def evaluate():
        gr = A @ x - b
        f = 0.5 * x @ (A @ x) - b @ x
        return torch.cat([gr, f.reshape(1)])

    return x, evaluate, torch.linalg.solve(A.double(), b.double())


def _rosenbrock():
    x = torch.tensor([-1.2, 1.0])

    def evaluate():
        a, b = x[0].double(), x[1].double()
        f = (1 - a) ** 2 + 100 * (b - a * a) ** 2
        ga = -2 * (1 - a) - 400 * a * (b - a * a)
        gb = 200 * (b - a * a)
        return torch.stack([ga, gb, f]).float()

    return x, evaluate


def test_quadratic_converges():
    x, ev, xs = _quadratic()
    opt = lbfgs_wolfe.minimize(ev, x, 200)
    err = ((x.double() - xs).norm() / xs.norm()).item()
    assert err < 1e-3, (err, opt.n_iter, opt.reason)
    assert opt.func_eval <= 3 * opt.n_iter + 5       # mostly one trial per iteration
    assert all(b <= a + 1e-6 * abs(a) for a, b in zip(opt.f_hist, opt.f_hist[1:]))   # monotone


def test_rosenbrock_matches_torch_lbfgs():
    x, ev = _rosenbrock()
    opt = lbfgs_wolfe.minimize(ev, x, 200)
    assert torch.allclose(x, torch.tensor([1.0, 1.0]), atol=2e-3), (x, opt.reason, opt.n_iter)
    # torch's strong-Wolfe L-BFGS from the same start reaches the same minimum
    y = torch.nn.Parameter(torch.tensor([-1.2, 1.0]))
    o = torch.optim.LBFGS([y], max_iter=200, history_size=10, line_search_fn="strong_wolfe",
                          tolerance_grad=1e-20, tolerance_change=1e-20)

    def closure():
        o.zero_grad()
        f = (1 - y[0]) ** 2 + 100 * (y[1] - y[0] ** 2) ** 2
        f.backward()
        return f

    o.step(closure)
    assert torch.allclose(x, y.detach(), atol=5e-3)


def test_stops_on_gradient_tolerance():
    x, ev, _ = _quadratic(p=8)
    opt = lbfgs_wolfe.minimize(ev, x, 500, tolerance=1e-3)
    assert opt.reason == "gradient tolerance"
    assert opt.n_iter < 500


def test_max_iterations_and_nan():
    x, ev, _ = _quadratic()
    opt = lbfgs_wolfe.minimize(ev, x, 3)
    assert opt.n_iter == 3 and opt.reason == "max_iterations"
    z = torch.zeros(3)
    opt = lbfgs_wolfe.minimize(lambda: torch.tensor([1.0, 1.0, 1.0, math.nan]), z, 5)
    assert opt.reason == "NaN loss" and opt.n_iter == 0


def test_solver_graph_mode_lbfgs_cpu():
    """fit(newton_eager=False) runs this optimizer and lowers the loss (reference fit.py:83-89)."""
    import tensordiffeq_amd as tdq
    from tests.test_solver import allen_cahn
    torch.manual_seed(0)
    D, bcs, f, kw = allen_cahn(n_f=300)
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 16, 16, 1], f, D, bcs, **kw)
    m.fit(tf_iter=5)
    before = m.min_loss["adam"]
    m.fit(newton_iter=15, newton_eager=False)
    info = m.fit_info["lbfgs"]
    assert info["impl"] == "strong-wolfe"
    assert 1 <= info["n_iter"] <= 15 and info["func_evals"] >= info["n_iter"]
    assert m.min_loss["l-bfgs"] < before


@pytest.mark.gpu
def test_graph_lbfgs_on_gpu():
    """newton_eager=False on the HIP objective (bf16x3, one-launch fused step): the line search
    does not give up early (it used to stop after 27 of 100 iterations with TFP's 1e-6
    approximate-Wolfe tolerance), and the loss it reaches is within the same range as the same
    algorithm on the float64 torch-jet objective from the same start (trajectories of a line
    search from a raw start are not reproducible across objectives: measured 301 -> 37.9 on the
    split-bf16 objective with the precision-aware tolerance 1e-3 vs -> 20.2 in fp64 with 1e-6)."""
    import time

    import bench
    from tensordiffeq_amd.optimizers import lbfgs_wolfe
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    m = bench.build_problem(20000, 1, "hip", dev, False, "bf16", newton_precision="bf16x3")
    m.fit(tf_iter=50)
    before = m.min_loss["adam"]
    x0 = m.u_model.flat.detach().clone()
    t0 = time.perf_counter()
    m.fit(newton_iter=100, newton_eager=False)
    dt = time.perf_counter() - t0
    info = m.fit_info["lbfgs"]
    # the same 100 iterations on the float64 objective (torch jet, no graphs)
    ref = bench.build_problem(20000, 1, "jet", dev, False, "bf16")
    prog = ref.program()
    lam64 = [lam.detach().double() for lam in m.lambdas]
    x = x0.double().clone()

    def evaluate():
        p = x.detach().requires_grad_(True)
        tot, _ = prog.evaluate(p, lam64)
        g, = torch.autograd.grad(tot, [p])
        return torch.cat([g.reshape(-1), tot.detach().reshape(1)])
    opt64 = lbfgs_wolfe.minimize(evaluate, x, 100, use_graph=False)
    print(f"WOLFE_GPU iters {info['n_iter']} evals {info['func_evals']} restarts {info['restarts']} reason "
          f"{info['reason']} eps {info['hz_eps']} loss {before:.4e} -> {m.min_loss['l-bfgs']:.4e} wall {dt:.2f}s; "
          f"fp64 objective: iters {opt64.n_iter} reason {opt64.reason} loss {opt64.min_loss:.4e}")
    assert info["impl"] == "strong-wolfe (device)"
    assert info["n_iter"] == 100, info          # no early stop on a failed line search
    assert opt64.n_iter == 100
    assert m.min_loss["l-bfgs"] < 0.25 * before
    assert info["func_evals"] <= 3 * info["n_iter"] + 5
    assert m.min_loss["l-bfgs"] < 2.5 * opt64.min_loss and opt64.min_loss < 2.5 * m.min_loss["l-bfgs"]
