"""CollocationSolverND / DiscoveryModel end-to-end on CPU (jet and autograd backends)."""
import math
import os

import numpy as np
import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import (DomainND, IC, FunctionDirichletBC, FunctionNeumannBC, dirichletBC,
                                         periodicBC)


def burgers(n_f=500, seed=0):
    tdq.set_seed(seed)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 64)
    D.add("t", [0.0, 1.0], 20)
    D.generate_collocation_points(n_f)
    init = IC(D, [lambda x: -np.sin(x * math.pi)], var=[["x"]])
    bcs = [init, dirichletBC(D, val=0.0, var="x", target="upper"), dirichletBC(D, val=0.0, var="x", target="lower")]

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t + u * u_x - (0.01 / math.pi) * u_xx
    return D, bcs, f_model


def allen_cahn(n_f=400, seed=0, sa=True):
    tdq.set_seed(seed)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 64)
    D.add("t", [0.0, 1.0], 21)
    D.generate_collocation_points(n_f)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return u, tdq.grad(u, x)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_xx = tdq.grad(tdq.grad(u, x), x)
        return tdq.grad(u, t) - 0.0001 * u_xx + 5.0 * u ** 3 - 5.0 * u
    init = IC(D, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]])
    per = periodicBC(D, ["x"], [deriv_model])
    kw = {}
    if sa:
        g = torch.Generator().manual_seed(seed)
        kw = dict(Adaptive_type="self-adaptive", dict_adaptive={"residual": [True], "BCs": [True, False]},
                  init_weights={"residual": [torch.rand(n_f, 1, generator=g)],
                                "BCs": [100 * torch.rand(64, 1, generator=g), None]})
    return D, [init, per], f_model, kw


def compiled(backend, problem="burgers", **extra):
    if problem == "burgers":
        D, bcs, f = burgers()
        kw = {}
    else:
        D, bcs, f, kw = allen_cahn()
    torch.manual_seed(0)
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 12, 12, 1], f, D, bcs, backend=backend, device="cpu", **kw, **extra)
    return m


@pytest.mark.parametrize("problem", ["burgers", "ac"])
def test_jet_backend_equals_autograd(problem):
    a, b = compiled("jet", problem), compiled("autograd", problem)
    assert a.active_backend == "jet" and b.active_backend == "autograd"
    la, ga = a.grad()
    lb, gb = b.grad()
    assert torch.allclose(la, lb, rtol=1e-5)
    for x, y in zip(ga, gb):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-6)


def test_fit_reduces_loss_and_tracks_best():
    m = compiled("jet")
    l0 = m.update_loss().item()
    m.fit(tf_iter=60)
    hist = m.losses
    assert len(hist) == 60 and set(hist[0]) >= {"BC_0", "BC_1", "BC_2", "Residual_0", "Total Loss"}
    assert hist[-1]["Total Loss"] < l0
    best = min(h["Total Loss"] for h in hist)
    assert m.min_loss["adam"] == pytest.approx(best)
    assert hist[m.best_epoch["adam"]]["Total Loss"] == pytest.approx(best)
    # best snapshot really reproduces the best loss
    cur = m.u_model.flat.detach().clone()
    with torch.no_grad():
        m.u_model.flat.copy_(m._best_flat["adam"])
    assert m.update_loss().item() == pytest.approx(best, rel=1e-5)
    with torch.no_grad():
        m.u_model.flat.copy_(cur)


def test_fit_resumes():
    m = compiled("jet")
    m.fit(tf_iter=10)
    m.fit(tf_iter=5)
    assert len(m.losses) == 15 and m.tf_optimizer.iterations == 15


def test_sa_weights_ascend():
    m = compiled("jet", "ac")
    lam0 = [l.detach().clone() for l in m.lambdas]
    m.fit(tf_iter=5)
    # gradient ascent: weights of points with nonzero residual grow
    assert (m.lambdas[0] - lam0[0]).mean().item() > 0
    assert (m.lambdas[1] - lam0[1]).mean().item() > 0


def test_adaptive_type_aliases():
    for t in (1, "self-adaptive", "SA"):
        m = compiled("jet", "ac") if t == 1 else None
    from tensordiffeq_amd.models.collocation import parse_adaptive_type
    assert parse_adaptive_type("self-adaptive") == 1 and parse_adaptive_type(0) == 0
    assert parse_adaptive_type("loss-weights") == 2
    with pytest.raises(NotImplementedError):
        parse_adaptive_type("ntk")
    with pytest.raises(Exception):
        parse_adaptive_type("bogus")


def test_minibatch_and_lbfgs():
    m = compiled("jet")
    m.fit(tf_iter=3, batch_sz=100)
    assert len(m.losses) == 15
    l0 = m.update_loss().item()
    m.fit(newton_iter=20)
    assert m.min_loss["l-bfgs"] < l0
    m.fit(newton_iter=5, newton_eager=False)
    assert math.isfinite(m.min_loss["l-bfgs"])


def test_predict_and_best_model():
    m = compiled("jet")
    m.fit(tf_iter=5)
    X = np.random.rand(37, 2)
    u, f = m.predict(X)
    assert u.shape == (37, 1) and f.shape == (37, 1)
    ub, _ = m.predict(X, best_model=True)
    assert ub.shape == (37, 1)
    # residual from predict equals autograd evaluation
    ma = compiled("autograd")
    with torch.no_grad():
        ma.u_model.flat.copy_(m.u_model.flat)
    _, fa = ma.predict(X)
    np.testing.assert_allclose(f, fa, rtol=1e-4, atol=1e-5)
    # u is the jet's value stream: equal to the network evaluated in float64
    ws = [(k.detach().double(), b.detach().double()) for k, b in m.u_model.weights()]
    h = torch.as_tensor(X, dtype=torch.float64)
    for i, (k, b) in enumerate(ws):
        h = torch.addmm(b, h, k)
        h = torch.tanh(h) if i < len(ws) - 1 else h
    np.testing.assert_allclose(u, h.numpy(), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("fmt", ["npz", "pt", "dir"])
def test_save_load_roundtrip(tmp_path, fmt):
    m = compiled("jet", "ac")
    m.fit(tf_iter=4)
    path = str(tmp_path / ("ck." + fmt if fmt != "dir" else "ckdir"))
    m.save(path)
    m2 = compiled("jet", "ac")
    m2.load_model(path)
    assert torch.equal(m2.u_model.flat, m.u_model.flat)
    if fmt != "npz":
        m3 = compiled("jet", "ac")
        m3.resume(path)
        assert torch.equal(m3.lambdas[0], m.lambdas[0])
        m.fit(tf_iter=2)
        m3.fit(tf_iter=2)
        assert torch.allclose(m3.u_model.flat, m.u_model.flat, atol=1e-6)


def test_periodic_legacy_only_u():
    a = compiled("jet", "ac", periodic_legacy=True)
    b = compiled("jet", "ac")
    ta = a.program().evaluate(a.u_model.flat, a.lambdas)[1]["BC_1"]
    tb = b.program().evaluate(b.u_model.flat, b.lambdas)[1]["BC_1"]
    assert ta.item() < tb.item()


def test_neumann_functiondirichlet_and_assimilation():
    tdq.set_seed(0)
    D = DomainND(["x", "y"])
    D.add("x", [0.0, 1.0], 11)
    D.add("y", [0.0, 1.0], 11)
    D.generate_collocation_points(200)

    def dx(u_model, x, y):
        return tdq.grad(u_model(torch.cat([x, y], 1)), x)

    bcs = [dirichletBC(D, val=0.0, var="x", target="lower"),
           FunctionDirichletBC(D, fun=[lambda y: np.sin(math.pi * y)], var="x", target="upper",
                               func_inputs=["y"], n_values=8),
           FunctionNeumannBC(D, fun=[lambda y: 0 * y], var="y", target="upper", deriv_model=[dx],
                             func_inputs=["x"])]

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        return tdq.grad(tdq.grad(u, x), x) + tdq.grad(tdq.grad(u, y), y) + torch.sin(math.pi * x)

    losses = {}
    for be in ("jet", "autograd"):
        torch.manual_seed(0)
        m = tdq.CollocationSolverND(assimilate=True, verbose=False)
        m.compile([2, 8, 8, 1], f_model, D, bcs, backend=be, device="cpu")
        m.compile_data(np.array([0.5, 0.25]), np.array([0.5, 0.75]), np.array([0.1, -0.2]))
        losses[be] = m.update_loss().item()
        assert "Data" in m.loss_terms
    assert losses["jet"] == pytest.approx(losses["autograd"], rel=1e-5)


def test_custom_network_uses_autograd():
    D, bcs, f = burgers()
    m = tdq.CollocationSolverND(verbose=False)
    net = torch.nn.Sequential(torch.nn.Linear(2, 8), torch.nn.Tanh(), torch.nn.Linear(8, 1))
    m.compile([2, 8, 1], f, D, bcs, device="cpu", network=net)
    assert m.active_backend == "autograd"
    assert torch.isfinite(m.update_loss())


def test_discovery_model_learns_coefficients():
    tdq.set_seed(0)
    x = np.linspace(-1, 1, 41)
    t = np.linspace(0, 1, 11)
    X, T = np.meshgrid(x, t)
    xs, ts = X.reshape(-1, 1), T.reshape(-1, 1)
    u = np.sin(math.pi * xs) * np.exp(-0.5 * ts)  # u_t = c * u_xx with c = 0.5/pi^2

    def f_model(u_model, var, x, t):
        uu = u_model(torch.cat([x, t], 1))
        return tdq.grad(uu, t) - var[0] * tdq.grad(tdq.grad(uu, x), x)

    for be in ("jet", "autograd"):
        torch.manual_seed(0)
        params = [tdq.Variable(0.0)]
        m = tdq.DiscoveryModel(verbose=False)
        m.compile([2, 16, 16, 1], f_model, [xs, ts], u, params, backend=be, device="cpu")
        l0 = m.loss().item()
        m.fit(tf_iter=150)
        assert m.loss().item() < l0
        assert abs(float(params[0].detach())) > 0  # coefficient moved and was mirrored into the user tensor


def test_discovery_lbfgs_phase_recovers_coefficient():
    """fit(tf_iter, newton_iter): L-BFGS over network + coefficient after Adam - the coefficient of
    u_t = c u_xx (c = 0.5/pi^2 = 0.0507) is recovered to a few percent on a tiny CPU problem, where
    Adam alone (lr 5e-3 moves c by ~lr per step) stays further off."""
    tdq.set_seed(0)
    x = np.linspace(-1, 1, 41)
    t = np.linspace(0, 1, 11)
    X, T = np.meshgrid(x, t)
    xs, ts = X.reshape(-1, 1), T.reshape(-1, 1)
    u = np.sin(math.pi * xs) * np.exp(-0.5 * ts)

    def f_model(u_model, var, x, t):
        uu = u_model(torch.cat([x, t], 1))
        return tdq.grad(uu, t) - var[0] * tdq.grad(tdq.grad(uu, x), x)

    torch.manual_seed(0)
    params = [tdq.Variable(0.0)]
    m = tdq.DiscoveryModel(verbose=False)
    m.compile([2, 16, 16, 1], f_model, [xs, ts], u, params, backend="jet", device="cpu")
    m.fit(tf_iter=300, newton_iter=300)
    c = float(params[0].detach())
    assert m.fit_info["lbfgs"]["n_iter"] > 10
    assert abs(c - 0.5 / math.pi ** 2) / (0.5 / math.pi ** 2) < 0.05, c
    # var_history: (step, values) throughout - the L-BFGS entry at Adam steps + its iterations
    steps = [s for s, _ in m.var_history]
    assert all(isinstance(s, int) for s in steps) and steps == sorted(steps)
    assert steps[-1] == 300 + m.fit_info["lbfgs"]["n_iter"]


def test_tensordiffeq_alias():
    import tensordiffeq
    from tensordiffeq.models import CollocationSolverND
    from tensordiffeq.boundaries import DomainND as D2
    assert CollocationSolverND is tdq.CollocationSolverND and D2 is DomainND
    assert tensordiffeq.utils.MSE is tdq.MSE


def test_load_model_with_other_layer_sizes_resets_best_snapshot(tmp_path):
    """After fit, load a checkpoint of a LARGER network and fit again: the best-weights
    snapshot is rebuilt for the new parameter vector (the fused Adam copies the parameters into
    it - a stale smaller snapshot would be an out-of-bounds write on a GPU)."""
    big = tdq.CollocationSolverND(verbose=False)
    D, bcs, f = burgers()
    torch.manual_seed(1)
    big.compile([2, 16, 16, 16, 1], f, D, bcs, backend="jet", device="cpu")
    path = str(tmp_path / "big.npz")
    big.save(path)
    m = compiled("jet")
    m.fit(tf_iter=3)
    m.load_model(path)
    assert m.u_model.flat.numel() == big.u_model.flat.numel()
    m.fit(tf_iter=3)
    st = m._state
    assert st["best_flat"].numel() == m.u_model.flat.numel()
    assert len(m.losses) == 6 and math.isfinite(m.min_loss["adam"])
    assert 3 <= m.best_epoch["adam"] < 6   # best tracking restarted with the new network
