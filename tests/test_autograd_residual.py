"""Residuals written with plain ``torch.autograd.grad`` (the PyTorch spelling of the reference's
``tf.gradients``, reference examples/burgers-new.py:26-32) run on the jet path under
``backend="auto"`` and match the nested-autograd backend; callables the jet cannot serve fall back
to autograd instead of crashing."""
import math

import numpy as np
import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import DomainND, IC, dirichletBC


def _domain(n_f=400, seed=0):
    tdq.set_seed(seed)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 64)
    D.add("t", [0.0, 1.0], 20)
    D.generate_collocation_points(n_f)
    bcs = [IC(D, [lambda x: -np.sin(x * math.pi)], var=[["x"]]),
           dirichletBC(D, val=0.0, var="x", target="upper"), dirichletBC(D, val=0.0, var="x", target="lower")]
    return D, bcs


def f_autograd(u_model, x, t):
    u = u_model(torch.cat([x, t], 1))
    u_x = torch.autograd.grad(u, x, grad_outputs=torch.ones_like(u), create_graph=True)[0]
    u_xx = torch.autograd.grad(u_x, x, torch.ones_like(u_x), create_graph=True)[0]
    u_t = torch.autograd.grad(u, t, torch.ones_like(u), create_graph=True)[0]
    return u_t + u * u_x - (0.01 / math.pi) * u_xx


def f_mixed(u_model, x, t):
    u = u_model(torch.cat([x, t], 1))
    u_x, u_t = torch.autograd.grad(u, [x, t], torch.ones_like(u), create_graph=True)
    u_xx = tdq.grad(u_x, x)
    return u_t + u * u_x - (0.01 / math.pi) * u_xx


def f_foreign(u_model, x, t):
    # derivative of a non-stream tensor (u^2): not servable from a jet -> autograd backend
    u = u_model(torch.cat([x, t], 1))
    q = u * u
    q_x = torch.autograd.grad(q, x, torch.ones_like(q), create_graph=True)[0]
    u_t = torch.autograd.grad(u, t, torch.ones_like(u), create_graph=True)[0]
    return u_t + 0.5 * q_x


def f_scaled_cotangent(u_model, x, t):
    u = u_model(torch.cat([x, t], 1))
    u_t = torch.autograd.grad(u, t, 2.0 * torch.ones_like(u), create_graph=True)[0]
    return u_t


def _solver(f, backend, n_f=400):
    D, bcs = _domain(n_f)
    torch.manual_seed(0)
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 12, 12, 1], f, D, bcs, backend=backend, device="cpu")
    return m


@pytest.mark.parametrize("f", [f_autograd, f_mixed])
def test_autograd_residual_runs_on_jet_and_matches(f):
    a, b = _solver(f, "auto"), _solver(f, "autograd")
    assert a.active_backend == "jet", a.program().reasons
    la, ga = a.grad()
    lb, gb = b.grad()
    assert torch.allclose(la, lb, rtol=1e-5)
    for x, y in zip(ga, gb):
        assert torch.allclose(x, y, rtol=1e-4, atol=1e-6)
    a.fit(tf_iter=15)
    b.fit(tf_iter=15)
    ha = [r["Total Loss"] for r in a.losses]
    hb = [r["Total Loss"] for r in b.losses]
    assert np.allclose(ha, hb, rtol=1e-3), (ha, hb)


@pytest.mark.parametrize("f", [f_foreign, f_scaled_cotangent])
def test_unservable_autograd_residual_falls_back(f):
    a = _solver(f, "auto")
    assert a.active_backend == "autograd"
    assert a.program().reasons
    a.fit(tf_iter=3)
    assert all(math.isfinite(r["Total Loss"]) for r in a.losses)


def test_torch_autograd_grad_restored_outside_contexts():
    from tensordiffeq_amd import autodiff
    _solver(f_autograd, "auto").grad()
    assert torch.autograd.grad is autodiff._ORIG_AUTOGRAD_GRAD


@pytest.mark.parametrize("f", [f_autograd, f_mixed])
def test_autograd_residual_traces_into_fused_loss(f):
    """The fused-loss tracer (symbolic tensors) resolves torch.autograd.grad like tdq.grad."""
    from tensordiffeq_amd import fusion
    m = _solver(f, "jet")
    prog = m.program()
    fl = fusion.build(prog, m.lambdas)
    assert fl is not None
    J = prog.jet(m.u_model.flat)
    _, ref = prog.evaluate(m.u_model.flat, m.lambdas)
    got = fusion.run_reference(fl, prog, J, m.lambdas, fusion.scalar_values(fl, m.lambdas, None))
    for name, l in zip(fl.term_names, got):
        assert l.item() == pytest.approx(ref[name].item(), rel=1e-5, abs=1e-7), name


@pytest.mark.gpu
def test_autograd_residual_on_hip_matches_autograd_backend():
    """MI355X: the torch.autograd.grad residual plans onto the HIP jet kernels (bf16x3, fused
    loss) and its loss / gradient match the nested-autograd backend."""
    D, bcs = _domain(2000)

    def make(backend):
        torch.manual_seed(0)
        m = tdq.CollocationSolverND(verbose=False)
        m.compile([2, 20, 20, 20, 1], f_autograd, D, bcs, backend=backend, device="cuda", precision="bf16x3")
        return m
    a, b = make("auto"), make("autograd")
    assert a.active_backend == "hip", a.program().reasons
    assert a.program().fused_op is not None
    la, ga = a.grad()
    lb, gb = b.grad()
    assert torch.allclose(la, lb, rtol=1e-4)
    assert torch.allclose(ga[0], gb[0], rtol=1e-3, atol=1e-5 * float(gb[0].abs().max()))
    a.fit(tf_iter=20)
    b.fit(tf_iter=20)
    ha = np.array([r["Total Loss"] for r in a.losses])
    hb = np.array([r["Total Loss"] for r in b.losses])
    assert np.allclose(ha, hb, rtol=2e-3), (ha, hb)
