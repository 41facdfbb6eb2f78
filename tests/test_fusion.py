"""Loss fusion: tracing user callables into bytecode reproduces the autograd-composed loss
(CPU, torch reference executor) and the HIP kernel reproduces losses AND gradients (GPU)."""
import math

import numpy as np
import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd import fusion
from tests.test_solver import allen_cahn, burgers, compiled


def _check_reference(m):
    prog = m.program()
    fl = fusion.build(prog, m.lambdas)
    assert fl is not None
    J = prog.jet(m.u_model.flat)
    _, ref = prog.evaluate(m.u_model.flat, m.lambdas)
    got = fusion.run_reference(fl, prog, J, m.lambdas, fusion.scalar_values(fl, m.lambdas, None))
    for name, l in zip(fl.term_names, got):
        assert l.item() == pytest.approx(ref[name].item(), rel=1e-5, abs=1e-7), name
    return fl


@pytest.mark.parametrize("problem", ["burgers", "ac"])
def test_fusion_reference_matches_loss_program(problem):
    fl = _check_reference(compiled("jet", problem))
    assert all(g.program.n_regs <= fusion.MAX_REGS for g in fl.groups)


def test_fusion_g_function_and_constants():
    D, bcs, f, kw = allen_cahn()
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 8, 8, 1], f, D, bcs, backend="jet", device="cpu", g=lambda lam: lam ** 2 + 0.5 * torch.exp(-lam),
              **kw)
    _check_reference(m)


def test_fusion_neumann_sin_forcing():
    tdq.set_seed(0)
    from tensordiffeq_amd.boundaries import DomainND, FunctionNeumannBC, dirichletBC
    D = DomainND(["x", "y"])
    D.add("x", [0.0, 1.0], 11)
    D.add("y", [0.0, 1.0], 11)
    D.generate_collocation_points(100)

    def dx(u_model, x, y):
        return tdq.grad(u_model(torch.cat([x, y], 1)), x)

    bcs = [dirichletBC(D, val=0.0, var="x", target="lower"),
           FunctionNeumannBC(D, fun=[lambda y: np.cos(y)], var="y", target="upper", deriv_model=[dx],
                             func_inputs=["x"])]

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        return tdq.grad(tdq.grad(u, x), x) + tdq.grad(tdq.grad(u, y), y) - torch.sin(math.pi * x) * torch.sin(
            tdq.constant(2.0) * y) / (1.0 + u ** 2)

    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 8, 8, 1], f_model, D, bcs, backend="jet", device="cpu")
    _check_reference(m)


def test_fusion_rejects_untraceable():
    D, bcs, _ = burgers()

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return tdq.grad(u, x) * u.mean()  # non-elementwise

    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 8, 1], f_model, D, bcs, backend="jet", device="cpu")
    assert fusion.build(m.program(), m.lambdas) is None


@pytest.mark.gpu
@pytest.mark.parametrize("problem", ["burgers", "ac"])
def test_fused_kernel_matches_autograd_gpu(problem):
    if problem == "burgers":
        D, bcs, f = burgers(n_f=3000)
        kw = {}
    else:
        D, bcs, f, kw = allen_cahn(n_f=3000)
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 128, 128, 128, 1], f, D, bcs, backend="hip", device="cuda", **kw)
    prog = m.program()
    assert prog.fused_op is not None
    eng = m._get_engine(None, 4)
    loss_f, grads_f, terms_f = eng._phase_a()
    loss_f, grads_f, terms_f = float(loss_f), [g.clone() for g in grads_f], [float(t) for t in terms_f]
    fop = prog.fused_op
    prog.fused_op = None
    try:
        loss_r, grads_r, terms_r = eng._phase_a()
    finally:
        prog.fused_op = fop
    assert loss_f == pytest.approx(float(loss_r), rel=1e-5)
    assert terms_f == pytest.approx([float(t) for t in terms_r], rel=1e-5)
    for a, b in zip(grads_f, grads_r):
        assert ((a - b).norm() / b.norm().clamp_min(1e-20)).item() < 1e-4
