"""Run-time specialized fused-loss kernels (ops/loss_jit.py, csrc/loss_jit.hip).

CPU: the generated HIP C++ of several traced programs (SA weights, periodic pairs, Dirichlet/IC,
g(lambda) with exp, sin forcing with division and powers, scalar coefficients) compiles with
hipRTC for gfx950.  GPU: the specialized kernel reproduces the interpreter BIT FOR BIT (dJ,
SA-weight gradients, block partials, whole-range and range launches, a training trajectory).
"""
import ctypes
import math

import numpy as np
import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd import fusion
from tests.test_solver import allen_cahn, burgers


def _neumann_sin(device, backend, width=8):
    tdq.set_seed(0)
    from tensordiffeq_amd.boundaries import DomainND, FunctionNeumannBC, dirichletBC
    D = DomainND(["x", "y"])
    D.add("x", [0.0, 1.0], 11)
    D.add("y", [0.0, 1.0], 11)
    D.generate_collocation_points(300)

    def dx(u_model, x, y):
        return tdq.grad(u_model(torch.cat([x, y], 1)), x)

    bcs = [dirichletBC(D, val=0.0, var="x", target="lower"),
           FunctionNeumannBC(D, fun=[lambda y: np.cos(y)], var="y", target="upper", deriv_model=[dx],
                             func_inputs=["x"])]

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        return tdq.grad(tdq.grad(u, x), x) + tdq.grad(tdq.grad(u, y), y) - torch.sin(math.pi * x) * torch.sin(
            tdq.constant(2.0) * y) / (1.0 + u ** 2) + 0.1 * torch.sqrt(1.0 + u * u) ** 1.5

    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, width, width, 1], f_model, D, bcs, backend=backend, device=device)
    return m


def _model(problem, device, backend, width=8, n_f=400):
    if problem == "neumann":
        return _neumann_sin(device, backend, width)
    torch.manual_seed(0)
    m = tdq.CollocationSolverND(verbose=False)
    if problem == "burgers":
        D, bcs, f = burgers(n_f=n_f)
        m.compile([2, width, width, 1], f, D, bcs, backend=backend, device=device)
    elif problem == "ac_g":
        D, bcs, f, kw = allen_cahn(n_f=n_f)
        m.compile([2, width, width, 1], f, D, bcs, backend=backend, device=device,
                  g=lambda lam: lam ** 2 + 0.5 * torch.exp(-lam), **kw)
    else:
        D, bcs, f, kw = allen_cahn(n_f=n_f)
        m.compile([2, width, width, 1], f, D, bcs, backend=backend, device=device, **kw)
    return m


PROBLEMS = ["ac", "burgers", "ac_g", "neumann"]


@pytest.mark.parametrize("problem", PROBLEMS)
def test_generated_kernel_compiles(problem):
    from tensordiffeq_amd.ops import _lib, loss_jit
    from tensordiffeq_amd.ops.loss_fused import FusedLossOp
    if not _lib.available():
        pytest.skip("native library not built")
    m = _model(problem, "cpu", "jet")
    prog = m.program()
    fl = fusion.build(prog, m.lambdas)
    assert fl is not None
    op = FusedLossOp(fl, prog, m.lambdas, fusion.scalar_values(fl, m.lambdas, None), fl.lam_offsets)
    assert op.jit is None                      # CPU programs keep the interpreter / torch path
    src = loss_jit.generate(op)
    assert "tdq_loss_jit" in src and "switch" not in src
    lib = _lib.load()
    code, size = ctypes.c_void_p(0), ctypes.c_longlong(0)
    log = ctypes.create_string_buffer(8192)
    rc = lib.tdq_rtc_compile(src.encode(), b"t.hip", b"gfx950", ctypes.byref(code), ctypes.byref(size), log, 8192)
    assert rc == 0, log.value.decode()
    assert size.value > 0
    lib.tdq_rtc_free(code)


def _run(op, J, ranges=None):
    if ranges is None:
        op(J, with_total=True, reduce=True)
    else:
        for b0, nb in ranges:
            op.run_range(J, b0, nb)
    torch.cuda.synchronize()
    return [op.dJ.clone(), op.partials.clone()] + [d.clone() for d in op.dlam] + [op.losses.clone()]


@pytest.mark.gpu
@pytest.mark.parametrize("problem", PROBLEMS)
def test_jit_matches_interpreter_bitwise(problem):
    m = _model(problem, "cuda", "hip", width=32, n_f=3000)
    prog = m.program()
    op = prog.fused_op
    assert op is not None and op.engine == "jit"
    torch.manual_seed(1)
    J = prog.jet(m.u_model.flat).detach().contiguous()
    J = J + 0.01 * torch.randn_like(J)
    jit = op.jit
    a = _run(op, J)
    nb = op.n_blocks
    ar = _run(op, J, [(0, nb // 3), (nb // 3, nb - nb // 3)])
    op.jit = None
    try:
        b = _run(op, J)
    finally:
        op.jit = jit
    for x, y in zip(a, b):
        assert torch.equal(x, y), (x - y).abs().max().item()
    for x, y in zip(ar[:-1], b[:-1]):
        assert torch.equal(x, y)


@pytest.mark.gpu
def test_jit_training_trajectory_matches_interpreter(monkeypatch):
    """The AC-SA solver (fused tail, point ranges, graphs) with the specialized loss kernel follows
    the interpreter's trajectory bit for bit."""
    import bench
    hist = {}
    for flag in ("1", "0"):
        monkeypatch.setenv("TDQ_LOSS_JIT", flag)
        m = bench.build_problem(20000, 1, "hip", torch.device("cuda", 0), False, "bf16")
        assert m.program().fused_op.engine == ("jit" if flag == "1" else "interpreter")
        m.fit(tf_iter=12)
        m.fit(newton_iter=4)
        hist[flag] = ([h["Total Loss"] for h in m.losses], m.u_model.flat.detach().cpu().clone())
    assert hist["1"][0] == hist["0"][0]
    assert torch.equal(hist["1"][1], hist["0"][1])
