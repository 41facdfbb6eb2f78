"""High-order (order 3 / 4) jet kernels of small point sets (csrc/jet_hi.hip, ops/jet_hi.py).

The reference's AC-baseline / AC-dist-new periodic BCs enforce u_xxx and u_xxxx (examples/
AC-baseline.py:23-29); those 2 x 201 points keep the fused step (fused loss, fused tail, K-step
graphs) with their extra streams from these kernels.  Oracles: the fp64 torch Taylor-jet engine
(jet.py, itself checked against nested autograd in test_sampling_jet.py) and nested autograd.
"""
import math

import numpy as np
import pytest
import torch

from tensordiffeq_amd.jet import JetPlan, jet_forward
from tensordiffeq_amd.models.networks import TanhMLP
from tensordiffeq_amd.ops import jet_hi


def test_build_spec_ac_baseline_plan():
    """u, u_x, u_xx, u_xxx, u_xxxx: Faa di Bruno term counts 1 + 2 + 3 + 5; only the requested rows out."""
    plan = JetPlan([(0, 0, 0, 0)], 2)
    si, sc = jet_hi.build_spec(plan, {(0, 0, 0): 4, (0, 0, 0, 0): 5})
    S = si[0]
    assert S == 5 and si[1:1 + S] == [0, 1, 2, 3, 4]
    assert si[1 + 2 * S:1 + 3 * S] == [-1, -1, -1, 4, 5]
    nt = si[1 + 3 * S]
    assert nt == 11 and len(sc) == 11
    terms = [si[2 + 3 * S + 7 * k:2 + 3 * S + 7 * k + 7] for k in range(nt)]
    # u_xxxx: k=1 (z4); k=2: 4 z1 z3, 3 z2^2; k=3: 6 z1^2 z2; k=4: z1^4
    last = {(t[1], tuple(sorted(t[3:3 + t[2]]))): c for t, c in zip(terms, sc) if t[0] == 4}
    assert last == {(1, (4,)): 1.0, (2, (1, 3)): 4.0, (2, (2, 2)): 3.0, (3, (1, 1, 2)): 6.0, (4, (1, 1, 1, 1)): 1.0}


def test_eligibility_limits():
    net = TanhMLP([2, 128, 128, 1], device="cpu")
    assert jet_hi.eligible(net, JetPlan([(0, 0, 0, 0)], 2))[0]
    assert not jet_hi.eligible(TanhMLP([2, 256, 1], device="cpu"), JetPlan([(0, 0, 0)], 2))[0]
    # a 3-variable order-4 closure has more than 8 streams
    assert not jet_hi.eligible(net, JetPlan([(0, 0, 1, 1), (0, 1, 1, 1), (0, 0, 0, 1)], 2))[0]


def _ref_fp64(net, X, plan, dJ):
    p = net.flat.detach().double().clone().requires_grad_(True)
    J = jet_forward(X.double(), net.weights(p), plan)
    g = torch.autograd.grad((J * dJ.double()).sum(), p)[0]
    return J.detach(), g


@pytest.mark.gpu
@pytest.mark.parametrize("sizes,reqs,n", [
    ([2, 128, 128, 128, 128, 1], [(0, 0, 0, 0)], 402),
    ([2, 64, 128, 32, 1], [(0, 0, 0), (0, 1, 1)], 37),
    ([3, 20, 20, 20, 2], [(0, 0, 0, 0), (1, 2)], 9),
])
def test_hi_kernels_match_fp64_jet(sizes, reqs, n):
    """Every stream row of the forward and the parameter gradient of <dJ, J> vs the fp64 torch jet
    (relative error per stream < 1e-4 forward and gradient: the layer GEMMs are split-bf16 (bf16x3)
    MFMA, the precision of the main kernels this path runs beside; ~1e-5 typical, mixed-variable
    streams with cancellation up to ~5e-5)."""
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    net = TanhMLP(sizes, device=dev)
    with torch.no_grad():
        net.flat.add_(0.05 * torch.randn_like(net.flat))
    plan = JetPlan(reqs, sizes[0])
    X = (2 * torch.rand(n, sizes[0], device=dev) - 1).contiguous()
    rows = {m: i for i, m in enumerate(plan.streams)}
    op = jet_hi.HiJetOp(net, plan, rows, X, n, dev)
    J = torch.full((plan.S, n, sizes[-1]), float("nan"), device=dev)
    op.forward(J, net.flat)
    dJ = torch.randn(plan.S, n, sizes[-1], device=dev)
    g = op.backward(dJ, net.flat).clone()
    torch.cuda.synchronize()
    Jr, gr = _ref_fp64(net, X, plan, dJ)
    for s, mi in enumerate(plan.streams):
        err = ((J[s].double() - Jr[s]).norm() / Jr[s].norm().clamp_min(1e-30)).item()
        print(f"HI fwd {sizes} stream {mi}: {err:.2e}")
        assert err < 1e-4, (mi, err)
    gerr = ((g.double() - gr).norm() / gr.norm()).item()
    print(f"HI grad {sizes}: {gerr:.2e}")
    assert gerr < 1e-4
    # deterministic: a second backward gives the same bits
    g2 = op.backward(dJ, net.flat)
    assert torch.equal(g, g2)
    # isolated kernel time (the AC-baseline periodic-BC set: 402 points, order 4)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    for _ in range(5):
        op.forward(J, net.flat)
        op.backward(dJ, net.flat)
    ev[0].record()
    for _ in range(50):
        op.forward(J, net.flat)
    ev[1].record()
    for _ in range(50):
        op.backward(dJ, net.flat)
    ev[2].record()
    torch.cuda.synchronize()
    print(f"HI time {sizes} n={n}: fwd {ev[0].elapsed_time(ev[1]) * 20:.1f} us, "
          f"bwd {ev[1].elapsed_time(ev[2]) * 20:.1f} us")


@pytest.mark.gpu
def test_hi_kernels_seed_only_their_rows():
    """Rows not owned by the kernel (out = -1: the fused kernels' streams) are neither written by the
    forward nor seeded in the backward."""
    torch.manual_seed(1)
    dev = torch.device("cuda", 0)
    net = TanhMLP([2, 32, 32, 1], device=dev)
    plan = JetPlan([(0, 0, 0, 0)], 2)
    X = torch.rand(50, 2, device=dev)
    rows = {(0, 0, 0): 0, (0, 0, 0, 0): 1}
    op = jet_hi.HiJetOp(net, plan, rows, X, 50, dev)
    J = torch.full((2, 50, 1), float("nan"), device=dev)
    op.forward(J, net.flat)
    assert torch.isfinite(J).all()
    dJ = torch.randn(2, 50, 1, device=dev)
    g = op.backward(dJ, net.flat)
    full = torch.zeros(plan.S, 50, 1, device=dev)
    full[3], full[4] = dJ[0], dJ[1]
    _, gr = _ref_fp64(net, X, plan, full)
    assert ((g.double() - gr).norm() / gr.norm()).item() < 1e-4


def _ac_baseline(n_f, backend, precision, seed=0):
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, IC, periodicBC
    tdq.set_seed(seed)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 512)
    D.add("t", [0.0, 1.0], 201)
    D.generate_collocation_points(n_f)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_xxx = tdq.grad(u_xx, x)
        return u, u_x, u_xxx, tdq.grad(u_xxx, x)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_xx = tdq.grad(tdq.grad(u, x), x)
        return tdq.grad(u, t) - 0.0001 * u_xx + 5.0 * u ** 3 - 5.0 * u

    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 128, 128, 128, 128, 1], f_model, D,
              [IC(D, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]]), periodicBC(D, ["x"], [deriv_model])],
              backend=backend, device="cuda", precision=precision)
    return m


@pytest.mark.gpu
@pytest.mark.timeout(300)
def test_ac_baseline_fused_high_order_path():
    """AC-baseline program in bf16x3: the high-order points run through the fused step (hi_op on,
    fused loss, fused tail, K-step graphs), and loss / gradient match the all-torch jet program."""
    a = _ac_baseline(6000, "auto", "bf16x3")
    b = _ac_baseline(6000, "jet", None)
    pa = a.program()
    assert a.active_backend == "hip" and pa.mixed and pa.hi_op is not None and pa.fused_op is not None
    assert pa.X_all.shape[0] == 6000 + 512 + 2 * 201 and pa.n_hi == 2 * 201
    la, ga = a.grad()
    lb, gb = b.grad()
    print(f"HI ac-baseline loss {la.item():.6e} vs {lb.item():.6e}")
    assert abs(la.item() - lb.item()) / abs(lb.item()) < 1e-4
    gerr = ((ga[0] - gb[0]).norm() / gb[0].norm()).item()
    print(f"HI ac-baseline grad rel err {gerr:.2e}")
    assert gerr < 1e-3
    a.fit(tf_iter=24)
    b.fit(tf_iter=24)
    eng = a._get_engine(None, 1)
    assert eng._tail_eligible() and getattr(eng, "graph_k", None) is not None
    ha, hb = [h["Total Loss"] for h in a.losses], [h["Total Loss"] for h in b.losses]
    print("HI fit", ha[-1], hb[-1])
    assert abs(ha[-1] - hb[-1]) / hb[-1] < 2e-2
    a.fit(newton_iter=20)
    assert np.isfinite(a.min_loss["l-bfgs"]) and a.min_loss["l-bfgs"] <= ha[-1] * 1.01
