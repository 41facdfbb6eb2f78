"""HIP kernel numerics vs plain PyTorch fp32 references (run on MI355X: ``pytest -m gpu``).

Jet forward: every derivative stream against the torch jet engine (itself checked against nested
autograd in test_jet.py) AND directly against nested ``torch.autograd.grad``.
Jet backward: the flat parameter gradient of a random linear functional of J against autograd
through the torch jet.  Shapes cover non-multiple-of-64 point counts, every width-tile class
(WT = 1, 2, 4, 8 incl. padded widths; WT = 16 in bf16), 1-8 streams, d_in 1-3, d_out 1-2, 1-4 hidden layers.
"""
import pytest
import torch

from tensordiffeq_amd.jet import JetPlan, jet_forward
from tensordiffeq_amd.models.networks import TanhMLP

pytestmark = pytest.mark.gpu

# max error relative to each stream's scale (forward) / relative gradient norm (backward).
# bf16x3: every GEMM product carries ~2^-16 relative error (split-bf16 MFMA, csrc/jet_bf3.hip);
# bf16: weights and activations rounded to bf16 (2^-9 relative), fp32 accumulation.
# Bounds are ~2-3x the largest error measured over CASES on MI355X (profiles/r3_kernel_errors.txt:
# fwd fp32 3.1e-6, bf16x3 1.0e-4, bf16 3.3e-2 (4.7e-2 for the 8-hidden-layer Burgers net);
# bwd fp32 4.7e-7, bf16x3 8.3e-6, bf16 5.5e-3).
TOL_FWD = {"fp32": 8e-6, "bf16x3": 2.5e-4, "bf16": 8e-2}
TOL_BWD = {"fp32": 1.5e-6, "bf16x3": 2.5e-5, "bf16": 1.4e-2}
TOL_FWD_BF16_SHALLOW = 5e-2   # bf16 forward bound for nets with <= 4 hidden layers (measured <= 3.3e-2)
PRECS = ["fp32", "bf16x3", "bf16"]

CASES = [
    # layer_sizes, requests, N
    ([2, 128, 128, 128, 128, 1], [(0,), (1,), (0, 0)], 1000),      # Allen-Cahn / Burgers plan
    ([2, 20, 20, 20, 20, 20, 20, 20, 20, 1], [(0,), (1,), (0, 0)], 777),  # Burgers net (WT=2)
    ([2, 50, 50, 50, 50, 1], [(0, 0), (1, 1)], 333),               # Helmholtz plan, S=5 (WT=4)
    ([3, 64, 64, 1], [(0, 0), (1, 1), (2,)], 130),                 # 3-D heat, S=6
    ([2, 16, 16, 1], [(0, 0), (0, 1), (1, 1)], 65),                # mixed derivative, S=6 (WT=1)
    ([1, 32, 2], [(0,), (0, 0)], 100),                             # 1-D, 2 outputs
    ([2, 128, 1], [], 70),                                          # value only, 1 hidden layer
    ([2, 128, 128, 128, 1], [(0,), (1,)], 64),                     # first order only
    ([3, 40, 40, 40, 1], [(0, 0), (1, 1), (2, 2), (0, 1)], 257),    # S=8, WT=4... (S*WT=32)
    # "wide" plans (S * WT > 32): one wave per SIMD; bf16x3 stages fragments in global scratch
    ([2, 128, 128, 128, 128, 1], [(0, 0), (1, 1)], 1000),          # 2-D Laplacian at width 128, S=5
    ([3, 128, 128, 128, 128, 1], [(0,), (1,), (2,), (0, 0), (1, 1), (0, 1)], 777),  # testing.py, S=7
    ([3, 96, 96, 96, 1], [(0, 0), (1, 1), (2, 2), (0, 1)], 300),   # S=8, padded WT=8
    ([2, 128, 128, 1], [(0, 0), (1, 1), (0, 1)], 200),             # S=6, 2 hidden layers
    ([4, 128, 128, 128, 1], [(0,), (1,), (2,), (3,)], 150),         # S=5, first order only
    # unequal hidden widths (the reference's neural_net takes any layer list): padded to the widest
    ([2, 64, 128, 32, 1], [(0,), (1,), (0, 0)], 500),              # AC plan, W = 128
    ([3, 50, 20, 80, 40, 2], [(0,), (1, 1), (2,)], 301),           # padded widths, d_out = 2
    ([2, 128, 96, 1], [(0, 0), (1, 1)], 200),                      # wide plan (S=5), 2 hidden layers
]


def _setup(sizes, reqs, N, seed=0):
    torch.manual_seed(seed)
    net = TanhMLP(sizes, device="cuda")
    with torch.no_grad():
        net.flat.add_(0.05 * torch.randn_like(net.flat))  # non-zero biases
    X = (torch.rand(N, sizes[0], device="cuda") * 2 - 1).contiguous()
    plan = JetPlan(reqs, sizes[0])
    return net, X, plan


def _fused_precision(jet_mlp, net, plan, prec):
    cfg = jet_mlp.hip_config(net, plan, prec)
    if cfg.get("engine") == "layered":   # e.g. fp32 wide plans: tests/test_layered_jet.py covers these
        pytest.skip(f"outside the fused kernels' envelope ({cfg['why']})")
    return cfg["precision"]


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("sizes,reqs,N", CASES)
def test_jet_forward_matches_torch(sizes, reqs, N, prec):
    from tensordiffeq_amd.ops import jet_hip, jet_mlp
    net, X, plan = _setup(sizes, reqs, N)
    prec = _fused_precision(jet_mlp, net, plan, prec)   # e.g. fp32 + unequal widths -> bf16x3
    with torch.no_grad():
        J = jet_hip.JetMLPFunction.apply(X, net.flat, net, plan, prec)
        Jref = jet_forward(X.double(), [(k.double(), b.double()) for k, b in net.weights()], plan)
    assert J.shape == Jref.shape
    scale = Jref.abs().amax(dim=(1, 2), keepdim=True).clamp_min(1e-3)
    err = ((J.double() - Jref).abs() / scale).max().item()
    print(f"KERNEL_ERR fwd {prec} {sizes} S={plan.S} {err:.3e}")
    tol = TOL_FWD_BF16_SHALLOW if (prec == "bf16" and len(sizes) <= 6) else TOL_FWD[prec]
    assert err < tol, err


@pytest.mark.parametrize("prec", PRECS)
def test_jet_forward_matches_autograd(prec):
    from tensordiffeq_amd.ops import jet_hip
    net, X, plan = _setup([2, 128, 128, 128, 128, 1], [(0,), (1,), (0, 0)], 300)
    with torch.no_grad():
        J = jet_hip.JetMLPFunction.apply(X, net.flat, net, plan, prec)
    cols = [X[:, j:j + 1].double().clone().requires_grad_(True) for j in range(2)]
    ws = [(k.double(), b.double()) for k, b in net.weights()]
    h = torch.cat(cols, 1)
    for i, (k, b) in enumerate(ws):
        h = torch.addmm(b, h, k)
        if i < len(ws) - 1:
            h = torch.tanh(h)
    u = h
    ux = torch.autograd.grad(u.sum(), cols[0], create_graph=True)[0]
    ut = torch.autograd.grad(u.sum(), cols[1], create_graph=True)[0]
    uxx = torch.autograd.grad(ux.sum(), cols[0])[0]
    for i, ref in enumerate([u, ux, ut, uxx]):
        err = (J[i].double() - ref.detach()).abs().max().item() / ref.abs().max().item()
        assert err < TOL_FWD[prec], (i, err)


@pytest.mark.parametrize("prec", PRECS)
@pytest.mark.parametrize("sizes,reqs,N", CASES)
def test_jet_backward_matches_autograd(sizes, reqs, N, prec):
    from tensordiffeq_amd.ops import jet_hip, jet_mlp
    net, X, plan = _setup(sizes, reqs, N, seed=1)
    prec = _fused_precision(jet_mlp, net, plan, prec)
    G = torch.randn(plan.S, N, sizes[-1], device="cuda", dtype=torch.float64)
    p = net.flat.detach().clone().requires_grad_(True)
    J = jet_hip.JetMLPFunction.apply(X, p, net, plan, prec)
    (J.double() * G).sum().backward()
    g_hip = p.grad.double()
    p64 = net.flat.detach().double().clone().requires_grad_(True)
    Jr = jet_forward(X.double(), net.weights(p64), plan)
    (Jr * G).sum().backward()
    g_ref = p64.grad
    rel = ((g_hip - g_ref).norm() / g_ref.norm()).item()
    print(f"KERNEL_ERR bwd {prec} {sizes} S={plan.S} {rel:.3e}")
    assert rel < TOL_BWD[prec], rel
    # every parameter block (per-layer kernels and biases) individually, not just the norm
    off = 0
    for k, b in net.weights(p64.detach()):
        for blk in (k, b):
            n = blk.numel()
            a, r = g_hip[off:off + n], g_ref[off:off + n]
            assert ((a - r).norm() / r.norm().clamp_min(1e-30)).item() < 20 * TOL_BWD[prec], (off, n)
            off += n


# hidden widths 129..256: the split-bf16 kernels at WT = 16, bf16 only, S <= 4 (csrc/jet_bf3_w16.hip)
WIDE256_CASES = [
    ([2, 256, 256, 256, 256, 1], [(0,), (1,), (0, 0)], 1000),      # AC plan at width 256, S = 4
    ([2, 200, 256, 1], [(0,), (0, 0)], 333),                         # unequal / padded widths, S = 3
    ([3, 160, 160, 2], [(0,), (1,)], 130),                           # padded, d_out = 2
    ([2, 256, 1], [(0,)], 70),                                       # one hidden layer, S = 2
    ([2, 256, 256, 1], [], 65),                                      # value only
]


@pytest.mark.parametrize("sizes,reqs,N", WIDE256_CASES)
def test_wide256_bf16_kernels_match_fp64(sizes, reqs, N):
    """Forward streams and the parameter gradient of the width-256 fused kernels vs the fp64 torch
    jet, at the bf16 bounds of the width-128 kernels."""
    from tensordiffeq_amd.ops import jet_hip, jet_mlp
    net, X, plan = _setup(sizes, reqs, N, seed=2)
    cfg = jet_mlp.hip_config(net, plan, "bf16")
    assert cfg.get("engine") != "layered" and cfg["WT"] == 16 and cfg["precision"] == "bf16"
    G = torch.randn(plan.S, N, sizes[-1], device="cuda", dtype=torch.float64)
    p = net.flat.detach().clone().requires_grad_(True)
    J = jet_hip.JetMLPFunction.apply(X, p, net, plan, "bf16")
    (J.double() * G).sum().backward()
    p64 = net.flat.detach().double().clone().requires_grad_(True)
    Jr = jet_forward(X.double(), net.weights(p64), plan)
    (Jr * G).sum().backward()
    scale = Jr.detach().abs().amax(dim=(1, 2), keepdim=True).clamp_min(1e-3)
    ferr = ((J.detach().double() - Jr.detach()).abs() / scale).max().item()
    g_hip, g_ref = p.grad.double(), p64.grad
    gerr = ((g_hip - g_ref).norm() / g_ref.norm()).item()
    print(f"KERNEL_ERR w256 bf16 {sizes} S={plan.S} fwd {ferr:.3e} bwd {gerr:.3e}")
    assert ferr < TOL_FWD_BF16_SHALLOW, ferr
    assert gerr < TOL_BWD["bf16"], gerr
    off = 0
    for k, b in net.weights(p64.detach()):
        for blk in (k, b):
            n = blk.numel()
            a, r = g_hip[off:off + n], g_ref[off:off + n]
            assert ((a - r).norm() / r.norm().clamp_min(1e-30)).item() < 20 * TOL_BWD["bf16"], (off, n)
            off += n
    # deterministic
    p2 = net.flat.detach().clone().requires_grad_(True)
    J2 = jet_hip.JetMLPFunction.apply(X, p2, net, plan, "bf16")
    (J2.double() * G).sum().backward()
    assert torch.equal(J2, J) and torch.equal(p2.grad, p.grad)


@pytest.mark.parametrize("prec", PRECS)
def test_jet_deterministic(prec):
    from tensordiffeq_amd.ops import jet_hip
    net, X, plan = _setup([2, 128, 128, 128, 128, 1], [(0,), (1,), (0, 0)], 5000)
    G = torch.randn(plan.S, 5000, 1, device="cuda")
    outs = []
    for _ in range(2):
        p = net.flat.detach().clone().requires_grad_(True)
        J = jet_hip.JetMLPFunction.apply(X, p, net, plan, prec)
        (J * G).sum().backward()
        outs.append(p.grad.clone())
    assert torch.equal(outs[0], outs[1])


def test_adam_multi_matches_reference():
    from tensordiffeq_amd.ops import fused
    from tensordiffeq_amd.optimizers.adam import torch_update
    torch.manual_seed(0)
    shapes = [(50049,), (1000, 1), (7,)]
    ps = [torch.randn(s, device="cuda") for s in shapes]
    gs = [torch.randn(s, device="cuda") for s in shapes]
    ms = [torch.zeros(s, device="cuda") for s in shapes]
    vs = [torch.zeros(s, device="cuda") for s in shapes]
    ref = [(p.clone(), m.clone(), v.clone()) for p, m, v in zip(ps, ms, vs)]
    t = torch.zeros((), dtype=torch.float64, device="cuda")
    for step in range(3):
        t.add_(1)
        fused.adam_multi([(p, g, m, v, -1.0 if i == 1 else 1.0) for i, (p, g, m, v) in enumerate(zip(ps, gs, ms, vs))],
                         t, 0.005, 0.99, 0.999, 1e-7)
        for i, ((p, m, v), g) in enumerate(zip(ref, gs)):
            torch_update(p, g, m, v, t, 0.005, 0.99, 0.999, 1e-7, -1.0 if i == 1 else 1.0)
    for p, (pr, _, _) in zip(ps, ref):
        assert torch.allclose(p, pr, rtol=1e-5, atol=1e-6)


def test_adam_multi_opts_two_optimizers_one_launch():
    """theta descent and SA-weight ascent with their own counters / hyper-parameters in ONE launch,
    plus the best-weights snapshot, against the torch reference update."""
    from tensordiffeq_amd.ops import fused
    from tensordiffeq_amd.optimizers.adam import torch_update
    torch.manual_seed(1)
    p1, g1 = torch.randn(50049, device="cuda"), torch.randn(50049, device="cuda")
    p2, g2 = torch.randn(50513, device="cuda"), torch.randn(50513, device="cuda")
    m1, v1, m2, v2 = (torch.zeros_like(x) for x in (p1, p1, p2, p2))
    r1, r2 = (p1.clone(), m1.clone(), v1.clone()), (p2.clone(), m2.clone(), v2.clone())
    t1 = torch.zeros((), dtype=torch.float64, device="cuda")
    t2 = torch.full((), 7.0, dtype=torch.float64, device="cuda")  # counters need not agree
    best = torch.zeros_like(p1)
    improved = torch.ones((), dtype=torch.int32, device="cuda")
    for _ in range(3):
        t1.add_(1)
        t2.add_(1)
        before = p1.clone()
        fused.adam_multi_opts([([(p1, g1, m1, v1, 1.0)], t1, 0.005, 0.99, 0.999, 1e-7),
                               ([(p2, g2, m2, v2, -1.0)], t2, 0.01, 0.9, 0.99, 1e-6)],
                              snapshot=(best, improved))
        assert torch.equal(best, before)
        torch_update(r1[0], g1, r1[1], r1[2], t1, 0.005, 0.99, 0.999, 1e-7, 1.0)
        torch_update(r2[0], g2, r2[1], r2[2], t2, 0.01, 0.9, 0.99, 1e-6, -1.0)
    assert torch.allclose(p1, r1[0], rtol=1e-5, atol=1e-6)
    assert torch.allclose(p2, r2[0], rtol=1e-5, atol=1e-6)


def test_best_track():
    from tensordiffeq_amd.ops import fused
    flat = torch.randn(1000, device="cuda")
    best = torch.zeros(1000, device="cuda")
    bl = torch.full((), float("inf"), device="cuda")
    be = torch.full((), -1, dtype=torch.int64, device="cuda")
    ep = torch.tensor(3, dtype=torch.int64, device="cuda")
    fused.best_track(torch.tensor(1.5, device="cuda"), bl, flat, best, be, ep)
    assert torch.equal(best, flat) and bl.item() == 1.5 and be.item() == 3
    flat2 = torch.randn(1000, device="cuda")
    fused.best_track(torch.tensor(2.5, device="cuda"), bl, flat2, best, be, ep + 1)
    assert torch.equal(best, flat) and bl.item() == 1.5 and be.item() == 3


@pytest.mark.parametrize("prec", PRECS)
def test_solver_hip_matches_jet_backend(prec):
    import math
    import numpy as np
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, IC, periodicBC

    def build(backend):
        tdq.set_seed(0)
        D = DomainND(["x", "t"], time_var="t")
        D.add("x", [-1.0, 1.0], 512)
        D.add("t", [0.0, 1.0], 201)
        D.generate_collocation_points(3000)

        def deriv_model(u_model, x, t):
            u = u_model(torch.cat([x, t], 1))
            return u, tdq.grad(u, x)

        def f_model(u_model, x, t):
            u = u_model(torch.cat([x, t], 1))
            u_xx = tdq.grad(tdq.grad(u, x), x)
            return tdq.grad(u, t) - 0.0001 * u_xx + 5.0 * u ** 3 - 5.0 * u

        init = IC(D, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]])
        per = periodicBC(D, ["x"], [deriv_model])
        m = tdq.CollocationSolverND(verbose=False)
        g = torch.Generator().manual_seed(1)
        m.compile([2, 128, 128, 128, 128, 1], f_model, D, [init, per], Adaptive_type="self-adaptive",
                  dict_adaptive={"residual": [True], "BCs": [True, False]},
                  init_weights={"residual": [torch.rand(3000, 1, generator=g)],
                                "BCs": [100 * torch.rand(512, 1, generator=g), None]},
                  backend=backend, device="cuda", precision=prec)
        return m

    a, b = build("hip"), build("jet")
    assert a.active_backend == "hip" and b.active_backend == "jet"
    la, ga = a.grad()
    lb, gb = b.grad()
    tl = {"fp32": 1.0, "bf16x3": 10.0, "bf16": 300.0}[prec]
    e_loss = abs(la.item() - lb.item()) / abs(lb.item())
    e_grad = max(((x - y).norm() / y.norm().clamp_min(1e-12)).item() for x, y in zip(ga, gb))
    a.fit(tf_iter=20)
    b.fit(tf_iter=20)
    la, lb = a.losses[-1]["Total Loss"], b.losses[-1]["Total Loss"]
    e_fit = abs(la - lb) / abs(lb)
    print(f"SOLVER_ERR {prec} loss {e_loss:.3e} grad {e_grad:.3e} fit20 {e_fit:.3e}")
    assert e_loss < 1e-5 * tl and e_grad < 1e-4 * tl
    assert e_fit < 1e-3 * tl, (la, lb)


def test_mixed_plan_high_order_periodic():
    """AC-baseline-style program: the residual (order 2) runs on the HIP kernels, the periodic
    u_xxx / u_xxxx boundary segments on the torch jet engine; loss, gradient and a short fit agree
    with the all-torch jet program."""
    import math
    import numpy as np
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, IC, periodicBC

    def build(backend):
        tdq.set_seed(0)
        D = DomainND(["x", "t"], time_var="t")
        D.add("x", [-1.0, 1.0], 512)
        D.add("t", [0.0, 1.0], 201)
        D.generate_collocation_points(3000)

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
                  backend=backend, device="cuda", precision="fp32")
        return m

    a, b = build("auto"), build("jet")
    pa = a.program()
    assert a.active_backend == "hip" and pa.mixed and pa.plan_hi.order == 4 and pa.plan.order == 2
    la, ga = a.grad()
    lb, gb = b.grad()
    assert abs(la.item() - lb.item()) / abs(lb.item()) < 1e-5
    for x, y in zip(ga, gb):
        assert ((x - y).norm() / y.norm().clamp_min(1e-12)).item() < 1e-4
    a.fit(tf_iter=10)
    b.fit(tf_iter=10)
    assert abs(a.losses[-1]["Total Loss"] - b.losses[-1]["Total Loss"]) / b.losses[-1]["Total Loss"] < 1e-3
    Xp = np.random.rand(100, 2)
    u, f = a.predict(Xp)
    assert np.isfinite(u).all() and np.isfinite(f).all()
    # u: the HIP jet's value stream (bf16x3 for a bf16 solver) vs the network in float64
    ws = [(k.detach().double(), b.detach().double()) for k, b in a.u_model.weights()]
    h = torch.as_tensor(Xp, dtype=torch.float64, device=ws[0][0].device)
    for i, (k, b) in enumerate(ws):
        h = torch.addmm(b, h, k)
        h = torch.tanh(h) if i < len(ws) - 1 else h
    err = float(np.abs(u - h.cpu().numpy()).max() / max(1e-6, np.abs(h.cpu().numpy()).max()))
    print(f"PREDICT_U_FP64 {err:.3e}")
    assert err < 1e-4, err


def test_step_book_and_adam_snapshot_match_torch():
    """Native bookkeeping (history row, best loss/epoch, counters, epoch, summed total) and the
    Adam-launch best-weights snapshot equal the torch fallback, over improving and non-improving steps."""
    from tensordiffeq_amd.ops import fused

    def run(device):
        torch.manual_seed(0)
        st = {"hist": torch.full((8, 4), float("nan"), device=device),
              "epoch": torch.zeros((), dtype=torch.int64, device=device),
              "best_loss": torch.full((), float("inf"), device=device),
              "best_epoch": torch.full((), -1, dtype=torch.int64, device=device),
              "improved": torch.zeros((), dtype=torch.int32, device=device),
              "best_flat": torch.zeros(1001, device=device)}
        cnt = [torch.zeros((), dtype=torch.float64, device=device) for _ in range(2)]
        gen = torch.Generator().manual_seed(0)
        p = torch.randn(1001, generator=gen).to(device)
        m, v = torch.zeros_like(p), torch.zeros_like(p)
        snaps = []
        for step, terms in enumerate(([1.0, 2.0, 3.0], [0.5, 0.5, 0.5], [4.0, 0.0, 0.0], [0.1, 0.2, 0.3])):
            tv = torch.tensor(terms, device=device)
            loss = torch.zeros((), device=device)
            fused.step_book(loss, tv, st, cnt, sum_terms=True)   # CPU tensors take the torch fallback
            g = torch.randn(1001, generator=gen).to(device)
            fused.adam_multi([(p, g, m, v, 1.0)], cnt[0], 0.005, 0.99, 0.999, 1e-7,
                             snapshot=(st["best_flat"], st["improved"]))
            snaps.append(st["best_flat"].clone())
        return st, cnt, p, snaps

    a = run("cuda")
    b = run("cpu")
    sa, sb = a[0], b[0]
    assert torch.allclose(sa["hist"][:4].cpu(), sb["hist"][:4], equal_nan=True)
    assert int(sa["epoch"]) == int(sb["epoch"]) == 4
    assert float(sa["best_loss"]) == pytest.approx(float(sb["best_loss"])) == pytest.approx(0.6)
    assert int(sa["best_epoch"]) == int(sb["best_epoch"]) == 3
    assert [float(c) for c in a[1]] == [4.0, 4.0]
    for x, y in zip(a[3], b[3]):
        assert torch.allclose(x.cpu(), y, rtol=1e-5, atol=1e-6)
    assert torch.allclose(a[2].cpu(), b[2], rtol=1e-5, atol=1e-6)


def _ac_sa_model(prec, n_f=3000, sizes=(2, 128, 128, 128, 128, 1), backend="hip"):
    import math
    import numpy as np
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, IC, periodicBC
    tdq.set_seed(0)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 512)
    D.add("t", [0.0, 1.0], 201)
    D.generate_collocation_points(n_f)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return u, tdq.grad(u, x)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_xx = tdq.grad(tdq.grad(u, x), x)
        return tdq.grad(u, t) - 0.0001 * u_xx + 5.0 * u ** 3 - 5.0 * u

    m = tdq.CollocationSolverND(verbose=False)
    g = torch.Generator().manual_seed(1)
    m.compile(list(sizes), f_model, D,
              [IC(D, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]]), periodicBC(D, ["x"], [deriv_model])],
              Adaptive_type="self-adaptive", dict_adaptive={"residual": [True], "BCs": [True, False]},
              init_weights={"residual": [torch.rand(n_f, 1, generator=g)],
                            "BCs": [100 * torch.rand(512, 1, generator=g), None]},
              backend=backend, device="cuda", precision=prec)
    return m


def _poisson_model(prec, n_f=3000, sizes=(2, 128, 128, 128, 128, 1)):
    """2-D Poisson u_xx + u_yy = -2 pi^2 sin(pi x) sin(pi y), zero Dirichlet on the unit square:
    5 jet streams - at width 128 a "wide" plan."""
    import math
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, dirichletBC
    tdq.set_seed(0)
    D = DomainND(["x", "y"])
    D.add("x", [0.0, 1.0], 101)
    D.add("y", [0.0, 1.0], 101)
    D.generate_collocation_points(n_f)

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        u_xx = tdq.grad(tdq.grad(u, x), x)
        u_yy = tdq.grad(tdq.grad(u, y), y)
        return u_xx + u_yy + 2 * math.pi ** 2 * torch.sin(math.pi * x) * torch.sin(math.pi * y)

    bcs = [dirichletBC(D, val=0.0, var=v, target=t) for v in ("x", "y") for t in ("upper", "lower")]
    m = tdq.CollocationSolverND(verbose=False)
    m.compile(list(sizes), f_model, D, bcs, backend="hip", device="cuda", precision=prec)
    return m


TAIL_GEOMS = [
    ("ac", (2, 128, 128, 128, 128, 1)),   # flagship: WT=8, width == W
    ("ac", (2, 64, 128, 96, 1)),          # unequal hidden widths (padded to 128)
    ("ac", (2, 20, 20, 20, 1)),           # WT=2, padded width
    ("ac", (2, 50, 50, 1)),               # WT=4, padded (bf16: 8-wave backward)
    ("ac", (2, 32, 1)),                   # one hidden layer
    ("poisson", (2, 128, 128, 128, 128, 1)),  # wide plan (S=5)
]


@pytest.mark.parametrize("problem,sizes", TAIL_GEOMS)
@pytest.mark.parametrize("prec", ["bf16", "bf16x3"])
def test_fused_step_tail_matches_unfused(prec, problem, sizes, monkeypatch):
    """The two-launch step tail (slab + loss reduction + bookkeeping, then reduction fused into
    Adam with the weight images rewritten in place) reproduces the seven-launch step bit for bit:
    parameters, SA weights, loss history, best loss / epoch / weights - across two fit() calls
    with the parameters changed in between (the images are re-packed before the first replay).
    Geometries: every width class incl. padded widths, one hidden layer, a wide plan."""
    build = _ac_sa_model if problem == "ac" else _poisson_model

    monkeypatch.setenv("TDQ_FUSED_STEP", "0")   # the tail's mechanics on the same kernels both ways

    def run(fused_tail):
        monkeypatch.setenv("TDQ_FUSED_TAIL", "1" if fused_tail else "0")
        m = build(prec, sizes=sizes)
        m.fit(tf_iter=25)
        with torch.no_grad():
            m.u_model.flat.mul_(0.97)
        m.fit(tf_iter=15)
        return m

    a = run(True)
    assert a._get_engine(None, 1)._tail_eligible()
    b = run(False)
    assert torch.equal(a.u_model.flat, b.u_model.flat)
    for x, y in zip(a.lambdas, b.lambdas):
        assert torch.equal(x, y)
    la = [r["Total Loss"] for r in a.losses]
    lb = [r["Total Loss"] for r in b.losses]
    assert la == lb and len(la) == 40
    assert a.min_loss["adam"] == b.min_loss["adam"] and a.best_epoch["adam"] == b.best_epoch["adam"]
    X = torch.rand(300, 2, generator=torch.Generator().manual_seed(3)).numpy()
    u1, _ = a.predict(X, best_model=True)
    u2, _ = b.predict(X, best_model=True)
    assert (u1 == u2).all()


def test_fused_step_tail_large_set_matches_unfused(monkeypatch):
    """300k points (bf16 backward: 2344 slab rows): the slab reduction's chunk count grows past the
    8 of the 50k-point steps (jet_common.h slab_chunks), range cuts land on the new chunk
    boundaries - the fused step still reproduces the unfused one bit for bit, and the loss falls."""
    from tensordiffeq_amd.ops import jet_hip
    from tensordiffeq_amd.ops.jet_mlp import hip_config

    def run(fused_tail):
        monkeypatch.setenv("TDQ_FUSED_TAIL", "1" if fused_tail else "0")
        m = _poisson_model("bf16", n_f=300_000, sizes=(2, 50, 50, 50, 50, 1))
        m.fit(tf_iter=20)
        return m

    a = run(True)
    prog = a.program()
    _, nwg, chunks, _ = jet_hip.slab_geometry(hip_config(prog.net, prog.plan, prog.precision), prog.X_all.shape[0])
    assert nwg >= 2048 and chunks > 8, (nwg, chunks)
    b = run(False)
    assert torch.equal(a.u_model.flat, b.u_model.flat)
    la = [r["Total Loss"] for r in a.losses]
    assert la == [r["Total Loss"] for r in b.losses]
    assert la[-1] < la[0]


@pytest.mark.parametrize("prec", ["bf16", "bf16x3"])
def test_fused_step_tail_discovery_matches_unfused(prec, monkeypatch):
    """DiscoveryModel (PDE coefficients as extra scalars through dscal, SA collocation weights)
    with and without the fused step tail: identical trajectories."""
    import numpy as np
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.models import DiscoveryModel

    def run(fused_tail):
        monkeypatch.setenv("TDQ_FUSED_TAIL", "1" if fused_tail else "0")
        tdq.set_seed(0)
        rng = np.random.default_rng(0)
        X = rng.uniform(-1, 1, (2000, 2)).astype(np.float32)
        X[:, 1] = (X[:, 1] + 1) / 2
        u = (X[:, :1] ** 2 * np.cos(np.pi * X[:, :1])).astype(np.float32)
        params = [tdq.Variable(0.0), tdq.Variable(0.0)]

        def f_model(u_model, var, x, t):
            uu = u_model(torch.cat([x, t], 1))
            u_xx = tdq.grad(tdq.grad(uu, x), x)
            return tdq.grad(uu, t) - var[0] * u_xx + var[1] * uu * uu * uu - var[1] * uu

        m = DiscoveryModel(verbose=False)
        m.compile([2, 64, 64, 64, 1], f_model, [X[:, :1], X[:, 1:]], u, params,
                  col_weights=torch.rand(2000, 1, generator=torch.Generator().manual_seed(0)),
                  backend="hip", device="cuda", precision=prec)
        m.fit(tf_iter=30)
        return m

    a = run(True)
    b = run(False)
    assert torch.equal(a.u_model.flat, b.u_model.flat)
    for x, y in zip(a.vars, b.vars):
        assert torch.equal(x, y)
    assert torch.equal(a.col_weights, b.col_weights)


@pytest.mark.parametrize("problem,sizes", [("ac", (2, 128, 128, 128, 128, 1)), ("ac", (2, 20, 20, 20, 1)),
                                           ("poisson", (2, 128, 128, 128, 128, 1))])
@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
def test_fused_lbfgs_objective_matches_unfused(prec, problem, sizes, monkeypatch):
    """The L-BFGS objective writing ``[grad | loss]`` in place through the fused tail gives the same
    device L-BFGS trajectory, bit for bit, as the loss-reduce / total / slab / concatenate path."""
    build = _ac_sa_model if problem == "ac" else _poisson_model

    monkeypatch.setenv("TDQ_FUSED_STEP", "0")   # same kernels both ways (the fused step: test_fused_step.py)

    def run(fused_tail):
        monkeypatch.setenv("TDQ_FUSED_TAIL", "1" if fused_tail else "0")
        m = build(prec, sizes=sizes)
        m.fit(tf_iter=5, newton_iter=30)
        return m

    a = run(True)
    b = run(False)
    assert torch.equal(a.u_model.flat, b.u_model.flat)
    assert a.min_loss["l-bfgs"] == b.min_loss["l-bfgs"] and np_isfinite(a.min_loss["l-bfgs"])


def np_isfinite(v):
    import math
    return math.isfinite(float(v))


@pytest.mark.parametrize("prec", ["bf16x3", "bf16"])
def test_solver_unequal_widths_hip_matches_jet(prec):
    """A network with unequal hidden widths trains on the HIP kernels (padded to the widest layer)
    and matches the torch jet engine's loss and gradients."""
    sizes = (2, 64, 128, 96, 1)
    a = _ac_sa_model(prec, sizes=sizes)
    b = _ac_sa_model(prec, sizes=sizes, backend="jet")
    assert a.active_backend == "hip" and b.active_backend == "jet"
    with torch.no_grad():
        b.u_model.flat.copy_(a.u_model.flat)
    la, ga = a.grad()
    lb, gb = b.grad()
    tol = {"bf16x3": 1e-4, "bf16": 3e-2}[prec]
    assert abs(la.item() - lb.item()) / abs(lb.item()) < tol
    for x, y in zip(ga, gb):
        assert ((x - y).norm() / y.norm().clamp_min(1e-12)).item() < 10 * tol
    a.fit(tf_iter=10)
    assert all(np_isfinite(r["Total Loss"]) for r in a.losses)


@pytest.mark.parametrize("prec,cuts", [("bf16x3", "0.4"), ("bf16", "0.5"), ("bf16", "0.3")])
def test_point_ranges_match_single_launch(prec, cuts, monkeypatch):
    """Point ranges on concurrent graph branches (fit.point_ranges: forward -> fused loss ->
    backward per range, one stream each) keep every workgroup's index and buffers, so the Adam
    trajectory, the L-BFGS objective and the L-BFGS trajectory are bitwise those of single
    launches."""
    res = []
    monkeypatch.setenv("TDQ_FUSED_STEP", "0")   # point ranges serve the separate-launch step
    for split in ("0", cuts):
        monkeypatch.setenv("TDQ_SPLIT", split)
        m = _ac_sa_model(prec, n_f=20000)
        m.fit(tf_iter=40)
        eng = m._get_engine(None, 1)
        assert (eng._ranges is None) == (split == "0")
        hist = [h["Total Loss"] for h in m.losses]
        flat = m.u_model.flat.detach().clone()
        lam = m.lambdas[0].detach().clone()
        from tensordiffeq_amd.fit import LossGradEngine
        le = LossGradEngine(m, m.program(precision=prec), m.lambdas)
        f0, g0 = le(m.u_model.flat.detach().clone())
        assert (le._ranges is None) == (split == "0")
        m.fit(newton_iter=30)
        res.append((hist, flat, lam, float(f0), g0.clone(), m.u_model.flat.detach().clone()))
    a, b = res
    assert a[0] == b[0]
    assert torch.equal(a[1], b[1]) and torch.equal(a[2], b[2])
    assert a[3] == b[3] and torch.equal(a[4], b[4])
    assert torch.equal(a[5], b[5])
