"""LHS sampler properties and forward-mode jet engine vs nested autograd."""
import numpy as np
import pytest
import torch

from tensordiffeq_amd.jet import JetPlan, closure, faa_terms, jet_forward, tanh_poly
from tensordiffeq_amd.models.networks import TanhMLP
from tensordiffeq_amd.sampling import LHS, lhs_device, lhs_unit


@pytest.mark.parametrize("crit", ["c", "center", "r", "m", "cm", "corr", "ese"])
def test_lhs_one_point_per_stratum(crit):
    n = 40 if crit == "ese" else 200
    u = lhs_unit(n, 3, crit, random_state=0)
    assert u.shape == (n, 3)
    for j in range(3):
        strata = np.floor(u[:, j] * n).astype(int)
        assert sorted(strata) == list(range(n))
    if crit in ("c", "center", "cm"):
        np.testing.assert_allclose(np.sort(u[:, 0]), (np.arange(n) + 0.5) / n)


def test_lhs_scaling_and_seed():
    xl = np.array([[-1.0, 1.0], [0.0, 5.0]])
    a = LHS(xlimits=xl, random_state=7)(100)
    b = LHS(xlimits=xl, random_state=7)(100)
    np.testing.assert_array_equal(a, b)
    assert a[:, 0].min() > -1 and a[:, 1].max() < 5


def test_lhs_device_cpu():
    x = lhs_device(1000, [[-1, 1], [0, 1]], "cpu", generator=torch.Generator().manual_seed(0))
    strata = torch.floor((x[:, 0] + 1) / 2 * 1000).long()
    assert torch.equal(torch.sort(strata).values, torch.arange(1000))


def test_closure_and_faa():
    assert closure([(0, 0)]) == [(), (0,), (0, 0)]
    assert closure([(0, 1, 1)]) == [(), (0,), (1,), (0, 1), (1, 1), (0, 1, 1)]
    # d3 tanh: s1 z_xxx + 3 s2 z_x z_xx + s3 z_x^3
    t = {(k, b): c for k, b, c in faa_terms((0, 0, 0))}
    assert t[(1, ((0, 0, 0),))] == 1 and t[(2, ((0,), (0, 0)))] == 3 and t[(3, ((0,), (0,), (0,)))] == 1
    assert tanh_poly(1) == (1.0, 0.0, -1.0)          # 1 - h^2
    assert tanh_poly(2) == (0.0, -2.0, 0.0, 2.0)     # -2h + 2h^3


@pytest.mark.parametrize("sizes", [[2, 16, 16, 1], [3, 8, 8, 8, 2], [1, 12, 1]])
def test_jet_matches_nested_autograd(sizes):
    torch.manual_seed(0)
    d = sizes[0]
    net = TanhMLP(sizes).double()
    with torch.no_grad():
        net.flat.add_(0.1 * torch.randn_like(net.flat))
    reqs = [(0,), (0, 0), (0, 0, 0), (0, 0, 0, 0)]
    if d > 1:
        reqs += [(0, 1), (1, 1), (0, 1, 1)]
    if d > 2:
        reqs += [(0, 1, 2), (2, 2)]
    plan = JetPlan(reqs, d)
    X = torch.randn(9, d, dtype=torch.float64)
    J = jet_forward(X, net.weights(), plan)
    cols = [X[:, j:j + 1].clone().requires_grad_(True) for j in range(d)]
    u = net(torch.cat(cols, 1))
    for i, mi in enumerate(plan.streams):
        for o in range(sizes[-1]):
            y = u[:, o:o + 1]
            for v in mi:
                y = torch.autograd.grad(y.sum(), cols[v], create_graph=True)[0]
            assert torch.allclose(y[:, 0], J[i, :, o], atol=1e-10, rtol=1e-9), mi


def test_jet_gradients_match_autograd():
    torch.manual_seed(1)
    net = TanhMLP([2, 10, 10, 1]).double()
    plan = JetPlan([(0,), (1,), (0, 0)], 2)
    X = torch.randn(7, 2, dtype=torch.float64)
    p = net.flat.detach().clone().requires_grad_(True)
    J = jet_forward(X, net.weights(p), plan)
    G = torch.randn_like(J)
    g1 = torch.autograd.grad((J * G).sum(), p)[0]
    # reference: nested autograd residual-style functional
    cols = [X[:, j:j + 1].clone().requires_grad_(True) for j in range(2)]
    p2 = net.flat.detach().clone().requires_grad_(True)
    u = net(torch.cat(cols, 1), params=p2)
    ux = torch.autograd.grad(u.sum(), cols[0], create_graph=True)[0]
    ut = torch.autograd.grad(u.sum(), cols[1], create_graph=True)[0]
    uxx = torch.autograd.grad(ux.sum(), cols[0], create_graph=True)[0]
    f = (torch.stack([u, ux, ut, uxx]) * G).sum()
    g2 = torch.autograd.grad(f, p2)[0]
    assert torch.allclose(g1, g2, atol=1e-10)


def test_hip_config_unequal_widths():
    """Unequal hidden widths are served by the split-bf16 kernels (padded to the widest layer);
    an exact-fp32 request with unequal widths keeps fp32 on the layer-wise engine."""
    from tensordiffeq_amd.jet import JetPlan
    from tensordiffeq_amd.models.networks import TanhMLP
    from tensordiffeq_amd.ops.jet_mlp import hip_config
    net = TanhMLP([2, 64, 128, 32, 1], device="cpu")
    plan = JetPlan([(0,), (1,), (0, 0)], 2)
    cfg = hip_config(net, plan, "bf16")
    assert cfg["WT"] == 8 and cfg["widths"] == (64, 128, 32) and cfg["width"] == 128
    cfg32 = hip_config(net, plan, "fp32")
    assert cfg32["precision"] == "fp32" and cfg32["engine"] == "layered" and "unequal" in cfg32["why"]
    cfg = hip_config(TanhMLP([2, 128, 128, 128, 128, 1], device="cpu"), JetPlan([(0, 0), (1, 1)], 2), "bf16")
    assert cfg["S"] == 5 and cfg["WT"] == 8   # a wide plan


def test_hip_config_wide_hidden_layers_use_layered_engine():
    """Hidden widths > 128 leave the fused kernels' envelope except in bf16 with S <= 4 up to
    width 256 (WT = 16); elsewhere the layer-wise engine serves them (library GEMMs in the
    requested precision + HIP epilogues), never the fused tail / point ranges."""
    from tensordiffeq_amd.jet import JetPlan
    from tensordiffeq_amd.models.networks import TanhMLP
    from tensordiffeq_amd.ops import jet_hip
    from tensordiffeq_amd.ops.jet_mlp import hip_config
    ac = JetPlan([(0,), (1,), (0, 0)], 2)
    cfg = hip_config(TanhMLP([2, 256, 256, 1], device="cpu"), ac, "bf16")
    assert not jet_hip.is_layered(cfg) and cfg["WT"] == 16 and jet_hip.is_split_bf16(cfg)
    for prec in ("bf16x3", "fp32"):
        cfg = hip_config(TanhMLP([2, 256, 256, 1], device="cpu"), ac, prec)
        assert jet_hip.is_layered(cfg) and cfg["precision"] == prec
    assert jet_hip.is_layered(hip_config(TanhMLP([2, 272, 1], device="cpu"), ac, "bf16"))
    assert jet_hip.is_layered(hip_config(TanhMLP([2, 256, 1], device="cpu"), JetPlan([(0, 0), (1, 1)], 2), "bf16"))
    cfg = hip_config(TanhMLP([2, 64, 200, 1], device="cpu"), JetPlan([(0, 0)], 2), "bf16x3")
    assert jet_hip.is_layered(cfg) and cfg["widths"] == (64, 200)
    assert not jet_hip.is_layered(hip_config(TanhMLP([2, 128, 1], device="cpu"), JetPlan([], 2), "bf16"))
