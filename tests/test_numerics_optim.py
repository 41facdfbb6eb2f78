"""Loss primitives, flat parameter layout / Keras interop, Keras-Adam formula, L-BFGS."""
import math

import numpy as np
import pytest
import torch

import tensordiffeq_amd as tdq
from tensordiffeq_amd.checkpoint import flat_from_keras, keras_arrays
from tensordiffeq_amd.models.networks import TanhMLP
from tensordiffeq_amd.optimizers import Adam, Struct, compact_direction, eager_lbfgs, graph_lbfgs
from tensordiffeq_amd.optimizers.lbfgs import _History
from tensordiffeq_amd.utils import MSE, g_MSE, get_sizes, get_weights, initialize_weights_loss, set_weights


def test_mse_variants():
    p = torch.tensor([[1.0], [2.0], [4.0]])
    a = torch.zeros(3, 1)
    w = torch.tensor([[1.0], [2.0], [0.5]])
    assert MSE(p, a).item() == pytest.approx((1 + 4 + 16) / 3)
    assert MSE(p, a, w).item() == pytest.approx((1 + 16 + 4) / 3)            # mean((w r)^2)
    assert MSE(p, a, torch.tensor(3.0), True).item() == pytest.approx(3 * 7)  # w * mean(r^2)
    assert g_MSE(p, a, w ** 2).item() == pytest.approx((1 + 16 + 4) / 3)
    assert MSE(p, a, denom=6.0).item() == pytest.approx(21 / 6)


def test_initialize_weights_loss_map():
    lam, m = initialize_weights_loss({"residual": [torch.ones(5, 1)], "BCs": [torch.ones(3, 1), None]},
                                     {"residual": [True], "BCs": [True, False]})
    assert len(lam) == 2 and m == {"residual": [0], "bcs": [1]}


def test_flat_layout_matches_keras_order():
    net = TanhMLP([2, 3, 4, 1])
    assert get_sizes([2, 3, 4, 1]) == ([6, 12, 4], [3, 4, 1])
    w = get_weights(net)
    assert w.numel() == 6 + 3 + 12 + 4 + 4 + 1
    # kernel (in, out) row-major then bias
    k0 = net.kernel(0)
    assert torch.equal(w[:6], k0.reshape(-1)) and torch.equal(w[6:9], net.bias(0))
    arr = keras_arrays(net)
    np.testing.assert_array_equal(arr["dense/kernel:0"], k0.detach().numpy())
    flat, sizes = flat_from_keras(arr)
    np.testing.assert_array_equal(flat, w.numpy())
    net2 = TanhMLP([2, 3, 4, 1])
    set_weights(net2, w)
    x = torch.randn(5, 2)
    assert torch.allclose(net(x), net2(x))


def test_glorot_normal_truncation_and_scale():
    torch.manual_seed(0)
    net = TanhMLP([200, 200, 1])
    k = net.kernel(0)
    std = math.sqrt(2 / 400) / 0.87962566103423978
    assert k.abs().max().item() <= 2 * std + 1e-6
    assert abs(k.std().item() / math.sqrt(2 / 400) - 1) < 0.05
    assert torch.all(net.bias(0) == 0)


def test_keras_adam_formula():
    p = torch.tensor([1.0, -2.0], dtype=torch.float64)
    opt = Adam(lr=0.005, beta_1=0.99)
    gs = [torch.tensor([0.3, -0.1], dtype=torch.float64), torch.tensor([0.2, 0.5], dtype=torch.float64)]
    ref = p.clone()
    m = torch.zeros(2, dtype=torch.float64)
    v = torch.zeros(2, dtype=torch.float64)
    for t, g in enumerate(gs, start=1):
        opt.apply_gradients([(g, p)])
        m = 0.99 * m + 0.01 * g
        v = 0.999 * v + 0.001 * g * g
        lr_t = 0.005 * math.sqrt(1 - 0.999 ** t) / (1 - 0.99 ** t)
        ref = ref - lr_t * m / (v.sqrt() + 1e-7)
    assert torch.allclose(p, ref, atol=1e-12)
    assert opt.iterations == 2


def _two_loop(g, S, Y, hdiag):
    q = -g.copy()
    al = []
    for s, y in reversed(list(zip(S, Y))):
        a = s @ q / (y @ s)
        al.append(a)
        q = q - a * y
    r = q * hdiag
    for (s, y), a in zip(zip(S, Y), reversed(al)):
        b = y @ r / (y @ s)
        r = r + (a - b) * s
    return r


def test_compact_lbfgs_equals_two_loop():
    rng = np.random.default_rng(0)
    p, m = 30, 7
    hist = _History(5, p, "cpu", torch.float64)
    S, Y = [], []
    A = rng.standard_normal((p, p))
    A = A @ A.T + p * np.eye(p)
    for _ in range(m):
        s = rng.standard_normal(p)
        y = A @ s
        hist.push(torch.tensor(s), torch.tensor(y))
        S.append(s)
        Y.append(y)
    S, Y = S[-5:], Y[-5:]
    g = rng.standard_normal(p)
    hd = 0.37
    d = compact_direction(torch.tensor(g), hist, hd).numpy()
    np.testing.assert_allclose(d, _two_loop(g, S, Y, hd), rtol=1e-8, atol=1e-10)


def test_eager_lbfgs_rosenbrock():
    def f(x):
        x = x.detach().clone().requires_grad_(True)
        v = (1 - x[0]) ** 2 + 100 * (x[1] - x[0] ** 2) ** 2
        g = torch.autograd.grad(v, x)[0]
        return v.detach(), g
    x0 = torch.tensor([-1.2, 1.0], dtype=torch.float64)
    x, hist, nev, best, fmin, ep = eager_lbfgs(f, x0, Struct(), maxIter=400, learningRate=0.8)
    assert fmin < float(f(x0)[0]) * 1e-3
    assert nev <= 400 * 1.25 + 1


def test_graph_lbfgs_quadratic():
    A = torch.diag(torch.arange(1.0, 11.0, dtype=torch.float64))

    def f(x):
        return 0.5 * x @ A @ x, A @ x
    x, n = graph_lbfgs(f, torch.ones(10, dtype=torch.float64), 50)
    assert x.abs().max() < 1e-6


def test_group_array_layout_and_limits():
    """The ctypes AdamGroup block used by the single-launch Adam / fused step tail: one row per
    tensor (theta first), refusing what one launch cannot take (non-contiguous, > 16 tensors)."""
    import torch
    from tensordiffeq_amd.ops import fused
    t = torch.zeros((), dtype=torch.float64)
    p, g, m, v = (torch.zeros(10) for _ in range(4))
    lam = [torch.zeros(5) for _ in range(4)]
    groups = [([(p, g, m, v, 1.0)], t, 0.005, 0.99, 0.999, 1e-7),
              ([(x, x, x, x, -1.0) for x in lam], t, 0.01, 0.9, 0.999, 1e-7)]
    arr, n = fused.group_array(groups)
    assert n == 5 and arr[0].n == 10 and arr[0].sign == 1.0 and arr[1].sign == -1.0
    assert arr[0].p == p.data_ptr() and abs(arr[1].lr - 0.01) < 1e-9
    big = [([(p, g, m, v, 1.0)] * 17, t, 0.005, 0.99, 0.999, 1e-7)]
    assert fused.group_array(big) is None
    nc = torch.zeros(10, 2)[:, 0]
    assert fused.group_array([([(nc, nc, nc, nc, 1.0)], t, 0.005, 0.99, 0.999, 1e-7)]) is None


def test_fused_tail_off_on_cpu():
    """The fused step tail is a GPU path: a CPU engine keeps the reference-order Adam step."""
    import tensordiffeq_amd as tdq
    from tests.test_solver import burgers
    D, bcs, f_model = burgers(n_f=200)
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 16, 16, 1], f_model, D, bcs)
    eng = m._get_engine(None, 5)
    assert eng._tail_eligible() is False
    m.fit(tf_iter=3)
    assert len(m.losses) == 3
