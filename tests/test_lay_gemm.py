"""Hand-written MFMA GEMMs of the layer-wise engine (csrc/lay_gemm.hip) against float64 torch:
NN (forward / backward shape, B given transposed) and TN (weight gradient, row-chunk partials) in
the bf16, bf16x3 and fp32 families, on shapes with tails in every dimension (M, N, K not multiples
of the tiles; K not a multiple of 8 takes the element-wise load path)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

SHAPES = [(1000, 300, 256), (130, 512, 512), (777, 1, 200), (64, 129, 33), (4096, 256, 160)]
TOL = {"fp32": 2e-6, "bf16x3": 2e-5, "bf16": 1.5e-2}


def _ops(x, prec):
    from tensordiffeq_amd.ops.jet_layered import _Op
    return _Op(x.contiguous(), prec)


@pytest.mark.parametrize("prec", ["fp32", "bf16x3", "bf16"])
@pytest.mark.parametrize("M,N,K", SHAPES)
def test_nn_matches_fp64(M, N, K, prec):
    from tensordiffeq_amd.ops import jet_layered
    torch.manual_seed(0)
    A = torch.randn(M, K, device="cuda")
    B = torch.randn(K, N, device="cuda") / K ** 0.5
    C = jet_layered._mm_w(_ops(A, prec), B, prec)
    ref = A.double() @ B.double()
    err = ((C.double() - ref).norm() / ref.norm()).item()
    print(f"LAY_NN {prec} {M}x{N}x{K} rel {err:.2e}")
    assert err < TOL[prec], err


@pytest.mark.parametrize("prec", ["fp32", "bf16x3", "bf16"])
@pytest.mark.parametrize("L,Ma,Nb", [(20000, 256, 256), (3001, 129, 512), (100, 64, 1), (65536, 512, 33)])
def test_tn_matches_fp64(L, Ma, Nb, prec):
    from tensordiffeq_amd.ops import jet_layered
    torch.manual_seed(1)
    A = torch.randn(L, Ma, device="cuda")
    B = torch.randn(L, Nb, device="cuda") / L ** 0.5
    out = torch.empty(Ma, Nb, device="cuda")
    jet_layered._mm_tn(_ops(A, prec), _ops(B, prec), out)
    ref = A.double().t() @ B.double()
    err = ((out.double() - ref).norm() / ref.norm()).item()
    print(f"LAY_TN {prec} L={L} {Ma}x{Nb} rel {err:.2e}")
    assert err < TOL[prec], err


def test_layer0_xtz_matches_fp64():
    from tensordiffeq_amd.ops import _lib
    torch.manual_seed(2)
    N, d, W = 5001, 3, 300
    X = torch.rand(N, d, device="cuda")
    Z = torch.randn(N, W, device="cuda")
    rows = 256
    part = torch.empty(((N + rows - 1) // rows, d, W), device="cuda")
    lib = _lib.load(required=True)
    _lib.check(lib.tdq_lay_xtz(_lib.ptr(X), d, _lib.ptr(Z), N, W, _lib.ptr(part), rows, _lib.stream_ptr(X.device)),
               "tdq_lay_xtz")
    out = part.sum(0)
    ref = X.double().t() @ Z.double()
    assert ((out.double() - ref).norm() / ref.norm()).item() < 1e-6


@pytest.mark.parametrize("prec", ["bf16x3", "bf16", "fp32"])
@pytest.mark.parametrize("sizes,reqs,N", [
    ([2, 256, 256, 256, 1], [(0,), (1,), (0, 0)], 1000),
    ([3, 132, 64, 1], [(0,), (1,), (2,), (0, 0), (1, 1), (0, 1)], 333),   # S = 7: 18-point tiles
    ([2, 512, 512, 1], [(0,), (1,)], 130),                              # S = 3: 42-point tiles
    ([2, 96, 1], [(0, 0)], 77),                                         # one hidden layer
])
def test_gemm_epilogue_path_matches_standalone_pass(sizes, reqs, N, prec, monkeypatch):
    """The GEMM-epilogue path (the layer jet inside tdq_lay_in_fwd / tdq_lay_nnj / tdq_lay_out_bwd,
    activations kept only as hi / lo bf16 planes, the input layer's gradient as tile partials)
    against the GEMM + standalone epilogue pass, both compared to the float64 jet + autograd: the
    epilogue path is no less accurate, and within 1e-5 of the standalone path in bf16x3 / fp32.  (Not
    bitwise: the input layer's X K0 is summed in another order, the adjoint reads H = hi + lo -
    relative 2^-16 - and the output layer's dKo comes from exact-fp32 FMA partials.)"""
    from tensordiffeq_amd.jet import JetPlan, jet_forward
    from tensordiffeq_amd.models.networks import TanhMLP
    from tensordiffeq_amd.ops import jet_layered
    torch.manual_seed(3)
    net = TanhMLP(sizes, device="cuda")
    with torch.no_grad():
        net.flat.add_(0.05 * torch.randn_like(net.flat))
    X = torch.rand(N, sizes[0], device="cuda") * 2 - 1
    plan = JetPlan(reqs, sizes[0])
    P = net.flat.detach()
    G = torch.randn(plan.S, N, sizes[-1], device="cuda")
    p64 = P.double().clone().requires_grad_(True)
    Jr = jet_forward(X.double(), net.weights(p64), plan)
    (Jr * G.double()).sum().backward()
    gr, Jr = p64.grad, Jr.detach()
    out = {}
    for fused in ("1", "0"):
        monkeypatch.setenv("TDQ_LAY_FUSED", fused)
        J, saved = jet_layered.forward_raw(X, P, net, plan, prec)
        assert saved[-1] == (fused == "1")
        out[fused] = (J.clone(), jet_layered.backward_raw(saved, G).double())
    (J1, g1), (J0, g0) = out["1"], out["0"]
    scale = Jr.abs().amax(dim=(1, 2), keepdim=True).clamp_min(1e-3)
    f1, f0 = (((J.double() - Jr).abs() / scale).max().item() for J in (J1, J0))
    e1, e0 = ((g1 - gr).norm() / gr.norm()).item(), ((g0 - gr).norm() / gr.norm()).item()
    rel = ((g1 - g0).norm() / g0.norm()).item()
    print(f"LAY_NNJ {prec} {sizes} S={plan.S} vs fp64: fwd {f1:.2e} (standalone {f0:.2e}), grad {e1:.2e} "
          f"(standalone {e0:.2e}); grads between {rel:.2e}")
    assert f1 <= 1.2 * f0 + 1e-6, (f1, f0)
    assert e1 <= 1.1 * e0 + 1e-6, (e1, e0)
    if prec != "bf16":
        assert rel < 1e-5, rel
