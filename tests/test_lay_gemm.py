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
