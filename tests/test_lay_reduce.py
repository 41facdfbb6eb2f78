"""The layer-wise engine's fixed-order HIP kernels (csrc/lay_reduce.hip) against torch in float64:
column sums over few / many rows (one and two passes), strided and transposed destinations, the
bias on the first elements; the bf16 weight planes (transposed or not, hi + lo); the input-layer
gradient from its summed partials.  Run-to-run bitwise determinism of the column sum."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _dev():
    return torch.device("cuda", 0)


@pytest.mark.parametrize("R,M", [(1, 7), (8, 262144), (37, 1000), (1563, 512), (50914, 1), (50000, 2), (4096, 96)])
def test_colsum_matches_fp64(R, M):
    from tensordiffeq_amd.ops.jet_layered import _colsum
    g = torch.Generator(device="cuda").manual_seed(R * 7 + M)
    src = torch.randn(R, M, device=_dev(), generator=g)
    out = torch.empty(M, device=_dev())
    _colsum(src, R, M, out)
    ref = src.double().sum(0)
    err = ((out.double() - ref).abs().max() / ref.abs().max().clamp_min(1e-30)).item()
    assert err < 1e-5 * max(1.0, R ** 0.5 / 10), err
    again = torch.empty_like(out)
    _colsum(src, R, M, again)
    assert torch.equal(out, again)


def test_colsum_strided_transposed_destination_and_bias():
    from tensordiffeq_amd.ops.jet_layered import _colsum
    R, nj, W = 300, 3, 64
    src = torch.randn(R, nj, W, device=_dev())
    big = torch.zeros(W, 5, device=_dev())          # out[f][j0 + j], j0 = 1
    _colsum(src, R, nj * W, big[:, 1:], W=W, sj=big.stride(1), sf=big.stride(0))
    ref = src.double().sum(0).t()
    assert torch.allclose(big[:, 1:1 + nj].double(), ref, rtol=1e-5, atol=1e-4)
    assert (big[:, 0] == 0).all() and (big[:, 1 + nj:] == 0).all()
    # bias on the first nbias elements (J's value stream)
    S, N, d_out = 3, 100, 2
    part = torch.randn(4, S * N * d_out, device=_dev())
    bo = torch.tensor([0.5, -2.0], device=_dev())
    J = torch.empty(S, N, d_out, device=_dev())
    _colsum(part, 4, S * N * d_out, J, bias=bo, nbias=N * d_out)
    ref = part.double().sum(0).view(S, N, d_out)
    ref[0] += bo.double()
    assert torch.allclose(J.double(), ref, rtol=1e-6, atol=1e-5)


@pytest.mark.parametrize("prec", ["bf16", "bf16x3"])
@pytest.mark.parametrize("transpose", [False, True])
def test_bplanes(prec, transpose):
    from tensordiffeq_amd.ops.jet_layered import _bplanes
    K = torch.randn(96, 160, device=_dev())
    bt = K.t() if transpose else K
    op = _bplanes(bt, prec)
    assert op.h.shape == bt.shape and op.h.dtype == torch.bfloat16
    assert torch.equal(op.h, bt.to(torch.bfloat16))
    if prec == "bf16x3":
        assert torch.equal(op.l, (bt - op.h.float()).to(torch.bfloat16))
    else:
        assert not hasattr(op, "l")


def test_l0grad():
    import ctypes
    from tensordiffeq_amd.ops import _lib
    S, d_in, W0 = 4, 2, 128
    spec = [0, 0, 0, 1, 0, 0, 1, 1, 0, 2, 0, 0]   # value, u_x, u_t, u_xx
    tot = torch.randn(S + d_in, W0, device=_dev())
    dK0 = torch.empty(d_in, W0, device=_dev())
    b0 = torch.empty(W0, device=_dev())
    lib = _lib.load(required=True)
    c = (ctypes.c_int * len(spec))(*spec)
    _lib.check(lib.tdq_lay_l0grad(_lib.ptr(tot), S, d_in, c, W0, _lib.ptr(dK0), _lib.ptr(b0),
                                  _lib.stream_ptr(tot.device)), "tdq_lay_l0grad")
    ref = tot[S:].clone()
    ref[0] += tot[1]
    ref[1] += tot[2]
    assert torch.allclose(dK0, ref, rtol=1e-6, atol=1e-6)
    assert torch.equal(b0, tot[0])
