"""Layer-wise jet engine (ops/jet_layered.py): stacked-stream GEMMs + fused tanh-jet epilogues.

CPU (float64, torch epilogues): forward streams and the flat parameter gradient against the torch
jet engine + autograd.  GPU (``-m gpu``): the HIP epilogues (csrc/jet_layered.hip) through the
normal HIP dispatch for hidden widths > 128, against the float64 reference.
"""
import pytest
import torch

from tensordiffeq_amd.jet import JetPlan, jet_forward
from tensordiffeq_amd.models.networks import TanhMLP

CASES = [
    ([2, 24, 24, 24, 1], [(0,), (1,), (0, 0)], 37),
    ([3, 20, 16, 2], [(0, 0), (1, 1), (0, 1), (2,)], 29),
    ([2, 16, 1], [], 11),
    ([1, 12, 12, 1], [(0, 0)], 17),
]
GPU_CASES = [
    ([2, 256, 256, 256, 256, 1], [(0,), (1,), (0, 0)], 1000),   # AC plan at width 256
    ([3, 256, 256, 1], [(0,), (1,), (2,), (0, 0), (1, 1), (0, 1)], 301),   # S=7, mixed derivative
    ([2, 160, 320, 200, 2], [(0, 0), (1, 1)], 257),               # unequal widths > 128, d_out 2
    ([2, 512, 512, 1], [(0,), (1,)], 130),
]


def _setup(sizes, reqs, N, device, dtype, seed=0):
    torch.manual_seed(seed)
    net = TanhMLP(sizes, device=device)
    with torch.no_grad():
        net.flat.add_(0.05 * torch.randn_like(net.flat))
    X = (torch.rand(N, sizes[0], device=device) * 2 - 1)
    return net, X.to(dtype), JetPlan(reqs, sizes[0])


def _ref(net, X, plan, G):
    p64 = net.flat.detach().double().clone().requires_grad_(True)
    Jr = jet_forward(X.double(), net.weights(p64), plan)
    (Jr * G.double()).sum().backward()
    return Jr.detach(), p64.grad


@pytest.mark.parametrize("sizes,reqs,N", CASES)
def test_layered_engine_cpu_float64(sizes, reqs, N):
    from tensordiffeq_amd.ops import jet_layered
    net, X, plan = _setup(sizes, reqs, N, "cpu", torch.float64)
    P = net.flat.detach().double()
    J, saved = jet_layered.forward_raw(X, P, net, plan)
    G = torch.randn(plan.S, N, sizes[-1], dtype=torch.float64)
    g = jet_layered.backward_raw(saved, G)
    Jr, gr = _ref(net, X, plan, G)
    assert torch.allclose(J, Jr, rtol=1e-10, atol=1e-12)
    assert torch.allclose(g, gr, rtol=1e-9, atol=1e-11)


@pytest.mark.gpu
@pytest.mark.parametrize("sizes,reqs,N", GPU_CASES)
def test_layered_engine_hip(sizes, reqs, N):
    from tensordiffeq_amd.ops import jet_hip, jet_mlp
    net, X, plan = _setup(sizes, reqs, N, "cuda", torch.float32, seed=1)
    cfg = jet_mlp.hip_config(net, plan, "bf16")
    assert jet_hip.is_layered(cfg) and not jet_hip.is_split_bf16(cfg)
    p = net.flat.detach().clone().requires_grad_(True)
    J = jet_hip.JetMLPFunction.apply(X, p, net, plan, "bf16")
    G = torch.randn(plan.S, N, sizes[-1], device="cuda", dtype=torch.float64)
    (J.double() * G).sum().backward()
    Jr, gr = _ref(net, X, plan, G)
    scale = Jr.abs().amax(dim=(1, 2), keepdim=True).clamp_min(1e-3)
    ferr = ((J.detach().double() - Jr).abs() / scale).max().item()
    rel = ((p.grad.double() - gr).norm() / gr.norm()).item()
    print(f"KERNEL_ERR layered {sizes} S={plan.S} fwd {ferr:.3e} bwd {rel:.3e}")
    # fp32 library GEMMs: forward error grows with the reduction length (measured 3.5e-6 at width
    # 256, 2.1e-5 at 512; gpurun_out r3u)
    assert ferr < 2e-5 * max(1, max(sizes[1:-1]) // 256) and rel < 2e-5, (ferr, rel)


@pytest.mark.gpu
def test_layered_engine_trains_wide_solver():
    """A width-256 Allen-Cahn SA-PINN picks the HIP backend (layered engine + fused loss) and
    follows the torch-jet trajectory (both fp32) through Adam and L-BFGS steps."""
    import bench
    from tensordiffeq_amd.ops import jet_hip, jet_mlp
    layers = (2, 256, 256, 256, 1)
    hist = {}
    for backend in ("auto", "jet"):
        m = bench.build_problem(4096, 1, backend, torch.device("cuda", 0), False, "bf16", layers=layers)
        if backend == "auto":
            assert m.active_backend == "hip"
            prog = m._get_engine(None, 10).program
            assert jet_hip.is_layered(jet_mlp.hip_config(prog.net, prog.plan, prog.precision))
        m.fit(tf_iter=6)
        m.fit(newton_iter=3)
        hist[backend] = ([h["Total Loss"] for h in m.losses], float(m.min_loss["l-bfgs"]))
    assert hist["auto"][0] == pytest.approx(hist["jet"][0], rel=2e-4)
    assert hist["auto"][1] == pytest.approx(hist["jet"][1], rel=2e-3)
