"""Per-parameter-block relative error of the HIP jet backward against autograd through the torch
jet (GPU debugging aid): python tools/debug_bwd_blocks.py [--prec bf16x3]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tensordiffeq_amd.jet import JetPlan, jet_forward  # noqa: E402
from tensordiffeq_amd.models.networks import TanhMLP  # noqa: E402
from tensordiffeq_amd.ops import jet_hip  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--prec", default="bf16x3")
    ap.add_argument("--sizes", default="2,128,128,128,128,1")
    ap.add_argument("--n", type=int, default=1000)
    ap.add_argument("--reqs", default="0;1;0,0")
    a = ap.parse_args()
    sizes = [int(v) for v in a.sizes.split(",")]
    reqs = [tuple(int(x) for x in r.split(",")) for r in a.reqs.split(";") if r]
    torch.manual_seed(1)
    net = TanhMLP(sizes, device="cuda")
    with torch.no_grad():
        net.flat.add_(0.05 * torch.randn_like(net.flat))
    X = (torch.rand(a.n, sizes[0], device="cuda") * 2 - 1).contiguous()
    plan = JetPlan(reqs, sizes[0])
    G = torch.randn(plan.S, a.n, sizes[-1], device="cuda", dtype=torch.float64)
    p = net.flat.detach().clone().requires_grad_(True)
    J = jet_hip.JetMLPFunction.apply(X, p, net, plan, a.prec)
    (J.double() * G).sum().backward()
    g_hip = p.grad.double()
    p64 = net.flat.detach().double().clone().requires_grad_(True)
    Jr = jet_forward(X.double(), net.weights(p64), plan)
    (Jr * G).sum().backward()
    g_ref = p64.grad
    print("total rel", ((g_hip - g_ref).norm() / g_ref.norm()).item())
    off = 0
    for li in range(len(sizes) - 1):
        for name, n in (("K", sizes[li] * sizes[li + 1]), ("b", sizes[li + 1])):
            h, r = g_hip[off:off + n], g_ref[off:off + n]
            print(f"layer {li} {name}: rel {((h - r).norm() / r.norm().clamp_min(1e-30)).item():.3e}  "
                  f"|ref| {r.norm().item():.3e} |hip| {h.norm().item():.3e}")
            off += n


if __name__ == "__main__":
    main()
