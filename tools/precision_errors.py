"""Print the jet-kernel errors (forward per-stream max / backward gradient norm) of every kernel
precision against the fp64 torch jet, for the shapes of tests/test_hip_kernels.py (GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from test_hip_kernels import CASES, _setup  # noqa: E402

from tensordiffeq_amd.jet import jet_forward  # noqa: E402
from tensordiffeq_amd.ops import jet_hip, jet_mlp  # noqa: E402


def main():
    for sizes, reqs, N in CASES:
        for prec in ("fp32", "bf16x3", "bf16"):
            net, X, plan = _setup(sizes, reqs, N, seed=1)
            try:
                cfg = jet_mlp.hip_config(net, plan, prec)
            except ValueError:
                continue
            G = torch.randn(plan.S, N, sizes[-1], device="cuda", dtype=torch.float64)
            p = net.flat.detach().clone().requires_grad_(True)
            J = jet_hip.JetMLPFunction.apply(X, p, net, plan, prec)
            (J.double() * G).sum().backward()
            p64 = net.flat.detach().double().clone().requires_grad_(True)
            Jr = jet_forward(X.double(), net.weights(p64), plan)
            (Jr * G).sum().backward()
            scale = Jr.detach().abs().amax(dim=(1, 2), keepdim=True).clamp_min(1e-3)
            fe = ((J.detach().double() - Jr.detach()).abs() / scale).amax(dim=(1, 2)).tolist()
            be = ((p.grad.double() - p64.grad).norm() / p64.grad.norm()).item()
            print(f"{str(sizes):32s} S={plan.S} {prec:7s} ({cfg['precision']:6s}) fwd {max(fe):.2e} "
                  f"[{' '.join(f'{e:.1e}' for e in fe)}]  bwd {be:.2e}", flush=True)


if __name__ == "__main__":
    main()
