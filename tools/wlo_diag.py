"""Per-block gradient error of the fused step (bf16 and the weight-lo variant) against the fp64 jet."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import bench
    from tensordiffeq_amd.fit import LossGradEngine
    from tensordiffeq_amd.ops import fused_step
    dev = torch.device("cuda", 0)
    m = bench.build_problem(20000, 1, "hip", dev, False, "bf16")
    prog = m.program()
    ref = bench.build_problem(20000, 1, "jet", dev, False, "bf16")
    p64 = m.u_model.flat.detach().double().requires_grad_(True)
    tot, _ = ref.program().evaluate(p64, [lam.detach().double() for lam in m.lambdas])
    g64, = torch.autograd.grad(tot, [p64])
    net = m.u_model
    for wlo in (False, True):
        fs = fused_step.for_program(prog, wlo=wlo)
        fg = LossGradEngine(m, prog, m.lambdas, weight_lo=wlo).evaluate_fg().double()
        torch.cuda.synchronize()
        g = fg[:-1]
        print(f"wlo={wlo} rows {fs.rows} total rel {((g - g64).norm() / g64.norm()).item():.3e}")
        for i, (wo, bo, fi, fo) in enumerate(net.offsets):
            for name, a, b in (("K", wo, bo), ("b", bo, bo + fo)):
                e = ((g[a:b] - g64[a:b]).norm() / g64[a:b].norm().clamp_min(1e-30)).item()
                print(f"   layer {i} {name} [{a}:{b}] rel {e:.3e}  |g64| {g64[a:b].norm().item():.3e}")


if __name__ == "__main__":
    main()
