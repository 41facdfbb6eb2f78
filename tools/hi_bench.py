"""Isolated timing of the high-order jet kernels (csrc/jet_hi.hip) on the AC-baseline periodic-BC set:
402 points, order-4 univariate chain, [2, 128 x 4, 1].  Each op is captured 20x in a HIP graph and
replayed, so the numbers are GPU time without host launch overhead.  Run under
``rocprofv3 --kernel-trace --stats`` for the per-kernel split."""
import argparse
import json

import torch

from tensordiffeq_amd.jet import JetPlan
from tensordiffeq_amd.models.networks import TanhMLP
from tensordiffeq_amd.ops import jet_hi


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=402)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--replays", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    sizes = [2, 128, 128, 128, 128, 1]
    net = TanhMLP(sizes, device=dev)
    plan = JetPlan([(0, 0, 0, 0)], 2)
    X = (2 * torch.rand(a.n, 2, device=dev) - 1).contiguous()
    rows = {m: i for i, m in enumerate(plan.streams)}
    op = jet_hi.HiJetOp(net, plan, rows, X, a.n, dev)
    J = torch.zeros(plan.S, a.n, 1, device=dev)
    dJ = torch.randn(plan.S, a.n, 1, device=dev)
    out = {}
    for name, fn in (("fwd", lambda: op.forward(J, net.flat)), ("bwd", lambda: op.backward(dJ, net.flat))):
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            with torch.cuda.graph(g, stream=s):
                for _ in range(a.reps):
                    fn()
        torch.cuda.synchronize()
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.replays):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        out[name + "_us"] = round(e0.elapsed_time(e1) * 1e3 / (a.reps * a.replays), 2)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
