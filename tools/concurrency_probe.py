"""Probe: do two point subsets on two graph branches fill the wave-slot quantisation holes?

The bf16 AC-SA step runs 3184 waves of 16 points per jet kernel over 2048 wave slots (1.55
rounds -> 2).  This times the jet forward + backward pair (no loss, a fixed adjoint) captured in
one HIP graph for the whole point set on one stream, against the same points split into subsets
whose forward -> backward chains sit on separate streams (graph branches), so the backward of one
subset can take the slots the other subset's forward leaves idle.  Prints one JSON line per layout.

    python tools/concurrency_probe.py [--n 51316] [--reps 200] [--prec bf16]
"""
import argparse
import json
import time

import torch

from tensordiffeq_amd.jet import JetPlan
from tensordiffeq_amd.models.networks import TanhMLP
from tensordiffeq_amd.ops import jet_hip


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=51316)
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--prec", default="bf16")
    ap.add_argument("--bwd-waves", default=None)
    a = ap.parse_args()
    torch.manual_seed(0)
    dev = torch.device("cuda", 0)
    net = TanhMLP([2, 128, 128, 128, 128, 1], device=dev)
    X = (torch.rand(a.n, 2, device=dev) * 2 - 1).contiguous()
    plan = JetPlan([(0,), (1,), (0, 0)], 2)
    P = net.flat.detach()

    def layout(fracs):
        cuts = [0]
        for f in fracs[:-1]:
            cuts.append(cuts[-1] + (int(round(f * a.n)) // 128) * 128)
        cuts.append(a.n)
        return [(cuts[i], cuts[i + 1]) for i in range(len(fracs))]

    def run(parts, streams):
        # eager warm-up allocates every buffer once; the capture re-allocates from its pool
        Xs = [X[lo:hi].contiguous() for lo, hi in parts]
        dJs = []
        for Xp in Xs:
            J, saved = jet_hip.forward_raw(Xp, P, net, plan, a.prec)
            dJs.append(torch.randn_like(J) * 1e-3)
            jet_hip.backward_raw(saved, dJs[-1], reduce=False)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        main_s = torch.cuda.Stream(device=dev)
        side = [torch.cuda.Stream(device=dev) for _ in parts]
        keep = []
        with torch.cuda.stream(main_s):
            with torch.cuda.graph(g, stream=main_s):
                for i, Xp in enumerate(Xs):
                    s = side[i] if streams else main_s
                    if streams:
                        s.wait_stream(main_s)
                    with torch.cuda.stream(s):
                        J, saved = jet_hip.forward_raw(Xp, P, net, plan, a.prec)
                        keep.append(jet_hip.backward_raw(saved, dJs[i], reduce=False))
                if streams:
                    for s in side:
                        main_s.wait_stream(s)
        torch.cuda.synchronize()
        for _ in range(20):
            g.replay()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(a.reps):
            g.replay()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / a.reps * 1e3

    base = None
    for fracs, streams in [([1.0], False), ([0.5, 0.5], True), ([0.64, 0.36], True), ([0.4, 0.6], True),
                           ([1 / 3, 1 / 3, 1 / 3], True), ([0.5, 0.5], False), ([1.0], False)]:
        ms = run(layout(fracs), streams)
        if base is None:
            base = ms
        print(json.dumps({"parts": [round(f, 3) for f in fracs], "streams": streams, "ms_fwd_bwd": round(ms, 4),
                          "vs_single": round(ms / base, 3), "prec": a.prec, "n": a.n}), flush=True)


if __name__ == "__main__":
    main()
