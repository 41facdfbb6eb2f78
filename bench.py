#!/usr/bin/env python
"""Flagship benchmark: Allen-Cahn self-adaptive PINN training throughput (BASELINE.json).

Config (reference examples/AC-SA.py:9-64): u_t - 1e-4 u_xx + 5u^3 - 5u = 0 on x in [-1,1],
t in [0,1]; IC u(x,0) = x^2 cos(pi x) on 512 points with self-adaptive weights (init 100 U[0,1]);
periodic BC on u and u_x (201 points per face); tanh MLP [2,128,128,128,128,1] (random Keras
init); N_f = 50,000 collocation points PER GPU (weak scaling: global N_f = 50,000 x n_gpus),
residual SA weights init U[0,1]; Keras Adam lr 0.005, beta1 0.99 on theta, gradient ascent on
the SA weights.  One step = full-batch loss + gradients (HIP jet kernels) + DP all-reduce +
fused Adam/SA update - the complete reference training step, nothing skipped.

Precision (BASELINE.json names AC-SA "bf16"): the jet GEMMs run bf16 x bf16 MFMAs with fp32
accumulation (fp32 master weights rounded once per step); tanh jets, loss, reductions and the
optimizer are fp32.  Under the reference schedule (Adam 10k in this precision + L-BFGS 10k in bf16x3) the L2 on
AC.mat matches all-bf16x3 training over three seeds (profiles/r2_v2_accuracy_mixed.jsonl).
``--precision bf16x3`` measures the split-activation kernels.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--npts 50000] [--backend auto]

Multi-GPU: launched by ``torch.distributed.run`` (one rank per GPU, RCCL); the timed region is
bracketed by barrier + device synchronize on every rank and the max over ranks is reported.
Rank 0 prints ONE JSON line.  The relative L2 error on the reference's ground-truth AC.mat grid
(data/AC.mat) is evaluated after the timed steps (outside the timed region).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = "collocation-pts/sec + L2 rel-error, Allen-Cahn SA-PINN @ 1/2/4/8 GPU"
PRECISION_NOTES = {
    "bf16x3": "bf16x3: split-bf16 MFMA (hi*hi+hi*lo+lo*hi), fp32 accumulate, fp32 elementwise/loss/optimizer",
    "bf16": "bf16: bf16 x bf16 MFMA (weights and activations rounded), fp32 accumulate, "
            "fp32 master weights/elementwise/loss/optimizer",
    "fp32": "fp32 MFMA",
}


def build_problem(n_per_gpu, world, backend, device, dist, precision=None):
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, IC, periodicBC

    tdq.set_seed(1234)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 512)
    D.add("t", [0.0, 1.0], 201)
    n_glob = n_per_gpu * world
    D.generate_collocation_points(n_glob)

    def func_ic(x):
        return x ** 2 * np.cos(math.pi * x)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        return u, u_x

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t - 0.0001 * u_xx + 5.0 * u * u * u - 5.0 * u

    init = IC(D, [func_ic], var=[["x"]])
    x_periodic = periodicBC(D, ["x"], [deriv_model])
    g = torch.Generator().manual_seed(99)
    init_weights = {"residual": [torch.rand(n_glob, 1, generator=g)],
                    "BCs": [100 * torch.rand(512, 1, generator=g), None]}
    model = tdq.CollocationSolverND(verbose=False)
    model.compile([2, 128, 128, 128, 128, 1], f_model, D, [init, x_periodic],
                  Adaptive_type="self-adaptive",
                  dict_adaptive={"residual": [True], "BCs": [True, False]},
                  init_weights=init_weights, backend=backend, device=device, dist=dist,
                  precision=precision)
    return model


def l2_on_ac_grid(model):
    import scipy.io
    data = scipy.io.loadmat(os.path.join(HERE, "data", "AC.mat"))
    x = data["x"].flatten()
    t = data["tt"].flatten()
    X, T = np.meshgrid(x, t)
    X_star = np.hstack((X.flatten()[:, None], T.flatten()[:, None]))
    u_star = np.real(data["uu"]).T.flatten()[:, None]
    u_pred, _ = model.predict(X_star)
    from tensordiffeq_amd.helpers import find_L2_error
    return find_L2_error(u_pred, u_star)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--npts", type=int, default=50000, help="collocation points per GPU")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--no-l2", action="store_true")
    ap.add_argument("--precision", default="bf16", choices=["bf16x3", "bf16", "fp32"],
                    help="GEMM precision of the HIP jet kernels (bf16x3 = split-bf16 MFMA, fp32 accumulate; "
                         "bf16 = bf16 x bf16 MFMA, fp32 accumulate)")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with "
                 f"'python -m torch.distributed.run --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}'")
    dist = world > 1
    from tensordiffeq_amd.parallel import init_distributed, get_context
    ctx = init_distributed() if dist else get_context()
    device = ctx.device if dist else (torch.device("cuda", 0) if torch.cuda.is_available()
                                      else torch.device("cpu"))
    if device.type == "cuda":
        torch.cuda.set_device(device)

    model = build_problem(args.npts, world, args.backend, device, dist, args.precision)
    eng = model._get_engine(None, args.warmup + args.steps + 2)
    backend = model.active_backend

    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    eng.run(max(1, args.warmup))
    sync()
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    eng.run(args.steps)
    sync()
    ctx.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    elapsed = ctx.max_scalar(elapsed)

    loss = float(model._state["hist"][int(model._state["epoch_host"]) - 1, 0])
    n_glob = args.npts * world
    pts_per_s = n_glob * args.steps / elapsed
    l2 = None
    if not args.no_l2 and ctx.rank == 0:
        try:
            l2 = l2_on_ac_grid(model)
        except Exception as e:  # pragma: no cover
            l2 = f"unavailable: {e}"
    if ctx.rank == 0:
        print(json.dumps({
            "metric": METRIC,
            "value": pts_per_s,
            "unit": "collocation-pts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if (backend == "hip" and args.precision != "fp32") else "fp32",
            "data": "synthetic (LHS collocation points, random Keras-init weights); L2 on data/AC.mat",
            "config": {"model": "Allen-Cahn SA-PINN tanh MLP [2,128,128,128,128,1]",
                       "global_batch": n_glob, "seq_len": None, "parallelism": f"dp{world}",
                       "points_per_gpu": args.npts, "backend": backend,
                       "precision": PRECISION_NOTES[args.precision] if backend == "hip" else "fp32",
                       "bc_points": "IC 512 (SA) + periodic 2x201 (u, u_x)",
                       "accuracy_evidence": "profiles/r2_v26_accuracy_final.jsonl"},
            "loss_after": loss,
            "l2_rel_error_after_steps": l2,
            "total_adam_steps": int(model._state["epoch_host"]),
        }), flush=True)
    if dist:
        from tensordiffeq_amd.parallel import destroy
        destroy()


if __name__ == "__main__":
    main()
