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
optimizer are fp32.  ``--precision bf16x3`` measures the split-activation kernels.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--npts 50000 | --global-npts G]

Timing: W untimed warm-up steps, then more untimed steps until at least ``--min-warmup-s`` of
warm-up has elapsed (a fresh box starts at low clocks: 20 timed steps are only ~5 ms), then
EXACTLY K steps bracketed by barrier + device synchronize on every rank; the max over ranks is
reported.  Weak scaling by default (``--npts`` per GPU); ``--global-npts`` fixes the total
(strong scaling, e.g. the reference's AC-dist-new config: 500,000 points, examples/AC-dist-new.py).

Accuracy half of the metric (single GPU, after the timed region, ``--acc-seeds``): the reference
AC-SA schedule (examples/AC-SA.py:64-88: Adam 10k + L-BFGS 10k; Adam in the bench precision,
L-BFGS in ``newton_precision`` bf16x3) from scratch per seed, relative L2 on data/AC.mat, wall
time per phase and why L-BFGS stopped.  ``--force-dp`` (single GPU) also times the data-parallel
step - a real RCCL process group at world 1, the all-reduce captured in the step graph - next to
the plain one.

Multi-GPU: launched by ``torch.distributed.run`` (one rank per GPU, RCCL).  Rank 0 prints ONE
JSON line.
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


def build_problem(n_glob, world, backend, device, dist, precision=None, seed=1234, newton_precision=None,
                  lbfgs_stop=None, layers=(2, 128, 128, 128, 128, 1), problem="ac-sa"):
    """The AC-SA problem of BASELINE.json with ``n_glob`` collocation points in total (sharded over
    ``world`` ranks when ``dist``).  ``problem="ac-baseline"``: the reference's AC-baseline /
    AC-dist-new program instead (examples/AC-baseline.py:14-52, AC-dist-new.py:14-48): no
    self-adaptive weights, periodic BC on u, u_x, u_xxx and u_xxxx."""
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, IC, periodicBC

    tdq.set_seed(seed)
    D = DomainND(["x", "t"], time_var="t")
    D.add("x", [-1.0, 1.0], 512)
    D.add("t", [0.0, 1.0], 201)
    D.generate_collocation_points(n_glob)

    def func_ic(x):
        return x ** 2 * np.cos(math.pi * x)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        return u, u_x

    def deriv_model4(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_xxx = tdq.grad(u_xx, x)
        u_xxxx = tdq.grad(u_xxx, x)
        return u, u_x, u_xxx, u_xxxx

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t - 0.0001 * u_xx + 5.0 * u * u * u - 5.0 * u

    init = IC(D, [func_ic], var=[["x"]])
    if problem == "ac-baseline":
        model = tdq.CollocationSolverND(verbose=False)
        model.compile(list(layers), f_model, D, [init, periodicBC(D, ["x"], [deriv_model4])],
                      backend=backend, device=device, dist=dist, precision=precision,
                      newton_precision=newton_precision, lbfgs_stop=lbfgs_stop)
        return model
    x_periodic = periodicBC(D, ["x"], [deriv_model])
    g = torch.Generator().manual_seed(99 if seed == 1234 else seed)
    init_weights = {"residual": [torch.rand(n_glob, 1, generator=g)],
                    "BCs": [100 * torch.rand(512, 1, generator=g), None]}
    model = tdq.CollocationSolverND(verbose=False)
    model.compile(list(layers), f_model, D, [init, x_periodic],
                  Adaptive_type="self-adaptive",
                  dict_adaptive={"residual": [True], "BCs": [True, False]},
                  init_weights=init_weights, backend=backend, device=device, dist=dist,
                  precision=precision, newton_precision=newton_precision, lbfgs_stop=lbfgs_stop)
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


def time_steps(eng, ctx, device, steps, warmup, min_warmup_s):
    """Warm up (>= ``warmup`` steps and >= ``min_warmup_s`` seconds), then time exactly ``steps``
    steps between barrier + synchronize pairs; returns (seconds, warm-up steps run, warm-up s)."""
    def sync():
        if device.type == "cuda":
            torch.cuda.synchronize(device)

    t_w = time.perf_counter()
    eng.run(max(1, warmup))
    n_warm = max(1, warmup)
    sync()
    # the stop decision is collective (max over ranks): a rank-local clock would let ranks run
    # different numbers of warm-up steps, i.e. different numbers of all-reduces, and the DP step of
    # the rank with the extra steps would wait for peers that never arrive
    while ctx.max_scalar(time.perf_counter() - t_w) < min_warmup_s:
        eng.run(max(10, warmup))
        n_warm += max(10, warmup)
        sync()
    # room in the device loss history for the timed steps: a re-allocation would re-capture the
    # step graphs inside the timed region; K + 1 more (untimed) steps capture / replay the final
    # 1-step and K-step graphs (fit.AdamEngine._unroll)
    K = eng._unroll()
    eng._ensure_hist(steps + K + 3)
    eng.run(K + 1)
    n_warm += K + 1
    sync()
    warm_s = time.perf_counter() - t_w
    ctx.barrier()
    sync()
    t0 = time.perf_counter()
    eng.run(steps)
    sync()
    local = time.perf_counter() - t0    # this rank's own steps, before waiting for the others
    ctx.barrier()
    sync()
    el = time.perf_counter() - t0
    time_steps.rank_ms = (1000.0 * ctx.min_scalar(local) / steps, 1000.0 * ctx.max_scalar(local) / steps)
    return ctx.max_scalar(el), n_warm, warm_s


def allreduce_replay_us(ctx, n_floats, calls=10, reps=20):
    """Per-call time of the DP step's collective on a bucket-sized buffer, measured the way the
    step runs it: ``calls`` all-reduces captured in one HIP graph (RCCL / peer kernel in the
    graph) and replayed ``reps`` times, or launched from the host when the backend keeps the
    collective out of the graph (gloo).  Max over ranks, microseconds."""
    dev = ctx.device
    buf = torch.randn(int(n_floats), device=dev)
    sync = (lambda: torch.cuda.synchronize(dev)) if dev.type == "cuda" else (lambda: None)
    if ctx.graph_collectives:
        from tensordiffeq_amd.graphs import capture_graph
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            ctx.all_reduce_(buf)
        torch.cuda.current_stream(dev).wait_stream(s)
        sync()
        g = torch.cuda.CUDAGraph()
        with capture_graph(g):
            for _ in range(calls):
                ctx.all_reduce_(buf)
        g.replay()
        sync()
        ctx.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        sync()
        us = (time.perf_counter() - t0) / (reps * calls) * 1e6
        mode = "in-graph"
    else:
        for _ in range(3):
            ctx.all_reduce_(buf)
        sync()
        ctx.barrier()
        t0 = time.perf_counter()
        for _ in range(reps):
            ctx.all_reduce_(buf)
        sync()
        us = (time.perf_counter() - t0) / reps * 1e6
        mode = "host-launched"
    return {"us_per_call": round(ctx.max_scalar(us), 2), "floats": int(n_floats), "mode": mode}


def accuracy_runs(seeds, device, backend, precision, newton_precision, iters, newton, lbfgs_stop, problem="ac-sa"):
    """Reference AC-SA schedule per seed (examples/AC-SA.py:9-88): L2 on AC.mat, phase times,
    L-BFGS stop reason."""
    out = []
    for sd in seeds:
        m = build_problem(50000, 1, backend, device, False, precision, seed=sd,
                          newton_precision=newton_precision, lbfgs_stop=lbfgs_stop, problem=problem)
        m.fit(tf_iter=iters)
        m.fit(newton_iter=newton)
        info = m.fit_info
        lb = info.get("lbfgs", {})
        out.append({"seed": sd, "l2": float(l2_on_ac_grid(m)),
                    "adam_s": round(info.get("adam", {}).get("wall_s", 0.0), 3),
                    "lbfgs_s": round(lb.get("wall_s", 0.0), 3),
                    "lbfgs_n_iter": lb.get("n_iter"), "lbfgs_reason": lb.get("reason"),
                    "lbfgs_stop": lb.get("stop")})
        del m
        if device.type == "cuda":
            torch.cuda.empty_cache()
    return out


def forced_dp_timing(n_glob, backend, device, precision, steps, warmup, min_warmup_s):
    """The DP step on one GPU: RCCL process group at world 1 (TDQ_FORCE_DP semantics), bucket
    all-reduce captured in the step graph.  Returns (ms/step, loss-history max |diff| vs the plain
    run is checked by tests/test_dist_gpu.py, not here)."""
    from tensordiffeq_amd.parallel import dist as pdist
    ctx = pdist.init_distributed(device=device, force=True)
    try:
        m = build_problem(n_glob, 1, backend, device, True, precision)
        eng = m._get_engine(None, warmup + steps + 2)
        el, _, _ = time_steps(eng, ctx, device, steps, warmup, min_warmup_s)
        return {"ms_per_step": 1000.0 * el / steps, "backend": ctx.backend,
                "collective_in_graph": bool(ctx.graph_collectives)}
    finally:
        pdist.destroy()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--problem", default="ac-sa", choices=["ac-sa", "ac-baseline"],
                    help="ac-sa: the BASELINE.json flagship (examples/AC-SA.py); ac-baseline: the reference's "
                         "AC-baseline / AC-dist-new program (no SA weights, periodic u, u_x, u_xxx, u_xxxx)")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--min-warmup-s", type=float, default=1.0,
                    help="keep warming up (untimed) until this much time has passed")
    ap.add_argument("--npts", type=int, default=50000, help="collocation points per GPU (weak scaling)")
    ap.add_argument("--global-npts", type=int, default=None,
                    help="total collocation points, split over the GPUs (strong scaling)")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--layers", default="2,128,128,128,128,1",
                    help="network layer sizes (default: the AC-SA net of BASELINE.json; widths > 128 run the "
                         "layer-wise engine)")
    ap.add_argument("--no-l2", action="store_true", help="skip the accuracy runs")
    ap.add_argument("--acc-seeds", type=int, nargs="*", default=[0, 1, 2],
                    help="seeds of the full-schedule accuracy runs (single GPU only)")
    ap.add_argument("--acc-iters", type=int, default=10000)
    ap.add_argument("--acc-newton", type=int, default=10000)
    ap.add_argument("--newton-precision", default="bf16x3")
    ap.add_argument("--lbfgs-stop", default=None, choices=["fixed", "legacy"],
                    help="L-BFGS function-change test (default: the library's, legacy = the reference's)")
    ap.add_argument("--force-dp", action="store_true",
                    help="also time the DP step at world 1 (RCCL process group, single GPU only)")
    ap.add_argument("--precision", default="bf16", choices=["bf16x3", "bf16", "fp32"],
                    help="GEMM precision of the HIP jet kernels (bf16x3 = split-bf16 MFMA, fp32 accumulate; "
                         "bf16 = bf16 x bf16 MFMA, fp32 accumulate)")
    args = ap.parse_args(argv)

    from tensordiffeq_amd.parallel import dist as pdist
    if args.gpus > 1 and not pdist.launcher_env():
        # one command for N GPUs: re-run this script as N ranks (child processes under
        # torch.distributed.run, 127.0.0.1); rank 0's JSON line goes straight to our stdout
        sys.exit(pdist.self_launch(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if args.gpus != world:
        ap.error(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    dist = world > 1
    from tensordiffeq_amd.parallel import init_distributed, get_context
    ctx = init_distributed() if dist else get_context()
    device = ctx.device if dist else (torch.device("cuda", 0) if torch.cuda.is_available()
                                      else torch.device("cpu"))
    if device.type == "cuda":
        torch.cuda.set_device(device)

    strong = args.global_npts is not None
    n_glob = args.global_npts if strong else args.npts * world
    if "TDQ_STEP_UNROLL" not in os.environ:
        # steps per captured graph: a divisor of --steps, so the timed steps are all multi-step graph
        # replays (a 1-step replay leaves ~9 us idle between graphs; 8 and 16 per graph measured
        # equal, profiles/r3_m_unroll_ab.jsonl; at --steps 20 one 20-step graph measured slower than
        # two 10-step replays, 0.206-0.211 vs 0.202-0.203 ms, profiles/r3_au_driver_shape_unroll_ab.jsonl)
        divs = [k for k in range(16, 3, -1) if args.steps % k == 0]
        os.environ["TDQ_STEP_UNROLL"] = str(8 if args.steps % 8 == 0 else (divs[0] if divs else 8))
    layers = tuple(int(v) for v in args.layers.split(","))
    model = build_problem(n_glob, world, args.backend, device, dist, args.precision, layers=layers,
                          problem=args.problem)
    eng = model._get_engine(None, args.warmup + args.steps + 2)
    backend = model.active_backend
    elapsed, n_warm, warm_s = time_steps(eng, ctx, device, args.steps, args.warmup, args.min_warmup_s)
    steps_per_graph = eng._unroll()
    loss = float(model._state["hist"][int(model._state["epoch_host"]) - 1, 0])
    total_steps = int(model._state["epoch_host"])
    pts_per_s = n_glob * args.steps / elapsed
    rank_ms = getattr(time_steps, "rank_ms", None)
    ar = None
    if dist:
        bucket = getattr(eng, "_dp_buf", None)
        n_bucket = bucket.numel() if bucket is not None else model.u_model.flat.numel() + 8
        try:
            ar = allreduce_replay_us(ctx, n_bucket)
        except Exception as e:  # pragma: no cover - reported, never hides the throughput number
            ar = {"error": f"{type(e).__name__}: {e}"}
    del eng, model

    acc, acc_err = None, None
    if not args.no_l2 and world == 1 and args.acc_seeds:
        try:
            acc = accuracy_runs(args.acc_seeds, device, args.backend, args.precision, args.newton_precision,
                                args.acc_iters, args.acc_newton, args.lbfgs_stop, problem=args.problem)
        except Exception as e:  # pragma: no cover - reported, never hides the throughput number
            acc_err = f"{type(e).__name__}: {e}"
    dp = None
    if args.force_dp and world == 1 and device.type == "cuda":
        try:
            dp = forced_dp_timing(n_glob, args.backend, device, args.precision, args.steps, args.warmup,
                                  args.min_warmup_s)
        except Exception as e:  # pragma: no cover
            dp = {"error": f"{type(e).__name__}: {e}"}

    if ctx.rank == 0:
        rec = {
            "metric": METRIC,
            "value": pts_per_s,
            "unit": "collocation-pts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "bf16" if (backend == "hip" and args.precision != "fp32") else "fp32",
            "data": "synthetic (LHS collocation points, random Keras-init weights); L2 on data/AC.mat",
            "config": {"model": (f"Allen-Cahn SA-PINN tanh MLP [{','.join(map(str, layers))}]" if args.problem == "ac-sa"
                                 else f"Allen-Cahn baseline PINN tanh MLP [{','.join(map(str, layers))}]"),
                       "problem": args.problem,
                       "global_batch": n_glob, "seq_len": None, "parallelism": f"dp{world}",
                       "points_per_gpu": n_glob // world, "backend": backend,
                       "precision": PRECISION_NOTES[args.precision] if backend == "hip" else "fp32",
                       "bc_points": ("IC 512 (SA) + periodic 2x201 (u, u_x)" if args.problem == "ac-sa" else
                                     "IC 512 + periodic 2x201 (u, u_x, u_xxx, u_xxxx; order 3/4 on jet_hi.hip)")},
            "warmup_steps_run": n_warm,
            "warmup_s": round(warm_s, 3),
            "loss_after": loss,
            "total_adam_steps": total_steps,
        }
        if acc is not None:
            l2s = sorted(a["l2"] for a in acc)
            rec["l2_full_schedule"] = l2s[len(l2s) // 2]
            rec["l2_full_schedule_seeds"] = [a["l2"] for a in acc]
            rec["accuracy_schedule"] = (f"Adam {args.acc_iters} ({args.precision}) + L-BFGS {args.acc_newton} "
                                        f"({args.newton_precision}), N_f 50000, reference examples/AC-SA.py; "
                                        f"median over seeds {args.acc_seeds}")
            rec["time_to_solution_s"] = [{"adam_s": a["adam_s"], "lbfgs_s": a["lbfgs_s"]} for a in acc]
            rec["lbfgs"] = [{"reason": a["lbfgs_reason"], "n_iter": a["lbfgs_n_iter"], "stop": a["lbfgs_stop"]}
                            for a in acc]
        elif acc_err is not None:
            rec["l2_full_schedule"] = None
            rec["accuracy_error"] = acc_err
        rec["steps_per_graph"] = steps_per_graph
        if dist:
            # which all-reduce the DP step captured: RCCL, or the one-shot peer kernel (csrc/peer.hip)
            # when its start-up self-test passed and it timed faster on this node
            rec["allreduce"] = dict(ctx.allreduce_info)
            rec["allreduce"]["replay"] = ar
            rec["rank_ms_per_step"] = {"min": round(rank_ms[0], 5), "max": round(rank_ms[1], 5)} if rank_ms else None
        if dp is not None:
            rec["forced_dp"] = dp
        print(json.dumps(rec), flush=True)
    if dist:
        from tensordiffeq_amd.parallel import destroy
        destroy()


if __name__ == "__main__":
    main()
