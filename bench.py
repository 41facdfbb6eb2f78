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

Accuracy half of the metric (after the timed region, ``--acc-seeds``, at every GPU count): the
reference AC-SA schedule (examples/AC-SA.py:64-88: Adam 10k + L-BFGS 10k; Adam in the bench
precision, L-BFGS in ``newton_precision`` bf16x3) from scratch per seed on its 50k points -
sharded over the ranks, with their SA weights, at ``--gpus N`` - relative L2 on data/AC.mat, wall
time per phase and why L-BFGS stopped (``--problem ac-dist``: AC-dist-new's Adam 1001 x 2 on 500k).  ``--force-dp`` (single GPU) also times the data-parallel
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
                  lbfgs_stop=None, layers=(2, 128, 128, 128, 128, 1), problem="ac-sa", newton_schedule=None):
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
                      newton_precision=newton_precision, lbfgs_stop=lbfgs_stop, newton_schedule=newton_schedule)
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
                  precision=precision, newton_precision=newton_precision, lbfgs_stop=lbfgs_stop,
                  newton_schedule=newton_schedule)
    return model


# c1 parametrization of the discovery problem: "linear" (the reference's raw c1 = v from 0, the
# default) or "log" (c1 = exp(v) from v = -6, Raissi et al.'s form for a small positive coefficient:
# NOT the reference program; c1 median 51 % off over seeds 0-4, profiles/r4disc_c1_param_ab.jsonl).
# Why the linear c1 lands 1-10x high: profiles/r5s2_discovery_c1_explained.md.  bench --c1-param.
DISCOVERY_C1 = "linear"


def discovery_c1(v):
    return float(torch.exp(v.detach())) if DISCOVERY_C1 == "log" else float(v.detach())


def build_discovery(n_data, world, backend, device, dist, precision=None, seed=1234, newton_precision=None,
                    lbfgs_stop=None, layers=(2, 128, 128, 128, 128, 1), newton_schedule=None):
    """The reference's AC-discovery program (examples/AC-discovery.py:14-66): learn c1, c2 of
    u_t - c1 u_xx + c2 u^3 - c2 u = 0 (truth 1e-4, 5) from the AC.mat field (102,912 points, or a
    seeded subsample of ``n_data``), self-adaptive collocation weights (col-weight Adam beta_1 0.95)."""
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.models import DiscoveryModel
    from tensordiffeq_amd.optimizers import Adam
    import scipy.io
    tdq.set_seed(seed)
    data = scipy.io.loadmat(os.path.join(HERE, "data", "AC.mat"))
    x, t = data["x"].flatten(), data["tt"].flatten()
    X, T = np.meshgrid(x, t)
    X_star = np.hstack((X.flatten()[:, None], T.flatten()[:, None]))
    u_star = np.real(data["uu"]).T.flatten()[:, None]
    if n_data and n_data < X_star.shape[0]:
        idx = np.random.default_rng(seed).choice(X_star.shape[0], n_data, replace=False)
        X_star, u_star = X_star[idx], u_star[idx]
    log_c1 = DISCOVERY_C1 == "log"
    params = [tdq.Variable(-6.0 if log_c1 else 0.0), tdq.Variable(0.0)]

    def f_model(u_model, var, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        c1 = torch.exp(var[0]) if log_c1 else var[0]
        return u_t - c1 * u_xx + var[1] * u * u * u - var[1] * u

    g = torch.Generator().manual_seed(99 if seed == 1234 else seed)
    col_weights = torch.rand(X_star.shape[0], 1, generator=g)
    m = DiscoveryModel(verbose=False)
    m.compile(list(layers), f_model, [X_star[:, 0:1], X_star[:, 1:2]], u_star, params, col_weights=col_weights,
              backend=backend, device=device, dist=dist, precision=precision, newton_precision=newton_precision,
              lbfgs_stop=lbfgs_stop)
    m.tf_optimizer_weights = Adam(lr=0.005, beta_1=0.95)
    return m


def build_poisson(n_glob, world, backend, device, dist, precision=None, seed=1234, newton_precision=None,
                  lbfgs_stop=None, layers=(2, 50, 50, 50, 50, 1), newton_schedule=None):
    """The reference's 2-D steady-state (Helmholtz-type) program, examples/steady-state.py:10-55:
    u_xx + u_yy + u = q on [-1, 1]^2, exact u = sin(pi x) sin(4 pi y), 4 Dirichlet faces of 1001
    points, [2, 50x4, 1]; BASELINE.json sizes it at 10M collocation points per GPU."""
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, dirichletBC
    tdq.set_seed(seed)
    D = DomainND(["x", "y"])
    D.add("x", [-1.0, 1.0], 1001)
    D.add("y", [-1.0, 1.0], 1001)
    D.generate_collocation_points(n_glob, device=device if device.type == "cuda" else None)

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        u_xx = tdq.grad(tdq.grad(u, x), x)
        u_yy = tdq.grad(tdq.grad(u, y), y)
        s = torch.sin(math.pi * x) * torch.sin(4 * math.pi * y)
        return u_xx + u_yy + u - (-(math.pi ** 2) * s - (4 * math.pi) ** 2 * s + s)

    bcs = [dirichletBC(D, 0.0, v, tg) for v in ("x", "y") for tg in ("upper", "lower")]
    m = tdq.CollocationSolverND(verbose=False)
    m.compile(list(layers), f_model, D, bcs, backend=backend, device=device, dist=dist, precision=precision,
              newton_precision=newton_precision, lbfgs_stop=lbfgs_stop, newton_schedule=newton_schedule)
    return m


# BASELINE.json configs: builder, default points (per GPU for weak scaling, total for strong),
# scaling, default net, model name, BC description, unit of the throughput
PROBLEMS = {
    "ac-sa": dict(build=lambda *a, **k: build_problem(*a, problem="ac-sa", **k), npts=50000, scaling="weak",
                  layers="2,128,128,128,128,1", model="Allen-Cahn SA-PINN tanh MLP",
                  bc="IC 512 (SA) + periodic 2x201 (u, u_x)", unit="collocation-pts/s"),
    "ac-baseline": dict(build=lambda *a, **k: build_problem(*a, problem="ac-baseline", **k), npts=50000,
                        scaling="weak", layers="2,128,128,128,128,1", model="Allen-Cahn baseline PINN tanh MLP",
                        bc="IC 512 + periodic 2x201 (u, u_x, u_xxx, u_xxxx; order 3/4 on jet_hi.hip)",
                        unit="collocation-pts/s"),
    "ac-dist": dict(build=lambda *a, **k: build_problem(*a, problem="ac-baseline", **k), npts=500000,
                    scaling="strong", layers="2,128,128,128,128,1",
                    model="Allen-Cahn distributed (AC-dist-new) tanh MLP",
                    bc="IC 512 + periodic 2x201 (u, u_x, u_xxx, u_xxxx)", unit="collocation-pts/s"),
    "discovery": dict(build=build_discovery, npts=102912, scaling="strong", layers="2,128,128,128,128,1",
                      model="Allen-Cahn discovery (c1, c2) tanh MLP", bc="AC.mat data points (SA col weights)",
                      unit="data-pts/s"),
    "poisson": dict(build=build_poisson, npts=10_000_000, scaling="weak", layers="2,50,50,50,50,1",
                    model="2-D steady-state Helmholtz/Poisson tanh MLP", bc="4 Dirichlet faces x 1001",
                    unit="collocation-pts/s"),
}


def get_engine(model, n_hint):
    """The model's captured Adam engine (solver and discovery models name it differently)."""
    from tensordiffeq_amd.models.discovery import DiscoveryModel
    if isinstance(model, DiscoveryModel):
        return model._get_engine(n_hint)
    return model._get_engine(None, n_hint)


def backend_of(model):
    return model.program().backend


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


def accuracy_runs(seeds, device, backend, precision, newton_precision, iters, newton, lbfgs_stop, problem="ac-sa",
                  layers=None, newton_schedule=None, world=1, npts=None, newton_eager=True):
    """Reference schedule per seed (AC-SA / AC-baseline: examples/AC-SA.py:9-88, Adam + L-BFGS, L2 on
    AC.mat; AC-dist: examples/AC-dist-new.py:48-78, 500k points, ``fit(tf_iter=1001)`` twice, L2 on
    AC.mat; discovery: examples/AC-discovery.py, Adam + L-BFGS over network and coefficients,
    c1 / c2 errors), with phase times and the L-BFGS stop reason.  ``world > 1``: every rank runs
    it under data parallelism - the schedule's point set (50k, or AC-dist's 500k) sharded over the
    ranks with its SA weights, one all-reduce per step - as the reference's distributed example
    trains with ``dist=True`` before evaluating (AC-dist-new.py:51-54,78).  ``newton_eager=False``:
    the L-BFGS phase is the line-search L-BFGS (the reference's graph mode, fit.py:83-89)."""
    out = []
    spec = PROBLEMS[problem]
    layers = layers or tuple(int(v) for v in spec["layers"].split(","))
    dist = world > 1
    for sd in seeds:
        n = npts or (spec["npts"] if problem in ("discovery", "ac-dist") else 50000)
        m = spec["build"](n, world, backend, device, dist, precision, seed=sd, newton_precision=newton_precision,
                          lbfgs_stop=lbfgs_stop, layers=layers, newton_schedule=newton_schedule)
        if problem == "discovery":
            m.fit(tf_iter=iters, newton_iter=newton)
            c1, c2 = discovery_c1(m.vars[0]), float(m.vars[1].detach())
            res = {"seed": sd, "c1": c1, "c2": c2, "c1_rel_err": abs(c1 - 1e-4) / 1e-4, "c2_rel_err": abs(c2 - 5.0) / 5.0}
        elif problem == "ac-dist":
            m.fit(tf_iter=AC_DIST_ADAM)
            a1 = m.fit_info.get("adam", {}).get("wall_s", 0.0)
            m.fit(tf_iter=AC_DIST_ADAM)
            m.fit_info.setdefault("adam", {})["wall_s"] = a1 + m.fit_info.get("adam", {}).get("wall_s", 0.0)
            res = {"seed": sd, "l2": float(l2_on_ac_grid(m))}
        else:
            m.fit(tf_iter=iters)
            m.fit(newton_iter=newton, newton_eager=newton_eager)
            res = {"seed": sd, "l2": float(l2_on_ac_grid(m))}
        info = m.fit_info
        lb = info.get("lbfgs", {})
        if lb.get("phases"):
            res["lbfgs_phases"] = lb["phases"]
        res.update({"adam_s": round(info.get("adam", {}).get("wall_s", 0.0), 3),
                    "lbfgs_s": round(lb.get("wall_s", 0.0), 3),
                    "lbfgs_n_iter": lb.get("n_iter"), "lbfgs_reason": lb.get("reason"),
                    "lbfgs_stop": lb.get("stop"), "lbfgs_impl": lb.get("impl"),
                    "lbfgs_func_evals": lb.get("func_evals")})
        out.append(res)
        del m
        if device.type == "cuda":
            torch.cuda.empty_cache()
    return out


AC_DIST_ADAM = 1001  # examples/AC-dist-new.py:52-54: fit(tf_iter=1001) twice


def forced_dp_timing(n_glob, backend, device, precision, steps, warmup, min_warmup_s):
    """The DP step on one GPU: RCCL process group at world 1 (TDQ_FORCE_DP semantics), bucket
    all-reduce captured in the step graph.  Returns (ms/step, loss-history max |diff| vs the plain
    run is checked by tests/test_dist_gpu.py, not here)."""
    from tensordiffeq_amd.parallel import dist as pdist
    ctx = pdist.init_distributed(device=device, force=True)
    try:
        m = build_problem(n_glob, 1, backend, device, True, precision)
        eng = get_engine(m, warmup + steps + 2)
        el, _, _ = time_steps(eng, ctx, device, steps, warmup, min_warmup_s)
        return {"ms_per_step": 1000.0 * el / steps, "backend": ctx.backend,
                "collective_in_graph": bool(ctx.graph_collectives)}
    finally:
        pdist.destroy()


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--problem", default="ac-sa", choices=sorted(PROBLEMS),
                    help="ac-sa: the BASELINE.json flagship (examples/AC-SA.py, 50k pts/GPU); ac-baseline: the "
                         "reference's AC-baseline program (no SA weights, periodic u, u_x, u_xxx, u_xxxx; 50k/GPU); "
                         "ac-dist: AC-dist-new (the same program, 500k points in total, strong scaling); "
                         "discovery: AC-discovery (102,912 AC.mat points in total, c1/c2 errors); "
                         "poisson: 2-D steady state at 10M points per GPU")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--min-warmup-s", type=float, default=1.0,
                    help="keep warming up (untimed) until this much time has passed")
    ap.add_argument("--npts", type=int, default=None,
                    help="collocation points per GPU (weak scaling; default: the problem's)")
    ap.add_argument("--global-npts", type=int, default=None,
                    help="total collocation points, split over the GPUs (strong scaling; default for "
                         "ac-dist / discovery)")
    ap.add_argument("--backend", default="auto")
    ap.add_argument("--layers", default=None,
                    help="network layer sizes (default: the problem's reference net; widths 129-256 run "
                         "the fused kernels in bf16, wider nets / other precisions the layer-wise engine)")
    ap.add_argument("--no-l2", action="store_true", help="skip the accuracy runs")
    ap.add_argument("--acc-seeds", type=int, nargs="*", default=[0, 1, 2],
                    help="seeds of the full-schedule accuracy runs (under data parallelism at --gpus N)")
    ap.add_argument("--acc-iters", type=int, default=10000)
    ap.add_argument("--acc-npts", type=int, default=None,
                    help="points of the accuracy runs (default: the reference schedule's, 50k / AC-dist 500k)")
    ap.add_argument("--acc-newton", type=int, default=None,
                    help="L-BFGS iterations of the accuracy runs (default 10000; discovery 15000)")
    ap.add_argument("--newton-precision", default="bf16x3")
    ap.add_argument("--newton-schedule", default=None,
                    help="leading L-BFGS phases of the accuracy runs, 'prec:iters,...' (e.g. bf16:7000)")
    ap.add_argument("--newton-eager", type=int, default=1, choices=[0, 1],
                    help="0: the accuracy runs' L-BFGS is the line-search L-BFGS (reference graph mode)")
    ap.add_argument("--lbfgs-stop", default=None, choices=["fixed", "legacy"],
                    help="L-BFGS function-change test (default: the library's, legacy = the reference's)")
    ap.add_argument("--force-dp", action="store_true",
                    help="also time the DP step at world 1 (RCCL process group, single GPU only)")
    ap.add_argument("--precision", default="bf16", choices=["bf16x3", "bf16", "fp32"],
                    help="GEMM precision of the HIP jet kernels (bf16x3 = split-bf16 MFMA, fp32 accumulate; "
                         "bf16 = bf16 x bf16 MFMA, fp32 accumulate)")
    ap.add_argument("--c1-param", default="linear", choices=["log", "linear"],
                    help="discovery: the reference's raw c1 = v from 0 (default) or c1 = exp(v) from v = -6 "
                         "(not the reference's parametrization)")
    args = ap.parse_args(argv)
    global DISCOVERY_C1
    DISCOVERY_C1 = args.c1_param

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

    spec = PROBLEMS[args.problem]
    strong = args.global_npts is not None or (args.npts is None and spec["scaling"] == "strong")
    if strong:
        n_glob = args.global_npts if args.global_npts is not None else spec["npts"]
    else:
        n_glob = (args.npts if args.npts is not None else spec["npts"]) * world
    if args.acc_newton is None:
        args.acc_newton = 15000 if args.problem == "discovery" else 10000  # discovery: c2 to 0.03 % (r4o)
    # accuracy runs: the reference schedules of the single-GPU configs (AC-dist-new runs Adam 1001
    # twice without L-BFGS and the 10M-point Poisson config is a throughput sizing)
    acc_ok = args.problem in ("ac-sa", "ac-baseline", "ac-dist", "discovery")
    if "TDQ_STEP_UNROLL" not in os.environ:
        # steps per captured graph: a divisor of --steps, so the timed steps are all multi-step graph
        # replays (a 1-step replay leaves ~9 us idle between graphs; 8 and 16 per graph measured
        # equal, profiles/r3_m_unroll_ab.jsonl; at --steps 20 one 20-step graph measured slower than
        # two 10-step replays, 0.206-0.211 vs 0.202-0.203 ms, profiles/r3_au_driver_shape_unroll_ab.jsonl)
        divs = [k for k in range(16, 3, -1) if args.steps % k == 0]
        os.environ["TDQ_STEP_UNROLL"] = str(8 if args.steps % 8 == 0 else (divs[0] if divs else 8))
    layers = tuple(int(v) for v in (args.layers or spec["layers"]).split(","))
    model = spec["build"](n_glob, world, args.backend, device, dist, args.precision, layers=layers,
                          newton_precision=args.newton_precision)
    eng = get_engine(model, args.warmup + args.steps + 2)
    backend = backend_of(model)
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
    if not args.no_l2 and args.acc_seeds and acc_ok:
        try:
            acc = accuracy_runs(args.acc_seeds, device, args.backend, args.precision, args.newton_precision,
                                args.acc_iters, args.acc_newton, args.lbfgs_stop, problem=args.problem,
                                layers=layers, newton_schedule=args.newton_schedule, world=world,
                                npts=args.acc_npts, newton_eager=bool(args.newton_eager))
        except Exception as e:  # pragma: no cover - reported, never hides the throughput number
            acc_err = f"{type(e).__name__}: {e}"
    dp = None
    if args.force_dp and world == 1 and device.type == "cuda" and args.problem == "ac-sa":
        try:
            dp = forced_dp_timing(n_glob, args.backend, device, args.precision, args.steps, args.warmup,
                                  args.min_warmup_s)
        except Exception as e:  # pragma: no cover
            dp = {"error": f"{type(e).__name__}: {e}"}

    if ctx.rank == 0:
        rec = {
            "metric": METRIC,
            "value": pts_per_s,
            "unit": spec["unit"],
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1000.0 * elapsed / args.steps,
            "higher_is_better": True,
            "scaling": "strong" if strong else "weak",
            "vs_baseline": None,
            "dtype": "bf16" if (backend == "hip" and args.precision != "fp32") else "fp32",
            "data": ("AC.mat observations (102,912-point field), random Keras-init weights" if args.problem == "discovery"
                     else "synthetic (LHS collocation points, random Keras-init weights)"
                     + ("; L2 on data/AC.mat" if args.problem.startswith("ac") else "")),
            "config": {"model": f"{spec['model']} [{','.join(map(str, layers))}]",
                       "problem": args.problem,
                       "global_batch": n_glob, "seq_len": None, "parallelism": f"dp{world}",
                       "points_per_gpu": n_glob // world, "backend": backend,
                       "precision": PRECISION_NOTES[args.precision] if backend == "hip" else "fp32",
                       "bc_points": spec["bc"]},
            "warmup_steps_run": n_warm,
            "warmup_s": round(warm_s, 3),
            "loss_after": loss,
            "total_adam_steps": total_steps,
        }
        if acc is not None and args.problem == "discovery":
            rec["coefficients"] = [{k: a[k] for k in ("seed", "c1", "c2", "c1_rel_err", "c2_rel_err")} for a in acc]
            rec["c1_parametrization"] = ("reference: c1 = v from 0" if args.c1_param == "linear"
                                         else "NON-reference: c1 = exp(v) from v = -6")
            rec["accuracy_schedule"] = (f"Adam {args.acc_iters} ({args.precision}) + L-BFGS {args.acc_newton} "
                                        f"({args.newton_precision}) over network + c1, c2 (c1 parametrization "
                                        f"{args.c1_param}); reference "
                                        f"examples/AC-discovery.py (Adam 10k); seeds {args.acc_seeds}")
            rec["time_to_solution_s"] = [{"adam_s": a["adam_s"], "lbfgs_s": a["lbfgs_s"]} for a in acc]
            rec["lbfgs"] = [{"reason": a["lbfgs_reason"], "n_iter": a["lbfgs_n_iter"]} for a in acc]
        elif acc is not None:
            l2s = sorted(a["l2"] for a in acc)
            rec["l2_full_schedule"] = l2s[len(l2s) // 2]
            rec["l2_full_schedule_seeds"] = [a["l2"] for a in acc]
            on = f"on {world} GPUs (data parallel, points and SA weights sharded)" if world > 1 else "on 1 GPU"
            if args.problem == "ac-dist":
                rec["accuracy_schedule"] = (f"Adam {AC_DIST_ADAM} x 2 ({args.precision}), N_f {args.acc_npts or spec['npts']}, "
                                            f"reference examples/AC-dist-new.py, {on}; median over seeds "
                                            f"{args.acc_seeds}")
            else:
                ref = "AC-SA" if args.problem == "ac-sa" else "AC-baseline"
                rec["accuracy_schedule"] = (f"Adam {args.acc_iters} ({args.precision}) + L-BFGS {args.acc_newton} "
                                            f"({args.newton_precision}), N_f {args.acc_npts or 50000}, reference "
                                            f"examples/{ref}.py, "
                                            f"{on}; median over seeds {args.acc_seeds}")
            rec["time_to_solution_s"] = [{"adam_s": a["adam_s"], "lbfgs_s": a["lbfgs_s"]} for a in acc]
            rec["lbfgs"] = [{"reason": a["lbfgs_reason"], "n_iter": a["lbfgs_n_iter"], "stop": a["lbfgs_stop"],
                             "impl": a.get("lbfgs_impl"), "func_evals": a.get("lbfgs_func_evals"),
                             **({"phases": a["lbfgs_phases"]} if a.get("lbfgs_phases") else {})} for a in acc]
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
