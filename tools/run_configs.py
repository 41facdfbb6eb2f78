"""Measure the BASELINE.json configurations on one GPU: accuracy with the reference schedules and
throughput at large per-GPU point counts.  One JSON line per configuration.

  python tools/run_configs.py --which burgers helmholtz discovery poisson10m
"""
import argparse
import importlib.util
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "examples"))


def _example(name):
    spec = importlib.util.spec_from_file_location(name.replace("-", "_"), os.path.join(ROOT, "examples", name + ".py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def timed(fn, *a):
    t0 = time.perf_counter()
    r = fn(*a)
    return r, time.perf_counter() - t0


def poisson_throughput(n_per_gpu, steps, warmup, precision):
    """2-D Helmholtz/Poisson-type residual (u_xx + u_yy + u - q) on a [2, 50x4, 1] net with n_per_gpu
    collocation points resident on the GPU: Adam step throughput (BASELINE config 5 sizing)."""
    import numpy as np
    import torch
    import tensordiffeq_amd as tdq
    from tensordiffeq_amd.boundaries import DomainND, dirichletBC
    tdq.set_seed(0)
    D = DomainND(["x", "y"])
    D.add("x", [-1.0, 1.0], 1001)
    D.add("y", [-1.0, 1.0], 1001)
    D.generate_collocation_points(n_per_gpu, device="cuda")

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        u_xx = tdq.grad(tdq.grad(u, x), x)
        u_yy = tdq.grad(tdq.grad(u, y), y)
        s = torch.sin(math.pi * x) * torch.sin(4 * math.pi * y)
        return u_xx + u_yy + u - (-(math.pi ** 2) * s - (4 * math.pi) ** 2 * s + s)

    bcs = [dirichletBC(D, 0.0, v, tg) for v in ("x", "y") for tg in ("upper", "lower")]
    m = tdq.CollocationSolverND(verbose=False)
    m.compile([2, 50, 50, 50, 50, 1], f_model, D, bcs, backend="hip", device="cuda", precision=precision)
    eng = m._get_engine(None, steps + warmup + 2)
    eng.run(warmup)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    eng.run(steps)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"config": "poisson-2d [2,50x4,1]", "n_points": n_per_gpu, "steps": steps, "ms_per_step": 1e3 * dt / steps,
            "pts_per_s": n_per_gpu * steps / dt, "loss": float(m.losses[-1]["Total Loss"]),
            "peak_mem_gb": torch.cuda.max_memory_allocated() / 2 ** 30, "precision": precision}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--which", nargs="+", default=["burgers", "helmholtz", "discovery", "poisson10m"])
    ap.add_argument("--precision", default="bf16x3")
    ap.add_argument("--scale", type=float, default=1.0, help="multiply iteration counts (smoke runs)")
    a = ap.parse_args()
    k = lambda n: str(max(1, int(n * a.scale)))
    prec, _, newton_prec = a.precision.partition("+")  # "adam+lbfgs", e.g. bf16+bf16x3
    pk = ["--precision", prec] + (["--newton-precision", newton_prec] if newton_prec else [])
    for w in a.which:
        if w == "burgers":
            r, dt = timed(_example("burgers-new").main, ["--iters", k(10000), "--newton", k(10000), "--quiet"] + pk)
            r.update(config="burgers [2,20x8,1] N_f 10k, adam 10k + lbfgs 10k", wall_s=dt)
        elif w == "helmholtz":
            r, dt = timed(_example("steady-state").main, ["--iters", k(10000), "--newton", k(10000), "--quiet"] + pk)
            r.update(config="helmholtz-2d [2,50x4,1] N_f 10k, adam 10k + lbfgs 10k", wall_s=dt)
        elif w == "discovery":
            r, dt = timed(_example("AC-discovery").main, ["--iters", k(10000), "--quiet", "--precision", prec])
            r.update(config="AC discovery [2,128x4,1] 102,912 data pts, adam 10k (SA col weights)", wall_s=dt)
        elif w == "poisson10m":
            r = poisson_throughput(int(10_000_000 * min(1.0, a.scale)), int(k(50)), 3, prec)
        else:
            raise SystemExit(f"unknown config {w}")
        r["precision_arg"] = a.precision
        print(json.dumps(r), flush=True)


if __name__ == "__main__":
    main()
