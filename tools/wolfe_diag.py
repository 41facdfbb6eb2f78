"""Line-search L-BFGS (``newton_eager=False``, optimizers/lbfgs_wolfe.py) on AC-SA: is an early stop
the algorithm or the reduced-precision objective?  

One Adam phase (bf16 fused step) gives a start point; from that SAME point the same WolfeLBFGS runs
on several objectives:
  * fp64  - the loss program on the torch Taylor-jet engine in float64, float64 optimizer state
            (no graphs): the algorithm on an exact objective;
  * fp32 / bf16x3 / bf16 - the HIP objectives (LossGradEngine.evaluate_fg, graphs).
Each run reports iterations, function evaluations, steepest-descent restarts, the stop reason, the
final loss, wall time and the L2 error on AC.mat.  One JSON line per run.

    python tools/wolfe_diag.py --npts 5000 --adam 10000 --iters 10000 --objectives fp64 bf16x3 fp32
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import bench
    from tensordiffeq_amd.fit import LossGradEngine
    from tensordiffeq_amd.optimizers import lbfgs_wolfe

    ap = argparse.ArgumentParser()
    ap.add_argument("--npts", type=int, default=5000)
    ap.add_argument("--adam", type=int, default=10000)
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--objectives", nargs="*", default=["fp64", "bf16x3", "fp32"])
    ap.add_argument("--out", default=None)
    ap.add_argument("--hz-eps", type=float, nargs="*", default=[1e-6],
                    help="approximate-Wolfe loss tolerances to run (HIP objectives)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    m = bench.build_problem(a.npts, 1, "hip", dev, False, "bf16", seed=a.seed)
    t0 = time.perf_counter()
    m.fit(tf_iter=a.adam)
    torch.cuda.synchronize()
    x_adam = m.u_model.flat.detach().clone()
    lams = [lam.detach().clone() for lam in m.lambdas]
    rec0 = {"what": "adam", "npts": a.npts, "adam": a.adam, "seed": a.seed, "s": round(time.perf_counter() - t0, 2),
            "l2": float(bench.l2_on_ac_grid(m))}
    print(json.dumps(rec0), flush=True)
    out = [rec0]
    runs = [(obj, e) for obj in a.objectives for e in (a.hz_eps if obj != "fp64" else [1e-6])]
    for obj, eps in runs:
        with torch.no_grad():
            m.u_model.flat.copy_(x_adam)
            for lam, v in zip(m.lambdas, lams):
                lam.copy_(v)
        if obj == "fp64":
            ref = bench.build_problem(a.npts, 1, "jet", dev, False, "bf16", seed=a.seed)
            prog = ref.program()
            lam64 = [lam.detach().double() for lam in lams]
            x = x_adam.double().clone()

            def evaluate():
                p = x.detach().requires_grad_(True)
                tot, _ = prog.evaluate(p, lam64)
                g, = torch.autograd.grad(tot, [p])
                return torch.cat([g.reshape(-1), tot.detach().reshape(1)])
            use_graph = False
        else:
            eng = LossGradEngine(m, m.program(precision=obj), m.lambdas)
            x = m.u_model.flat.data
            evaluate = eng.evaluate_fg
            use_graph = True
        t0 = time.perf_counter()
        opt = lbfgs_wolfe.minimize(evaluate, x, a.iters, use_graph=use_graph, hz_eps=eps)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        with torch.no_grad():
            m.u_model.flat.copy_(x.float())
        f = opt.f_hist
        rec = {"what": "wolfe", "objective": obj, "hz_eps": eps, "npts": a.npts, "seed": a.seed, "n_iter": opt.n_iter,
               "func_evals": opt.func_eval, "restarts": opt.n_restarts, "reason": opt.reason,
               "f_start": f[0], "f_end": f[-1], "f_at": {str(k): f[k] for k in (10, 100, 1000, 3000, 5000) if k < len(f)},
               "s": round(wall, 2), "ms_per_eval": round(1e3 * wall / max(1, opt.func_eval), 3),
               "l2": float(bench.l2_on_ac_grid(m))}
        print(json.dumps(rec), flush=True)
        out.append(rec)
    if a.out:
        with open(a.out, "w") as fh:
            for r in out:
                fh.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
