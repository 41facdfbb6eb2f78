"""Allen-Cahn data-parallel training: one process per GPU over RCCL (torch.distributed).

Collocation points AND their SA weights are sharded across ranks; IC/periodic terms are replicated
and scaled 1/world; one flat fp32 gradient bucket is all-reduced per step.  The global loss and the
gradient equal single-GPU full-batch training (the intent of the reference's MirroredStrategy path,
SURVEY.md §2.3 / B3-B7; reference examples/AC-dist.py, examples/AC-dist-new.py).

Launch:  torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 8 examples/AC-dist.py
On CPU (gloo) for a smoke run:  torchrun --nproc-per-node 2 ... --device cpu --iters 5 --n-f 2000
"""
import math
import os

import numpy as np
import torch

from _common import ac_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC


def main(argv=None):
    ap = parser(__doc__.splitlines()[0], iters=1001, n_f=500000)
    ap.add_argument("--sa", action="store_true", help="self-adaptive weights on residual + IC")
    ap.add_argument("--passes", type=int, default=2, help="fit() calls (resumable; reference calls fit twice)")
    args = ap.parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 512)
    Domain.add("t", [0.0, 1.0], 201)
    N_f = args.n_f
    Domain.generate_collocation_points(N_f)   # same seed on every rank -> identical global point set

    def func_ic(x):
        return x ** 2 * np.cos(math.pi * x)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return u, tdq.grad(u, x)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t - 0.0001 * u_xx + 5.0 * u * u * u - 5.0 * u

    BCs = [IC(Domain, [func_ic], var=[["x"]]), periodicBC(Domain, ["x"], [deriv_model])]
    kw = solver_kw(args)
    if kw["device"] is None and not torch.cuda.is_available():
        kw["device"] = "cpu"
    extra = {}
    if args.sa:
        g = torch.Generator().manual_seed(args.seed)
        extra = dict(Adaptive_type="self-adaptive", dict_adaptive={"residual": [True], "BCs": [True, False]},
                     init_weights={"residual": [torch.rand(N_f, 1, generator=g)],
                                   "BCs": [100 * torch.rand(512, 1, generator=g), None]})
    world = int(os.environ.get("WORLD_SIZE", "1"))
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, Domain, BCs, dist=world > 1, **extra, **kw)
    for k in range(args.passes):
        model.fit(tf_iter=args.iters)
        if not args.quiet and model.dist_ctx.rank == 0:
            print(f"training pass {k + 1} completed")
    res = {"loss": float(model.losses[-1]["Total Loss"]), "world": world}
    if model.dist_ctx.rank == 0:
        x, t, U = ac_data()
        res["l2_error"], *_ = l2_on_data_grid(model, x, t, U)
        report("AC-dist", res, args.quiet, model=model)
    if world > 1:
        tdq.parallel.destroy()
    return res


if __name__ == "__main__":
    main()
