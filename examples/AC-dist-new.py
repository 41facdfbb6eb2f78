"""Allen-Cahn DP run with the 4th-order periodic derivative model (reference examples/AC-dist-new.py).

Thin wrapper over AC-dist.py's machinery with u, u_x, u_xxx, u_xxxx enforced periodic.
Launch:  torchrun --standalone --local-addr 127.0.0.1 --nproc-per-node 8 examples/AC-dist-new.py
"""
import math
import os

import numpy as np
import torch

from _common import ac_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=1001, n_f=500000).parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 512)
    Domain.add("t", [0.0, 1.0], 201)
    Domain.generate_collocation_points(args.n_f)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_xxx = tdq.grad(u_xx, x)
        return u, u_x, u_xxx, tdq.grad(u_xxx, x)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t - 0.0001 * u_xx + 5.0 * u * u * u - 5.0 * u

    BCs = [IC(Domain, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]]),
           periodicBC(Domain, ["x"], [deriv_model])]
    kw = solver_kw(args)
    if kw["device"] is None and not torch.cuda.is_available():
        kw["device"] = "cpu"
    world = int(os.environ.get("WORLD_SIZE", "1"))
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, Domain, BCs, dist=world > 1, **kw)
    model.fit(tf_iter=args.iters)
    model.fit(tf_iter=args.iters)   # resumable: continues training (reference re-initialised, B6)
    res = {"loss": float(model.losses[-1]["Total Loss"]), "world": world}
    if model.dist_ctx.rank == 0:
        x, t, U = ac_data()
        res["l2_error"], *_ = l2_on_data_grid(model, x, t, U)
        report("AC-dist-new", res, args.quiet, model=model)
    if world > 1:
        tdq.parallel.destroy()
    return res


if __name__ == "__main__":
    main()
