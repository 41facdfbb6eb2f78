"""Allen-Cahn baseline on a coarser 256 x 100 domain, N_f = 20,000, Adam 1k + L-BFGS 1k
(reference examples/testing1D-AC.py, which scored against burgers_shock.mat by mistake; this port
scores against AC.mat)."""
import math

import numpy as np
import torch

from _common import ac_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=1000, newton=1000).parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 256)
    Domain.add("t", [0.0, 1.0], 100)
    Domain.generate_collocation_points(args.n_f or 20000)

    def deriv_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        return u, tdq.grad(u, x)

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t - 0.0001 * u_xx + 5.0 * u * u * u - 5.0 * u

    BCs = [IC(Domain, [lambda x: x ** 2 * np.cos(math.pi * x)], var=[["x"]]),
           periodicBC(Domain, ["x"], [deriv_model])]
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, Domain, BCs, **solver_kw(args))
    model.fit(tf_iter=args.iters, newton_iter=args.newton)
    x, t, U = ac_data()
    err, *_ = l2_on_data_grid(model, x, t, U)
    return report("testing1D-AC", {"l2_error": err, "loss": float(model.losses[-1]["Total Loss"])}, args.quiet, model=model)


if __name__ == "__main__":
    main()
