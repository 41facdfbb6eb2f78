"""3-D (x, y, t) viscous Burgers-type problem with a mixed-derivative periodic model.

IC u(x, y, 0) = -sin(pi x) - sin(pi y); periodic in x and y for u, u_x, u_y, u_xx, u_yy, u_xy, u_yx;
residual u_t + u u_x - (0.05/pi) u_xx.  Net [3, 128 x 4, 1], N_f = 20,000, Adam 1k + L-BFGS 1k
(reference examples/testing.py, which compared against a 1-D data file; no ground truth exists for
this 3-D problem, so the driver reports the loss only).
"""
import math

import numpy as np
import torch

from _common import parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=1000, newton=1000).parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "y", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 256)
    Domain.add("y", [-1.0, 1.0], 256)
    Domain.add("t", [0.0, 1.0], 100)
    Domain.generate_collocation_points(args.n_f or 20000)

    def func_ic_xy(x, y):
        return -np.sin(x * math.pi) + -np.sin(y * math.pi)

    def deriv_model(u_model, x, y, t):
        u = u_model(torch.cat([x, y, t], 1))
        u_x = tdq.grad(u, x)
        u_y = tdq.grad(u, y)
        return u, u_x, u_y, tdq.grad(u_x, x), tdq.grad(u_y, y), tdq.grad(u_x, y), tdq.grad(u_y, x)

    def f_model(u_model, x, y, t):
        u = u_model(torch.cat([x, y, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t + u * u_x - (0.05 / math.pi) * u_xx

    BCs = [IC(Domain, [func_ic_xy], var=[["x", "y"]]), periodicBC(Domain, ["x", "y"], [deriv_model])]
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([3, 128, 128, 128, 128, 1], f_model, Domain, BCs, **solver_kw(args))
    model.fit(tf_iter=args.iters, newton_iter=args.newton)
    return report("testing-3d", {"loss": float(model.losses[-1]["Total Loss"]),
                                 "terms": len(model.losses[-1]) - 1}, args.quiet, model=model)


if __name__ == "__main__":
    main()
