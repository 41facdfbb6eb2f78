"""2-D Helmholtz: u_xx + u_yy + k^2 u = q(x, y) on [-1,1]^2, u = 0 on the boundary.

Exact solution u = sin(pi x) sin(4 pi y).  Net [2, 50 x 4, 1], N_f = 10,000, Adam 10k + L-BFGS 10k
(reference examples/steady-state.py).
"""
import math

import numpy as np
import torch

from _common import parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import DomainND, dirichletBC
from tensordiffeq_amd.utils import constant


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=10000, newton=10000).parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "y"])
    Domain.add("x", [-1.0, 1.0], 1001)
    Domain.add("y", [-1.0, 1.0], 1001)
    Domain.generate_collocation_points(args.n_f or 10000)

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        u_x = tdq.grad(u, x)
        u_y = tdq.grad(u, y)
        u_xx = tdq.grad(u_x, x)
        u_yy = tdq.grad(u_y, y)
        a1, a2, ksq, pi = constant(1.0), constant(4.0), constant(1.0), constant(math.pi)
        s = torch.sin(a1 * pi * x) * torch.sin(a2 * pi * y)
        forcing = -(a1 * pi) ** 2 * s - (a2 * pi) ** 2 * s + ksq * s
        return u_xx + u_yy + ksq * u - forcing

    BCs = [dirichletBC(Domain, val=0.0, var="x", target="upper"),
           dirichletBC(Domain, val=0.0, var="x", target="lower"),
           dirichletBC(Domain, val=0.0, var="y", target="upper"),
           dirichletBC(Domain, val=0.0, var="y", target="lower")]
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 50, 50, 50, 50, 1], f_model, Domain, BCs, **solver_kw(args))
    model.fit(tf_iter=args.iters, newton_iter=args.newton)

    x = np.linspace(-1, 1, 201)
    X, Y = np.meshgrid(x, x)
    X_star = np.hstack((X.flatten()[:, None], Y.flatten()[:, None]))
    u_star = (np.sin(math.pi * X) * np.sin(4 * math.pi * Y)).flatten()[:, None]
    u_pred, _ = model.predict(X_star)
    res = report("steady-state", {"l2_error": float(tdq.find_L2_error(u_pred, u_star)),
                                  "loss": float(model.losses[-1]["Total Loss"])}, args.quiet, model=model)
    if args.plot:
        tdq.plotting.plot_solution_domain1D(model, [x, x], ub=np.array([1.0, 1.0]), lb=np.array([-1.0, -1.0]),
                                            Exact_u=(np.sin(math.pi * X) * np.sin(4 * math.pi * Y)).T)
    return res


if __name__ == "__main__":
    main()
