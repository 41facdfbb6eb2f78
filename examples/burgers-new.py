"""Viscous Burgers: u_t + u u_x - (0.01/pi) u_xx = 0, u(x,0) = -sin(pi x), u(+-1, t) = 0.

Net [2, 20 x 8, 1], N_f = 10,000, Adam 10k + L-BFGS 10k (reference examples/burgers-new.py).
"""
import math

import numpy as np
import torch

from _common import burgers_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, dirichletBC


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=10000, newton=10000).parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 256)
    Domain.add("t", [0.0, 1.0], 100)
    Domain.generate_collocation_points(args.n_f or 10000)

    def func_ic(x):
        return -np.sin(x * math.pi)

    BCs = [IC(Domain, [func_ic], var=[["x"]]),
           dirichletBC(Domain, val=0.0, var="x", target="upper"),
           dirichletBC(Domain, val=0.0, var="x", target="lower")]

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t + u * u_x - (0.01 / math.pi) * u_xx

    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2] + [20] * 8 + [1], f_model, Domain, BCs, **solver_kw(args))
    model.fit(tf_iter=args.iters, newton_iter=args.newton)
    x, t, U = burgers_data()
    err, *_ = l2_on_data_grid(model, x, t, U)
    res = report("burgers", {"l2_error": err, "loss": float(model.losses[-1]["Total Loss"])}, args.quiet, model=model)
    if args.plot:
        tdq.plotting.plot_solution_domain1D(model, [x, t], ub=np.array([1.0, 1.0]), lb=np.array([-1.0, 0.0]),
                                            Exact_u=U)
    return res


if __name__ == "__main__":
    main()
