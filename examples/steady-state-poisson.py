"""2-D Poisson u_xx + u_yy = -sin(pi x) sin(pi y) on [0,1]^2 with function-valued Dirichlet BCs.

Exact u = sin(pi x) sin(pi y) / (2 pi^2).  Net [2, 16, 16, 1], N_f = 100, the user swaps the network
optimizer for Adam(lr=0.005) like the reference (examples/steady-state-poisson.py).  The reference
declares its ``lower_x`` BC with target="upper" (SURVEY.md §2.4 B29); this port uses "lower".
"""
import math

import numpy as np
import torch

from _common import parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import DomainND, FunctionDirichletBC, dirichletBC
from tensordiffeq_amd.optimizers import Adam
from tensordiffeq_amd.utils import constant


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=4000).parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "y"])
    Domain.add("x", [0, 1.0], 11)
    Domain.add("y", [0, 1.0], 11)
    Domain.generate_collocation_points(args.n_f or 100)

    def f_model(u_model, x, y):
        u = u_model(torch.cat([x, y], 1))
        u_xx = tdq.grad(tdq.grad(u, x), x)
        u_yy = tdq.grad(tdq.grad(u, y), y)
        pi = constant(math.pi)
        forcing = -torch.sin(pi * x) * torch.sin(pi * y)
        return u_xx + u_yy - forcing

    def func_upper_x(y):
        return -np.sin(math.pi * y) * np.sin(math.pi)

    def func_upper_y(x):
        return -np.sin(math.pi * x) * np.sin(math.pi)

    BCs = [FunctionDirichletBC(Domain, fun=[func_upper_x], var="x", target="upper", func_inputs=["y"], n_values=10),
           dirichletBC(Domain, val=0.0, var="x", target="lower"),
           FunctionDirichletBC(Domain, fun=[func_upper_y], var="y", target="upper", func_inputs=["x"], n_values=10),
           dirichletBC(Domain, val=0.0, var="y", target="lower")]
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 16, 16, 1], f_model, Domain, BCs, **solver_kw(args))
    model.tf_optimizer = Adam(lr=.005)
    model.fit(tf_iter=args.iters)

    x = np.linspace(0, 1, 11)
    X, Y = np.meshgrid(x, x)
    X_star = np.hstack((X.flatten()[:, None], Y.flatten()[:, None]))
    u_star = ((np.sin(math.pi * X) * np.sin(math.pi * Y)) / (2 * math.pi ** 2)).flatten()[:, None]
    u_pred, _ = model.predict(X_star)
    return report("poisson", {"l2_error": float(tdq.find_L2_error(u_pred, u_star)),
                              "loss": float(model.losses[-1]["Total Loss"])}, args.quiet, model=model)


if __name__ == "__main__":
    main()
