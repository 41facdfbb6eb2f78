"""Burgers (nu = 0.05/pi) with data assimilation: 200 observations of the shock solution at t = 0.75.

``compile_data(x, t, y)`` adds MSE(u(x_d, t_d), y_d) to the loss (the reference stored the data but
never used it - SURVEY.md §2.4 B17; reference examples/burgers-assimilate.py used the removed 1-D
API, ported here to DomainND).  The observations come from burgers_shock.mat (nu = 0.01/pi), so
they pull the nu = 0.05/pi solution toward the sharper shock, as in the reference.
"""
import math

import numpy as np
import torch

from _common import burgers_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, dirichletBC


def main(argv=None):
    ap = parser(__doc__.splitlines()[0], iters=100, newton=100)
    ap.add_argument("--n-obs", type=int, default=200)
    args = ap.parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 256)
    Domain.add("t", [0.0, 1.0], 100)
    Domain.generate_collocation_points(args.n_f or 10000)
    BCs = [IC(Domain, [lambda x: -np.sin(math.pi * x)], var=[["x"]], n_values=60),
           dirichletBC(Domain, val=0.0, var="x", target="upper"),
           dirichletBC(Domain, val=0.0, var="x", target="lower")]

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t + u * u_x - (0.05 / math.pi) * u_xx

    x, t, U = burgers_data()
    rng = np.random.default_rng(args.seed)
    idx_xs = rng.choice(x.shape[0], args.n_obs, replace=False)
    it = 75
    x_s = x[idx_xs][:, None]
    t_s = np.full_like(x_s, t[it])
    y_s = U[idx_xs, it][:, None]

    model = tdq.CollocationSolverND(assimilate=True, verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, Domain, BCs, **solver_kw(args))
    model.compile_data(x_s, t_s, y_s)
    model.fit(tf_iter=args.iters, newton_iter=args.newton)
    err, *_ = l2_on_data_grid(model, x, t, U)
    data_err = float(np.sqrt(np.mean((model.predict(np.hstack([x_s, t_s]))[0] - y_s) ** 2)))
    return report("burgers-assimilate", {"l2_error": err, "obs_rmse": data_err}, args.quiet, model=model)


if __name__ == "__main__":
    main()
