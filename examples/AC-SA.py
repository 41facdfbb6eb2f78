"""Allen-Cahn self-adaptive PINN (McClenny & Braga-Neto) - the flagship configuration.

u_t - 1e-4 u_xx + 5 u^3 - 5 u = 0 on x in [-1, 1], t in [0, 1]; u(x, 0) = x^2 cos(pi x);
periodic in x for u and u_x.  SA weights on the residual (U[0,1] init) and on the IC (100 U[0,1]).
Net [2, 128 x 4, 1], N_f = 50,000, Adam 10k + L-BFGS 10k (reference examples/AC-SA.py).
Run:  python examples/AC-SA.py [--iters 10000 --newton 10000]
"""
import math

import numpy as np
import torch

from _common import ac_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC


def build(args):
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 512)
    Domain.add("t", [0.0, 1.0], 201)
    N_f = args.n_f or 50000
    Domain.generate_collocation_points(N_f)

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
        c1 = tdq.utils.constant(.0001)
        c2 = tdq.utils.constant(5.0)
        return u_t - c1 * u_xx + c2 * u * u * u - c2 * u

    init = IC(Domain, [func_ic], var=[["x"]])
    x_periodic = periodicBC(Domain, ["x"], [deriv_model])
    g = torch.Generator().manual_seed(args.seed)
    dict_adaptive = {"residual": [True], "BCs": [True, False]}
    init_weights = {"residual": [torch.rand(N_f, 1, generator=g)],
                    "BCs": [100 * torch.rand(512, 1, generator=g), None]}
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, Domain, [init, x_periodic],
                  Adaptive_type="self-adaptive", dict_adaptive=dict_adaptive, init_weights=init_weights,
                  **solver_kw(args))
    return model, Domain


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=10000, newton=10000).parse_args(argv)
    import time
    model, Domain = build(args)
    t0 = time.perf_counter()
    model.fit(tf_iter=args.iters)
    t1 = time.perf_counter()
    if args.newton:
        model.fit(newton_iter=args.newton)
    t2 = time.perf_counter()
    x, t, U = ac_data()
    err, X_star, u_pred, f_pred = l2_on_data_grid(model, x, t, U)
    res = report("AC-SA", {"l2_error": err, "loss": float(model.losses[-1]["Total Loss"]),
                           "min_loss_adam": float(model.min_loss["adam"]),
                           "min_loss_lbfgs": float(model.min_loss["l-bfgs"]),
                           "adam_s": t1 - t0, "lbfgs_s": t2 - t1, "backend": model.active_backend,
                           "lbfgs_n_iter": model.fit_info.get("lbfgs", {}).get("n_iter"),
                           "lbfgs_reason": model.fit_info.get("lbfgs", {}).get("reason")}, args.quiet, model=model)
    if args.plot:
        tdq.plotting.plot_solution_domain1D(model, [x, t], ub=np.array([1.0, 1.0]), lb=np.array([-1.0, 0.0]),
                                            Exact_u=U)
    return res


if __name__ == "__main__":
    main()
