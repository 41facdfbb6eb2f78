"""Allen-Cahn SA-PINN with the 4th-order periodic model (reference examples/testing1D.py, written for
the removed CollocationSolver1D ``isAdaptive/col_weights/u_weights`` API; ported to the ND solver's
``dict_adaptive/init_weights``)."""
import math

import numpy as np
import torch

from _common import ac_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC


def main(argv=None):
    args = parser(__doc__.splitlines()[0], iters=10000, newton=10000).parse_args(argv)
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 512)
    Domain.add("t", [0.0, 1.0], 201)
    N_f = args.n_f or 50000
    Domain.generate_collocation_points(N_f)

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
    g = torch.Generator().manual_seed(args.seed)
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, Domain, BCs, Adaptive_type=1,
                  dict_adaptive={"residual": [True], "BCs": [True, False]},
                  init_weights={"residual": [torch.rand(N_f, 1, generator=g)],
                                "BCs": [100 * torch.rand(512, 1, generator=g), None]}, **solver_kw(args))
    model.fit(tf_iter=args.iters, newton_iter=args.newton)
    x, t, U = ac_data()
    err, *_ = l2_on_data_grid(model, x, t, U)
    return report("testing1D", {"l2_error": err, "loss": float(model.losses[-1]["Total Loss"])}, args.quiet, model=model)


if __name__ == "__main__":
    main()
