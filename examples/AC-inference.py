"""Allen-Cahn inference of PDE coefficients from data (reference examples/AC-inference.py).

Same problem as AC-discovery.py; kept as its own driver because the reference ships both.  The
baseline (non-adaptive) inverse problem is obtained with ``--no-sa``.
"""
import torch

from _common import ac_data, grid_points, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.models import DiscoveryModel
from tensordiffeq_amd.optimizers import Adam


def main(argv=None):
    ap = parser(__doc__.splitlines()[0], iters=10000)
    ap.add_argument("--no-sa", action="store_true", help="baseline inverse problem (no col_weights)")
    args = ap.parse_args(argv)
    tdq.set_seed(args.seed)
    params = [tdq.Variable(0.0), tdq.Variable(0.0)]

    def f_model(u_model, var, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        return u_t - var[0] * u_xx + var[1] * u * u * u - var[1] * u

    x, t, U = ac_data()
    X_star, _, _ = grid_points(x, t)
    u_star = U.T.flatten()[:, None]
    X = [X_star[:, 0:1], X_star[:, 1:2]]
    col_weights = None if args.no_sa else torch.rand(X_star.shape[0], 1,
                                                      generator=torch.Generator().manual_seed(args.seed))
    model = DiscoveryModel(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, X, u_star, params, col_weights=col_weights,
                  **solver_kw(args))
    if col_weights is not None:
        model.tf_optimizer_weights = Adam(lr=0.005, beta_1=.95)
    model.fit(tf_iter=args.iters)
    c1, c2 = (float(v.detach()) for v in model.vars)
    return report("AC-inference", {"c1": c1, "c2": c2}, args.quiet, model=model)


if __name__ == "__main__":
    main()
