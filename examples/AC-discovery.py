"""Allen-Cahn coefficient discovery (inverse problem) with self-adaptive collocation weights.

Learns c1, c2 in u_t - c1 u_xx + c2 u^3 - c2 u = 0 (truth: 1e-4, 5) jointly with the network
from the full AC.mat field (102,912 points).  The col_weights optimizer is replaced by a user Adam
(beta_1 = 0.95) exactly like the reference (examples/AC-discovery.py, Adam 10k).  ``--newton N``
adds N L-BFGS iterations over the network and the coefficients after Adam (not in the reference,
which notes the example "doesnt work quite yet": Adam alone cannot resolve c1 = 1e-4).
"""
import numpy as np
import torch

from _common import ac_data, grid_points, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.models import DiscoveryModel
from tensordiffeq_amd.optimizers import Adam


def main(argv=None):
    ap = parser(__doc__.splitlines()[0], iters=10000)
    ap.add_argument("--n-data", type=int, default=None, help="subsample the data points (default: all)")
    ap.add_argument("--c1-param", default="linear", choices=["linear", "scaled", "log"],
                    help="c1 = v (reference), 1e-3 v, or exp(v) from v = -6 (Raissi et al.'s parametrization "
                         "of a small positive coefficient)")
    args = ap.parse_args(argv)
    tdq.set_seed(args.seed)
    params = [tdq.Variable(-6.0 if args.c1_param == "log" else 0.0), tdq.Variable(0.0)]

    def coef1(v):
        if args.c1_param == "log":
            return torch.exp(v)
        return 1e-3 * v if args.c1_param == "scaled" else v

    def f_model(u_model, var, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x)
        u_xx = tdq.grad(u_x, x)
        u_t = tdq.grad(u, t)
        c1, c2 = coef1(var[0]), var[1]
        return u_t - c1 * u_xx + c2 * u * u * u - c2 * u

    x, t, U = ac_data()
    X_star, _, _ = grid_points(x, t)
    u_star = U.T.flatten()[:, None]
    if args.n_data:
        idx = np.random.default_rng(args.seed).choice(X_star.shape[0], args.n_data, replace=False)
        X_star, u_star = X_star[idx], u_star[idx]
    X = [X_star[:, 0:1], X_star[:, 1:2]]
    col_weights = torch.rand(X_star.shape[0], 1, generator=torch.Generator().manual_seed(args.seed))
    model = DiscoveryModel(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, X, u_star, params, col_weights=col_weights,
                  **solver_kw(args))
    model.tf_optimizer_weights = Adam(lr=0.005, beta_1=.95)
    model.fit(tf_iter=args.iters, newton_iter=args.newton)
    c1, c2 = float(coef1(model.vars[0].detach())), float(model.vars[1].detach())
    info = {k: round(v.get("wall_s", 0.0), 3) for k, v in model.fit_info.items()}
    return report("AC-discovery", {"c1": c1, "c2": c2, "c1_rel_err": abs(c1 - 1e-4) / 1e-4,
                                   "c2_rel_err": abs(c2 - 5.0) / 5.0, "wall_s": info,
                                   "lbfgs": model.fit_info.get("lbfgs")}, args.quiet, model=model)


if __name__ == "__main__":
    main()
