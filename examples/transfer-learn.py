"""Transfer learning / resume: train, save, re-create the solver, load, continue at smaller LRs.

Reference examples/transfer-learn.py (5k + 5k + 5k Adam steps with lr 0.005 -> 1e-4 -> 1e-5 after
``save``/``load_model``).  ``save`` writes the flat weights in Keras order plus (optionally) the SA
weights and Adam state, so ``load_model(restore_state=True)`` resumes exactly.
"""
import math
import os
import tempfile

import numpy as np
import torch

from _common import ac_data, l2_on_data_grid, parser, report, solver_kw

import tensordiffeq_amd as tdq
from tensordiffeq_amd.boundaries import IC, DomainND, periodicBC
from tensordiffeq_amd.optimizers import Adam


def make(args, N_f):
    tdq.set_seed(args.seed)
    Domain = DomainND(["x", "t"], time_var="t")
    Domain.add("x", [-1.0, 1.0], 512)
    Domain.add("t", [0.0, 1.0], 201)
    Domain.generate_collocation_points(N_f)

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
    g = torch.Generator().manual_seed(args.seed)
    model = tdq.CollocationSolverND(verbose=not args.quiet)
    model.compile([2, 128, 128, 128, 128, 1], f_model, Domain, BCs, Adaptive_type="self-adaptive",
                  dict_adaptive={"residual": [True], "BCs": [True, False]},
                  init_weights={"residual": [torch.rand(N_f, 1, generator=g)],
                                "BCs": [100 * torch.rand(512, 1, generator=g), None]}, **solver_kw(args))
    return model


def main(argv=None):
    ap = parser(__doc__.splitlines()[0], iters=5000)
    ap.add_argument("--ckpt", default=None, help="checkpoint path (default: a temp dir)")
    args = ap.parse_args(argv)
    N_f = args.n_f or 50000
    ckpt = args.ckpt or os.path.join(tempfile.mkdtemp(prefix="tdq_"), "test_model.npz")
    model = make(args, N_f)
    model.fit(tf_iter=args.iters)
    model.save(ckpt)
    losses = [float(model.losses[-1]["Total Loss"])]
    for lr in (1e-4, 1e-5):
        model = make(args, N_f)
        model.tf_optimizer = Adam(lr)
        model.tf_optimizer_weights = Adam(lr)
        model.load_model(ckpt, restore_state=True)
        model.fit(tf_iter=args.iters)
        model.save(ckpt)
        losses.append(float(model.losses[-1]["Total Loss"]))
    x, t, U = ac_data()
    err, *_ = l2_on_data_grid(model, x, t, U)
    return report("transfer-learn", {"l2_error": err, "loss_stage1": losses[0], "loss_final": losses[-1]},
                  args.quiet, model=model)


if __name__ == "__main__":
    main()
