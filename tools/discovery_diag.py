"""Why does the reference AC-discovery program (examples/AC-discovery.py:14-66, c1 = v from 0)
land c1 5-11x above its true 1e-4?  

For the trained network, and for the AC.mat field itself (finite differences on its 512 x 201
grid), this prints the least-squares coefficients of

    u_t = c1 u_xx - c2 (u^3 - u)

so the learned c1 can be compared with (a) what the DATA implies, (b) what the NETWORK's own
derivatives imply (the loss's minimizer in c1 for that network), and (c) how well the network's
u_xx matches the data's in the sharp interface layers.  Training runs the reference schedule
(Adam ``--iters``, col-weight Adam lr 0.005 / beta_1 0.95) in the bench's precision; ``--newton``
adds the L-BFGS phase.

    python tools/discovery_diag.py --seeds 0 1 2 --iters 10000 [--newton 5000] [--precision bf16|fp32]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def fd_coeffs(data):
    """Least-squares (c1, c2) of the data field: central differences, x periodic, interior t."""
    x, t = data["x"].flatten(), data["tt"].flatten()
    U = np.real(data["uu"]).astype(np.float64)        # (nx, nt)
    dx, dt = x[1] - x[0], t[1] - t[0]
    u = U[:, 1:-1]
    u_t = (U[:, 2:] - U[:, :-2]) / (2 * dt)
    u_xx = (np.roll(U, -1, 0) - 2 * U + np.roll(U, 1, 0))[:, 1:-1] / dx ** 2
    return _lsq(u_t.ravel(), u_xx.ravel(), u.ravel()), (u, u_t, u_xx)


def _lsq(u_t, u_xx, u):
    A = np.stack([u_xx, -(u ** 3 - u)], 1)
    sol, *_ = np.linalg.lstsq(A, u_t, rcond=None)
    return float(sol[0]), float(sol[1])


def net_derivs(m, X, dev):
    """u, u_t, u_xx of the network at X (float64 autograd on its float32 weights)."""
    net = m.u_model
    ws = [(k.double(), b.double()) for k, b in net.weights(net.flat.detach())]
    out = []
    for lo in range(0, X.shape[0], 32768):
        xt = torch.tensor(X[lo:lo + 32768], dtype=torch.float64, device=dev)
        x = xt[:, 0:1].clone().requires_grad_(True)
        t = xt[:, 1:2].clone().requires_grad_(True)
        h = torch.cat([x, t], 1)
        for i, (k, b) in enumerate(ws):
            h = h @ k + b
            if i < len(ws) - 1:
                h = torch.tanh(h)
        u = h
        u_x, u_t = torch.autograd.grad(u.sum(), [x, t], create_graph=True)
        u_xx, = torch.autograd.grad(u_x.sum(), [x])
        out.append(torch.cat([u, u_t, u_xx], 1).detach().cpu().numpy())
    return np.concatenate(out, 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, nargs="+", default=[0, 1, 2])
    ap.add_argument("--iters", type=int, default=10000)
    ap.add_argument("--newton", type=int, default=0)
    ap.add_argument("--precision", default="bf16")
    ap.add_argument("--c1-param", default="linear", choices=["linear", "log"])
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import scipy.io
    import bench
    bench.DISCOVERY_C1 = args.c1_param
    data = scipy.io.loadmat(os.path.join(HERE, "data", "AC.mat"))
    (c1_fd, c2_fd), (u, u_t, u_xx) = fd_coeffs(data)
    rec = {"data_fd": {"c1": c1_fd, "c2": c2_fd,
                       "max_abs_u_xx": float(np.abs(u_xx).max()),
                       "note": "central differences on the AC.mat grid (dx 3.9e-3, dt 5e-3)"}}
    print(json.dumps(rec["data_fd"]))
    # the data's u_xx on the grid points, in the bench's point order (t-major meshgrid of x, t)
    x, t = data["x"].flatten(), data["tt"].flatten()
    dev = torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu")
    runs = []
    for sd in args.seeds:
        m = bench.build_discovery(0, 1, "auto", dev, False, args.precision, seed=sd)
        t0 = time.perf_counter()
        m.fit(tf_iter=args.iters, newton_iter=args.newton)
        wall = time.perf_counter() - t0
        c1 = bench.discovery_c1(m.vars[0])
        c2 = float(m.vars[1].detach())
        X, T = np.meshgrid(x, t[1:-1])   # interior times, the FD grid's
        Xs = np.stack([X.ravel(), T.ravel()], 1)
        d = net_derivs(m, Xs, dev)
        un, un_t, un_xx = d[:, 0], d[:, 1], d[:, 2]
        # FD fields in the same (t-major) order
        u_d, u_t_d, u_xx_d = (a.T.ravel() for a in (u, u_t, u_xx))
        c1_net, c2_net = _lsq(un_t, un_xx, un)
        sharp = np.abs(u_xx_d) > 0.1 * np.abs(u_xx_d).max()
        r = {"seed": sd, "precision": args.precision, "c1_param": args.c1_param,
             "iters": args.iters, "newton": args.newton, "wall_s": round(wall, 2),
             "c1_learned": c1, "c2_learned": c2,
             "c1_lsq_net_derivs": c1_net, "c2_lsq_net_derivs": c2_net,
             "u_rel_l2": float(np.linalg.norm(un - u_d) / np.linalg.norm(u_d)),
             "u_t_rel_l2": float(np.linalg.norm(un_t - u_t_d) / np.linalg.norm(u_t_d)),
             "u_xx_rel_l2": float(np.linalg.norm(un_xx - u_xx_d) / np.linalg.norm(u_xx_d)),
             "u_xx_rel_l2_sharp": float(np.linalg.norm((un_xx - u_xx_d)[sharp]) / np.linalg.norm(u_xx_d[sharp])),
             "max_abs_u_xx_net": float(np.abs(un_xx).max()), "max_abs_u_xx_data": float(np.abs(u_xx_d).max()),
             "frac_sharp_points": float(sharp.mean())}
        # the residual the loss sees at the true c1 vs the learned c1 (network derivatives)
        for name, cc1 in (("true", 1e-4), ("learned", c1)):
            f = un_t - cc1 * un_xx + c2 * (un ** 3 - un)
            r[f"mse_f_at_{name}_c1"] = float(np.mean(f ** 2))
        print(json.dumps(r))
        runs.append(r)
    rec["runs"] = runs
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
