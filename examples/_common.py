"""Shared CLI / data helpers for the example drivers (not part of the library).

Every example exposes ``main(argv=None) -> dict`` so that tests can run it with a handful of
iterations; the defaults reproduce the reference scripts' settings (examples/*.py upstream).
Errors are reported on the ``.mat`` ground-truth grid (the reference evaluates on the Domain
linspace, which is misaligned with the data - SURVEY.md §2.4 B24); the legacy-grid number is
printed too where the reference prints one.
"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
DATA = os.path.join(ROOT, "data")

import numpy as np  # noqa: E402


def parser(desc, iters=10000, newton=0, n_f=None):
    ap = argparse.ArgumentParser(description=desc)
    ap.add_argument("--iters", type=int, default=iters, help="Adam steps (reference setting by default)")
    ap.add_argument("--newton", type=int, default=newton, help="L-BFGS iterations after Adam")
    ap.add_argument("--n-f", type=int, default=n_f, help="collocation points (reference setting by default)")
    ap.add_argument("--device", default=None, help="cuda / cpu (default: cuda if available)")
    ap.add_argument("--backend", default="auto", help="auto | hip | jet | autograd")
    ap.add_argument("--precision", default=None, help="bf16x3 | bf16 | fp32 (HIP jet GEMMs)")
    ap.add_argument("--newton-precision", default=None, help="jet precision of the L-BFGS phase (default: --precision)")
    ap.add_argument("--lbfgs-stop", default=None, choices=["fixed", "legacy"],
                    help="L-BFGS function-change test: |f - f_old| < tolX (fixed) or the reference's |f| < tolX")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--plot", action="store_true", help="draw the reference-style figures")
    ap.add_argument("--quiet", action="store_true")
    return ap


def solver_kw(args):
    kw = {"backend": args.backend, "device": args.device, "precision": args.precision}
    if getattr(args, "newton_precision", None):
        kw["newton_precision"] = args.newton_precision
    if getattr(args, "lbfgs_stop", None):
        kw["lbfgs_stop"] = args.lbfgs_stop
    return kw


def ac_data():
    import scipy.io
    d = scipy.io.loadmat(os.path.join(DATA, "AC.mat"))
    return d["x"].flatten(), d["tt"].flatten(), np.real(d["uu"])   # uu: (512 x, 201 t)


def burgers_data():
    import scipy.io
    d = scipy.io.loadmat(os.path.join(DATA, "burgers_shock.mat"))
    return d["x"].flatten(), d["t"].flatten(), np.real(d["usol"])  # usol: (256 x, 100 t)


def grid_points(x, t):
    X, T = np.meshgrid(x, t)
    return np.hstack((X.flatten()[:, None], T.flatten()[:, None])), X, T


def l2_on_data_grid(model, x, t, U):
    """Relative L2 of u on the data's own (x, t) grid; ``U`` is (len(x), len(t))."""
    import tensordiffeq_amd as tdq
    X_star, _, _ = grid_points(x, t)
    u_pred, f_pred = model.predict(X_star)
    return float(tdq.find_L2_error(u_pred, U.T.flatten()[:, None])), X_star, u_pred, f_pred


def report(name, res, quiet=False, model=None):
    """Print (unless quiet) and return ``res``; with ``model``, also which engine ran its loss
    (``hip`` = the fused MI355X kernels, ``jet`` = torch Taylor jets, ``autograd``)."""
    if model is not None:
        prog = model.program()
        res["backend"] = prog.backend
        fi = getattr(model, "fit_info", None) or {}
        adam = fi.get("adam") or {}
        if adam.get("steps"):   # wall time of the Adam phase per step (graph capture included)
            res["adam_ms_per_step"] = 1e3 * float(adam["wall_s"]) / int(adam["steps"])
        if fi.get("lbfgs"):
            res["lbfgs_iters"] = int(fi["lbfgs"].get("n_iter", 0))
    if not quiet:
        print(f"[{name}] " + ", ".join(f"{k}={v:.4e}" if isinstance(v, float) else f"{k}={v}"
                                       for k, v in res.items()))
    return res
