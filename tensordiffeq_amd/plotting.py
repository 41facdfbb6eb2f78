"""Post-processing plots (reference tensordiffeq/plotting.py:1-157, Raissi-style figures).

``plot_solution_domain1D`` draws the predicted field u(t, x) plus three time slices against the
exact solution; ``plot_weights`` / ``plot_glam_values`` scatter the self-adaptive collocation
weights (the reference read attributes that no longer existed, B26 - here they come from
``model.lambdas`` and the collocation points); ``plot_residuals`` heat-maps a residual field;
``get_griddata`` is cubic scattered-data interpolation.  matplotlib is imported lazily and the
figures are returned (``show=False`` or a non-interactive backend keeps scripts headless).
"""
from __future__ import annotations

import numpy as np


def _plt():
    import matplotlib
    if matplotlib.get_backend().lower().startswith("qt") is False:
        pass
    import matplotlib.pyplot as plt
    return plt


def figsize(scale, nplots=1):
    fig_width_pt = 390.0
    inches_per_pt = 1.0 / 72.27
    golden_mean = (np.sqrt(5.0) - 1.0) / 2.0
    fig_width = fig_width_pt * inches_per_pt * scale
    return [fig_width, nplots * fig_width * golden_mean]


def newfig(width, nplots=1):
    plt = _plt()
    fig = plt.figure(figsize=figsize(width, nplots))
    ax = fig.add_subplot(111)
    return fig, ax


def get_griddata(grid, data, dims):
    from scipy.interpolate import griddata
    return griddata(grid, data, dims, method="cubic")


def plot_solution_domain1D(model, domain, ub, lb, Exact_u=None, u_transpose=False, show=True,
                           save_path=None):
    plt = _plt()
    from mpl_toolkits.axes_grid1 import make_axes_locatable
    import matplotlib.gridspec as gridspec
    X, T = np.meshgrid(domain[0], domain[1])
    X_star = np.hstack((X.flatten()[:, None], T.flatten()[:, None]))
    u_pred, _ = model.predict(X_star)
    vals = u_pred.T.flatten() if u_transpose else u_pred.flatten()
    U_pred = vals.reshape(X.shape)  # predictions are on the tensor grid already
    fig, ax = newfig(1.3, 1.0)
    ax.axis("off")
    gs0 = gridspec.GridSpec(1, 2)
    gs0.update(top=1 - 0.06, bottom=1 - 1 / 3, left=0.15, right=0.85, wspace=0)
    ax = plt.subplot(gs0[:, :])
    h = ax.imshow(U_pred.T, interpolation="nearest", cmap="YlGnBu",
                  extent=[lb[1], ub[1], lb[0], ub[0]], origin="lower", aspect="auto")
    cax = make_axes_locatable(ax).append_axes("right", size="5%", pad=0.05)
    fig.colorbar(h, cax=cax)
    q = len(domain[1]) // 4
    line = np.linspace(np.min(domain[0]), np.max(domain[0]), 2)[:, None]
    for k in (1, 2, 3):
        ax.plot(domain[1][k * q] * np.ones((2, 1)), line, "k--", linewidth=1)
    ax.set_xlabel("t")
    ax.set_ylabel("x")
    ax.set_title("u(t,x)", fontsize=10)
    gs1 = gridspec.GridSpec(1, 3)
    gs1.update(top=1 - 1 / 3, bottom=0, left=0.1, right=0.9, wspace=0.5)
    for k in (1, 2, 3):
        ax = plt.subplot(gs1[0, k - 1])
        if Exact_u is not None:
            ax.plot(domain[0], Exact_u[:, k * q], "b-", linewidth=2, label="Exact")
        ax.plot(domain[0], U_pred[k * q, :], "r--", linewidth=2, label="Prediction")
        ax.set_xlabel("x")
        ax.set_ylabel("u(t,x)")
        ax.set_title("t = %.2f" % (domain[1][k * q]), fontsize=10)
        ax.set_xlim([lb[0] - 0.1, ub[0] + 0.1])
        if k == 2:
            ax.legend(loc="upper center", bbox_to_anchor=(0.5, -0.3), ncol=5, frameon=False)
    if save_path:
        fig.savefig(save_path, bbox_inches="tight")
    if show:
        plt.show()
    return fig


def _sa_points_and_weights(model, which=0):
    idx = model.lambdas_map["residual"][which] if hasattr(model, "lambdas_map") else 0
    lam = model.lambdas[idx].detach().cpu().numpy().reshape(-1)
    X = getattr(model, "X_f_local", None)
    if X is None:
        X = model.X
    X = X.detach().cpu().numpy()
    return X, lam


def plot_weights(model, scale=1, show=True, which=0):
    plt = _plt()
    X, lam = _sa_points_and_weights(model, which)
    fig = plt.figure()
    plt.scatter(X[:, -1], X[:, 0], c=lam, s=np.abs(lam) / float(scale))
    plt.colorbar()
    if show:
        plt.show()
    return fig


def plot_glam_values(model, scale=1, show=True, which=0):
    plt = _plt()
    import torch
    X, lam = _sa_points_and_weights(model, which)
    gl = model.g(torch.as_tensor(lam)).numpy() if model.g is not None else lam ** 2
    fig = plt.figure()
    plt.scatter(X[:, -1], X[:, 0], c=gl, s=np.abs(gl) / float(scale))
    plt.colorbar()
    if show:
        plt.show()
    return fig


def plot_residuals(FU_pred, extent, show=True):
    plt = _plt()
    fig, ax = plt.subplots()
    ec = plt.imshow(FU_pred.T, interpolation="nearest", cmap="rainbow", extent=extent,
                    origin="lower", aspect="auto")
    ax.autoscale_view()
    ax.set_xlabel("x")
    ax.set_ylabel("t")
    cbar = plt.colorbar(ec)
    cbar.set_label(r"$\overline{f}_u$ prediction")
    if show:
        plt.show()
    return fig
