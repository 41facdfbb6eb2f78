"""Checkpoints: weights (+ optional full training state) with a Keras-layout export.

Reference (models.py:315-319, examples/transfer-learn.py:56-72): ``u_model.save(path)`` writes a
Keras SavedModel/HDF5 - weights only, no SA weights, optimizer slots or epoch - and
``load_model`` replaces ``u_model``.

Here ``save(path)`` writes

* ``path`` ending in ``.npz``:  Keras-layout arrays only (``dense/kernel:0`` (in,out),
  ``dense/bias:0``, ``dense_1/kernel:0``, ...) + ``__layer_sizes__`` - interchangeable with the
  reference's per-layer ``get_weights()`` lists;
* ``path`` ending in ``.pt``:   torch file with the flat parameters, layer sizes and (if
  ``include_state``) SA lambdas (gathered across DP ranks), Adam moments/step counters, epoch
  counter and best-weights snapshot - everything needed to resume training exactly;
* anything else: a directory containing both (``model.pt`` and ``keras_weights.npz``) plus
  ``config.json``.

Loading uses only non-executing loaders (``torch.load(weights_only=True)``,
``numpy.load(allow_pickle=False)``).
"""
from __future__ import annotations

import json
import os

import numpy as np
import torch

from .models.networks import TanhMLP, layer_offsets


def keras_arrays(net, flat=None):
    flat = (net.flat if flat is None else flat).detach().cpu().numpy()
    out = {}
    for i, (wo, bo, fi, fo) in enumerate(net.offsets):
        name = "dense" if i == 0 else f"dense_{i}"
        out[f"{name}/kernel:0"] = flat[wo:bo].reshape(fi, fo).copy()
        out[f"{name}/bias:0"] = flat[bo:bo + fo].copy()
    out["__layer_sizes__"] = np.asarray(net.layer_sizes, dtype=np.int64)
    return out


def flat_from_keras(arrays, layer_sizes=None):
    if layer_sizes is None:
        layer_sizes = [int(x) for x in arrays["__layer_sizes__"]]
    offs, n = layer_offsets(layer_sizes)
    flat = np.zeros(n, dtype=np.float32)
    for i, (wo, bo, fi, fo) in enumerate(offs):
        name = "dense" if i == 0 else f"dense_{i}"
        flat[wo:bo] = np.asarray(arrays[f"{name}/kernel:0"], dtype=np.float32).reshape(-1)
        flat[bo:bo + fo] = np.asarray(arrays[f"{name}/bias:0"], dtype=np.float32).reshape(-1)
    return flat, list(layer_sizes)


def _gather_rows(t, ctx):
    """Concatenate a row-sharded tensor across DP ranks (rank order)."""
    if not ctx.is_distributed:
        return t
    import torch.distributed as dist
    n = torch.tensor([t.shape[0]], device=ctx.device)
    sizes = [torch.zeros_like(n) for _ in range(ctx.world)]
    dist.all_gather(sizes, n)
    m = int(max(int(s) for s in sizes))
    pad = torch.zeros((m,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[: t.shape[0]] = t
    parts = [torch.zeros_like(pad) for _ in range(ctx.world)]
    dist.all_gather(parts, pad.contiguous())
    return torch.cat([p[: int(s)] for p, s in zip(parts, sizes)], dim=0)


def solver_state(solver, include_state=True):
    net = solver.u_model
    st = {"format": "tensordiffeq_amd/1", "layer_sizes": list(net.layer_sizes),
          "flat": net.flat.detach().cpu()}
    if include_state:
        ctx = solver.dist_ctx
        lams = []
        for lam, rep in zip(solver.lambdas or [], solver._lam_replicated() if solver.lambdas else []):
            lams.append((lam if rep else _gather_rows(lam, ctx)).detach().cpu())
        st["lambdas"] = lams
        st["lambdas_map"] = json.dumps(solver.lambdas_map or {})
        reps_lam = solver._lam_replicated() if solver.lambdas else []
        for key, opt, tensors, reps in (("opt_theta", solver.tf_optimizer, [net.flat], [True]),
                                        ("opt_lam", solver.tf_optimizer_weights, solver.lambdas or [],
                                         reps_lam)):
            m, v = [], []
            for tt, rep in zip(tensors, reps):
                mm, vv = opt.state_for(tt)
                m.append((mm if rep else _gather_rows(mm, ctx)).detach().cpu())
                v.append((vv if rep else _gather_rows(vv, ctx)).detach().cpu())
            st[key] = {"m": m, "v": v, "t": float(0 if opt._t is None else opt._t.item()),
                       "hyper": [opt.learning_rate, opt.beta_1, opt.beta_2, opt.epsilon]}
        s = solver._state
        if s is not None:
            st["epoch"] = int(s["epoch_host"])
            st["best_flat"] = s["best_flat"].detach().cpu()
            st["best_loss"] = float(s["best_loss"])
            st["best_epoch"] = int(s["best_epoch"])
    return st


def save_solver(solver, path, include_state=True):
    path = str(path)
    ctx = solver.dist_ctx
    st = solver_state(solver, include_state) if path.endswith(".pt") or not path.endswith(".npz") else None
    if ctx.rank != 0:
        return
    if path.endswith(".npz"):
        np.savez(path, **keras_arrays(solver.u_model))
        return
    if path.endswith(".pt"):
        torch.save(st, path)
        return
    os.makedirs(path, exist_ok=True)
    torch.save(st, os.path.join(path, "model.pt"))
    np.savez(os.path.join(path, "keras_weights.npz"), **keras_arrays(solver.u_model))
    with open(os.path.join(path, "config.json"), "w") as f:
        json.dump({"layer_sizes": list(solver.u_model.layer_sizes), "activation": "tanh",
                   "format": "tensordiffeq_amd/1"}, f)


def load_state(path):
    path = str(path)
    if os.path.isdir(path):
        pt = os.path.join(path, "model.pt")
        if os.path.exists(pt):
            return torch.load(pt, map_location="cpu", weights_only=True)
        path = os.path.join(path, "keras_weights.npz")
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            arrays = {k: z[k] for k in z.files}
        flat, sizes = flat_from_keras(arrays)
        return {"layer_sizes": sizes, "flat": torch.from_numpy(flat)}
    return torch.load(path, map_location="cpu", weights_only=True)


def load_into_solver(solver, path, restore_state=False):
    """Replace the network weights (reference ``load_model``: weights only).  With
    ``restore_state=True`` also restore SA weights, Adam moments/step counters, epoch and the
    best-weights snapshot when the checkpoint has them and the problem matches (exact resume)."""
    st = load_state(path)
    sizes = list(st["layer_sizes"])
    net = solver.u_model if isinstance(getattr(solver, "u_model", None), TanhMLP) else None
    if net is None or list(net.layer_sizes) != sizes:
        net = TanhMLP(sizes, device=solver.device)
        solver.u_model = net
    with torch.no_grad():
        net.flat.copy_(st["flat"].to(net.flat.device))
    if not restore_state or "lambdas" not in st:
        return
    ctx = solver.dist_ctx
    lams = st["lambdas"]
    if solver.lambdas and len(lams) == len(solver.lambdas):
        reps = solver._lam_replicated()
        for cur, saved, rep in zip(solver.lambdas, lams, reps):
            src = saved if rep else saved.reshape(-1, 1)[solver._lo:solver._hi]
            if src.numel() == cur.numel():
                cur.data.copy_(src.reshape(cur.shape).to(cur.device))
        for key, opt, tensors in (("opt_lam", solver.tf_optimizer_weights, solver.lambdas),):
            if key in st:
                for tt, mm, vv, rep in zip(tensors, st[key]["m"], st[key]["v"], reps):
                    m, v = opt.state_for(tt)
                    sm = mm if rep else mm.reshape(-1, 1)[solver._lo:solver._hi]
                    sv = vv if rep else vv.reshape(-1, 1)[solver._lo:solver._hi]
                    if sm.numel() == m.numel():
                        m.copy_(sm.reshape(m.shape).to(m.device))
                        v.copy_(sv.reshape(v.shape).to(v.device))
                opt.step_counter(solver.device).fill_(st[key]["t"])
    if "opt_theta" in st:
        m, v = solver.tf_optimizer.state_for(net.flat)
        m.copy_(st["opt_theta"]["m"][0].to(m.device))
        v.copy_(st["opt_theta"]["v"][0].to(v.device))
        solver.tf_optimizer.step_counter(solver.device).fill_(st["opt_theta"]["t"])
    if "epoch" in st:
        s = solver._train_state(solver.device)
        s["epoch_host"] = st["epoch"]
        s["epoch"].fill_(st["epoch"])
        s["best_flat"].copy_(st["best_flat"].to(s["best_flat"].device))
        s["best_loss"].fill_(st["best_loss"])
        s["best_epoch"].fill_(st["best_epoch"])
    del ctx
