"""torch.autograd binding of the HIP jet kernels (``csrc/jet_mlp.hip``).

Forward: ``tdq_jet_fwd`` -> J (S, N, d_out) + scratch (saved pre-activation streams).
Backward: ``tdq_jet_bwd`` -> flat parameter gradient (per-workgroup slabs, deterministic
two-pass reduction).  Buffers are allocated with torch so they come from the caching
allocator (and from the private pool while a HIP graph is being captured).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from .jet_mlp import hip_config


def stream_spec(plan):
    """3 ints per stream: (type, a, b) - see ``make_spec`` in jet_mlp.hip."""
    idx = plan.index
    out = []
    for mi in plan.streams:
        if len(mi) == 0:
            out += [0, 0, 0]
        elif len(mi) == 1:
            out += [1, mi[0], 0]
        else:
            out += [2, idx[(mi[0],)], idx[(mi[1],)]]
    return out


def _fns(lib, cfg):
    if cfg["precision"] in ("bf16x3", "bf16"):
        return (lib.tdq_jet_fwd_bf3, lib.tdq_jet_bwd_bf3,
                lambda N: lib.tdq_jet_bf3_scratch_floats(N, cfg["d_in"], cfg["width"], cfg["n_hidden"], cfg["S"]),
                lambda N: lib.tdq_jet_bf3_slab_floats(N, cfg["d_in"], cfg["width"], cfg["d_out"], cfg["n_hidden"]))
    return (lib.tdq_jet_fwd, lib.tdq_jet_bwd,
            lambda N: lib.tdq_jet_scratch_floats(N, cfg["width"], cfg["n_hidden"], cfg["S"], 0),
            lambda N: lib.tdq_jet_slab_floats(N, cfg["d_in"], cfg["width"], cfg["d_out"], cfg["n_hidden"]))


def _lo_args(cfg):
    """Trailing kernel flag of the split-bf16 family: 1 = bf16x3, 0 = bf16."""
    if cfg["precision"] == "bf16x3":
        return (1,)
    if cfg["precision"] == "bf16":
        return (0,)
    return ()


def forward_raw(X, P, net, plan, precision=None):
    """Autograd-free forward: returns ``(J, saved)`` where ``saved`` feeds :func:`backward_raw`.

    ``precision``: ``"bf16x3"`` / ``"bf16"`` (csrc/jet_bf3.hip, saves post-activations) or ``"fp32"``
    (csrc/jet_mlp.hip, saves pre-activations); the saved buffer only fits its own backward."""
    lib = _lib.load()
    cfg = hip_config(net, plan, precision)
    fwd, _, scratch_floats, _ = _fns(lib, cfg)
    X = X.contiguous()
    N = X.shape[0]
    S = plan.S
    spec = stream_spec(plan)
    spec_c = (ctypes.c_int * len(spec))(*spec)
    J = torch.empty((S, N, cfg["d_out"]), dtype=torch.float32, device=X.device)
    nscr = scratch_floats(N)
    if nscr < 0:
        raise ValueError(f"jet kernels cannot serve {cfg}")
    scratch = torch.empty(max(int(nscr), 1), dtype=torch.float32, device=X.device)
    rc = fwd(_lib.ptr(X), _lib.ptr(P), _lib.ptr(J), _lib.ptr(scratch), N, cfg["d_in"],
                         cfg["width"], cfg["d_out"], cfg["n_hidden"], S, spec_c, *_lo_args(cfg), _lib.stream_ptr(X.device))
    _lib.check(rc, f"tdq_jet_fwd[{cfg['precision']}]")
    return J, (X, P, scratch, cfg, spec, S)


def backward_raw(saved, dJ):
    """Flat parameter gradient for the adjoint ``dJ`` of the jet."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    _, bwd, _, slab_floats = _fns(lib, cfg)
    N = X.shape[0]
    dJ = dJ.contiguous()
    nwork = slab_floats(N)
    work = torch.empty(max(int(nwork), 1), dtype=torch.float32, device=X.device)
    grad = torch.empty_like(P)
    spec_c = (ctypes.c_int * len(spec))(*spec)
    rc = bwd(_lib.ptr(X), _lib.ptr(P), _lib.ptr(dJ), _lib.ptr(scratch), _lib.ptr(work),
                         _lib.ptr(grad), N, cfg["d_in"], cfg["width"], cfg["d_out"], cfg["n_hidden"], S,
                         spec_c, *_lo_args(cfg), _lib.stream_ptr(X.device))
    _lib.check(rc, f"tdq_jet_bwd[{cfg['precision']}]")
    return grad


class JetMLPFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, params, net, plan, precision=None):
        J, saved = forward_raw(X, params.contiguous(), net, plan, precision)
        ctx.save_for_backward(saved[0], saved[1], saved[2])
        ctx.meta = saved[3:]
        return J

    @staticmethod
    def backward(ctx, dJ):
        X, P, scratch = ctx.saved_tensors
        cfg, spec, S = ctx.meta
        if dJ is None:
            dJ = torch.zeros((S, X.shape[0], cfg["d_out"]), device=X.device)
        return None, backward_raw((X, P, scratch, cfg, spec, S), dJ), None, None, None
