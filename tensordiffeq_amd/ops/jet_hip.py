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


def _warg(cfg):
    """The width argument of a kernel entry point: a pointer to the hidden-layer widths for the
    split-bf16 family (any widths, padded to the widest), the single width for exact fp32."""
    if cfg["precision"] in ("bf16x3", "bf16"):
        w = cfg["widths"]
        return (ctypes.c_int * len(w))(*w)
    return cfg["width"]


def _fns(lib, cfg):
    if cfg["precision"] in ("bf16x3", "bf16"):
        return (lib.tdq_jet_fwd_bf3, lib.tdq_jet_bwd_bf3,
                lambda N: lib.tdq_jet_bf3_scratch_floats(N, cfg["d_in"], _warg(cfg), cfg["n_hidden"], cfg["S"],
                                                         *_lo_args(cfg)),
                lambda N: lib.tdq_jet_bf3_slab_floats(N, cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"]))
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


def forward_raw(X, P, net, plan, precision=None, pack=True, rows=None):
    """Autograd-free forward: returns ``(J, saved)`` where ``saved`` feeds :func:`backward_raw`.

    ``precision``: ``"bf16x3"`` / ``"bf16"`` (csrc/jet_bf3.hip, saves post-activations) or ``"fp32"``
    (csrc/jet_mlp.hip, saves pre-activations); the saved buffer only fits its own backward.
    ``pack=False`` (split-bf16 only): the weight images inside the scratch are already current
    (a captured Adam step whose fused tail rewrote them, see :func:`step_tail`).  ``rows``: jet rows
    of ``J`` (default ``plan.S``; more leave room for the high-order streams of ops/jet_hi.py)."""
    lib = _lib.load()
    cfg = hip_config(net, plan, precision)
    if is_layered(cfg):
        from . import jet_layered
        return jet_layered.forward_raw(X.contiguous(), P, net, plan, cfg["precision"])
    fwd, _, scratch_floats, _ = _fns(lib, cfg)
    X = X.contiguous()
    N = X.shape[0]
    S = plan.S
    spec = stream_spec(plan)
    spec_c = (ctypes.c_int * len(spec))(*spec)
    J = torch.empty((max(S, rows or S), N, cfg["d_out"]), dtype=torch.float32, device=X.device)
    nscr = scratch_floats(N)
    if nscr < 0:
        raise ValueError(f"jet kernels cannot serve {cfg}")
    scratch = torch.empty(max(int(nscr), 1), dtype=torch.float32, device=X.device)
    if not pack and cfg["precision"] in ("bf16x3", "bf16"):
        rc = lib.tdq_jet_fwd_bf3_ex(_lib.ptr(X), _lib.ptr(P), _lib.ptr(J), _lib.ptr(scratch), N, cfg["d_in"],
                                    _warg(cfg), cfg["d_out"], cfg["n_hidden"], S, spec_c, *_lo_args(cfg), 0,
                                    _lib.stream_ptr(X.device))
    else:
        rc = fwd(_lib.ptr(X), _lib.ptr(P), _lib.ptr(J), _lib.ptr(scratch), N, cfg["d_in"],
                 _warg(cfg), cfg["d_out"], cfg["n_hidden"], S, spec_c, *_lo_args(cfg), _lib.stream_ptr(X.device))
    _lib.check(rc, f"tdq_jet_fwd[{cfg['precision']}]")
    return J, (X, P, scratch, cfg, spec, S)


def backward_raw(saved, dJ, reduce=True, grad=None):
    """Flat parameter gradient for the adjoint ``dJ`` of the jet.  ``reduce=False`` (split-bf16
    only): launch only the backward kernel and return ``(grad, work)`` - the per-workgroup
    gradient slabs in ``work`` are reduced into ``grad`` later by :func:`step_tail`."""
    if saved[0] == "layered":
        if not reduce:
            raise ValueError("backward_raw(reduce=False) needs the fused split-bf16 kernels")
        from . import jet_layered
        return jet_layered.backward_raw(saved, dJ, grad=grad)
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    _, bwd, _, slab_floats = _fns(lib, cfg)
    N = X.shape[0]
    dJ = dJ.contiguous()
    nwork = slab_floats(N)
    work = torch.empty(max(int(nwork), 1), dtype=torch.float32, device=X.device)
    if grad is None:
        grad = torch.empty_like(P)
    spec_c = (ctypes.c_int * len(spec))(*spec)
    if not reduce:
        if not is_split_bf16(cfg):
            raise ValueError("backward_raw(reduce=False) needs a split-bf16 precision")
        rc = lib.tdq_jet_bwd_bf3_ex(_lib.ptr(X), _lib.ptr(P), _lib.ptr(dJ), _lib.ptr(scratch), _lib.ptr(work),
                                    _lib.ptr(grad), N, cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"],
                                    S, spec_c, *_lo_args(cfg), 0, _lib.stream_ptr(X.device))
        _lib.check(rc, f"tdq_jet_bwd_bf3_ex[{cfg['precision']}]")
        return grad, work
    rc = bwd(_lib.ptr(X), _lib.ptr(P), _lib.ptr(dJ), _lib.ptr(scratch), _lib.ptr(work),
                         _lib.ptr(grad), N, cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"], S,
                         spec_c, *_lo_args(cfg), _lib.stream_ptr(X.device))
    _lib.check(rc, f"tdq_jet_bwd[{cfg['precision']}]")
    return grad


def alloc_forward(X, P, net, plan, precision=None, rows=None):
    """Buffers of a split-bf16 forward over the whole point set, nothing launched: ``(J, saved)``
    for :func:`pack_images`, :func:`forward_range` and :func:`backward_range`."""
    cfg = hip_config(net, plan, precision)
    if not is_split_bf16(cfg):
        raise ValueError("point-range launches need a split-bf16 precision")
    lib = _lib.load()
    _, _, scratch_floats, _ = _fns(lib, cfg)
    X = X.contiguous()
    N = X.shape[0]
    nscr = scratch_floats(N)
    if nscr < 0:
        raise ValueError(f"jet kernels cannot serve {cfg}")
    J = torch.empty((max(plan.S, rows or plan.S), N, cfg["d_out"]), dtype=torch.float32, device=X.device)
    scratch = torch.empty(max(int(nscr), 1), dtype=torch.float32, device=X.device)
    return J, (X, P, scratch, cfg, stream_spec(plan), plan.S)


def forward_range(saved, J, lo, hi):
    """Forward of the points ``[lo, hi)`` (``lo`` a multiple of 128, ``hi`` too or ``N``) into
    the whole-set ``J`` / saved activations, on the current stream; the weight images must be
    packed (:func:`pack_images`)."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    spec_c = (ctypes.c_int * len(spec))(*spec)
    rc = lib.tdq_jet_fwd_bf3_range(_lib.ptr(X), _lib.ptr(P), _lib.ptr(J), _lib.ptr(scratch), X.shape[0], int(lo),
                                   int(hi), cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"], S, spec_c,
                                   *_lo_args(cfg), 0, _lib.stream_ptr(X.device))
    _lib.check(rc, "tdq_jet_fwd_bf3_range")


def alloc_backward(saved):
    """Gradient-slab buffer of the whole point set (see :func:`backward_range`)."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    _, _, _, slab_floats = _fns(lib, cfg)
    return torch.empty(max(int(slab_floats(X.shape[0])), 1), dtype=torch.float32, device=X.device)


def backward_range(saved, dJ, work, lo, hi):
    """Backward of the points ``[lo, hi)``: the gradient slabs of their workgroups in ``work``
    (reduced with the others by :func:`step_tail` / :func:`dp_tail_a`), on the current stream."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    spec_c = (ctypes.c_int * len(spec))(*spec)
    rc = lib.tdq_jet_bwd_bf3_range(_lib.ptr(X), _lib.ptr(dJ), _lib.ptr(scratch), _lib.ptr(work), X.shape[0],
                                   int(lo), int(hi), cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"], S,
                                   spec_c, *_lo_args(cfg), _lib.stream_ptr(X.device))
    _lib.check(rc, "tdq_jet_bwd_bf3_range")


def is_split_bf16(cfg):
    """The fused split-bf16 kernels (csrc/jet_bf3.h) serve this configuration."""
    return cfg["precision"] in ("bf16x3", "bf16") and not is_layered(cfg)


def is_layered(cfg):
    """Hidden width beyond the fused kernels: the layer-wise engine (ops/jet_layered.py)."""
    return cfg.get("engine") == "layered"


def pack_images(saved):
    """Re-pack the weight images of a forward scratch from the current parameters (one launch)."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    rc = lib.tdq_jet_bf3_pack(_lib.ptr(P), _lib.ptr(scratch), X.shape[0], cfg["d_in"], _warg(cfg),
                              cfg["d_out"], cfg["n_hidden"], S, _lib.stream_ptr(X.device))
    _lib.check(rc, "tdq_jet_bf3_pack")


def img_target(saved):
    """The weight-image target of a forward scratch (``csrc`` ``TailImg``: forward / backward A
    images + aux image) as a ctypes buffer: kernels that update the parameters scatter the new
    values into it (the L-BFGS direction kernel), so the next evaluation needs no pack launch."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    buf = ctypes.create_string_buffer(256)
    rc = lib.tdq_img_target(_lib.ptr(scratch), cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"], buf, 256)
    if rc <= 0:
        raise RuntimeError("tdq_img_target: unsupported network")
    return buf


def slab_geometry(cfg, N):
    """``(points per backward workgroup, slab rows, first-pass chunks, rows per chunk)`` of the
    split-bf16 backward over N points (``tdq_bf3_slab_geometry``)."""
    lib = _lib.load()
    out = (ctypes.c_int * 4)()
    rc = lib.tdq_bf3_slab_geometry(int(N), cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"], cfg["S"],
                                   *_lo_args(cfg), out)
    _lib.check(rc, "tdq_bf3_slab_geometry")
    return tuple(out)


def slab_prereduce(saved, work, c0, c1):
    """First-pass chunks ``[c0, c1)`` of the slab reduction on the current stream (the first point
    range's rows, while the second range's backward runs)."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    rc = lib.tdq_slab_prereduce_bf3(_lib.ptr(work), X.shape[0], cfg["d_in"], _warg(cfg), cfg["d_out"],
                                    cfg["n_hidden"], S, *_lo_args(cfg), int(c0), int(c1), _lib.stream_ptr(X.device))
    _lib.check(rc, "tdq_slab_prereduce_bf3")


def step_tail(saved, work, grad, fop, book, counters, group_array, n_groups, snapshot, write_images=True,
              c_first=0, gextra=None, rows=0, lpart=None, n_lblocks=None):
    """End of a single-process Adam step in two launches (csrc/jet_bf3.hip ``tdq_step_tail_bf3``):
    slab reduction + loss reduction + bookkeeping, then the reduced gradient fused into Adam
    (theta, SA weights), the best-weights snapshot and - ``write_images`` - the next step's
    weight images.  ``book``: the engine's device state dict; ``group_array``: ctypes array of
    ``fused._Group`` with theta first; ``c_first``: first-pass chunks below it were pre-reduced
    (:func:`slab_prereduce`); ``gextra``: a gradient added to theta's (the high-order points',
    :class:`~tensordiffeq_amd.ops.jet_hi.HiJetOp`).  ``rows`` / ``lpart`` / ``n_lblocks``: the fused
    step's slab rows and loss-partial rows (:class:`~.fused_step.FusedStepOp`) instead of the
    backward's and the loss kernel's."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    hist = book["hist"]
    carr = (ctypes.c_void_p * max(1, len(counters)))(*[c.data_ptr() for c in counters])
    rc = lib.tdq_step_tail_bf3(
        _lib.ptr(work), _lib.ptr(grad), _lib.ptr(scratch) if write_images else None,
        X.shape[0], cfg["d_in"], _warg(cfg), cfg["d_out"], cfg["n_hidden"], S, *_lo_args(cfg),
        _lib.ptr(fop.partials if lpart is None else lpart), fop.n_blocks if n_lblocks is None else int(n_lblocks),
        fop.n_terms, fop.n_scal,
        _lib.ptr(fop.losses), _lib.ptr(fop.total), _lib.ptr(fop.dscal),
        _lib.ptr(hist), int(hist.shape[0]), _lib.ptr(book["epoch"]), _lib.ptr(book["best_loss"]),
        _lib.ptr(book["best_epoch"]), _lib.ptr(book["improved"]), ctypes.cast(carr, ctypes.c_void_p), len(counters),
        ctypes.cast(group_array, ctypes.c_void_p), n_groups,
        _lib.ptr(snapshot) if snapshot is not None else None, int(c_first), _lib.ptr(gextra), int(rows),
        _lib.stream_ptr(X.device))
    _lib.check(rc, "tdq_step_tail_bf3")


class JetMLPFunction(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, params, net, plan, precision=None):
        J, saved = forward_raw(X, params.contiguous(), net, plan, precision)
        if saved[0] == "layered":
            ctx.layered = saved
            return J
        ctx.layered = None
        ctx.save_for_backward(saved[0], saved[1], saved[2])
        ctx.meta = saved[3:]
        return J

    @staticmethod
    def backward(ctx, dJ):
        if ctx.layered is not None:
            saved = ctx.layered
            if dJ is None:
                dJ = torch.zeros((len(saved[4]) // 3, saved[1].shape[0], saved[3].layer_sizes[-1]),
                                 device=saved[1].device)
            return None, backward_raw(saved, dJ), None, None, None
        X, P, scratch = ctx.saved_tensors
        cfg, spec, S = ctx.meta
        if dJ is None:
            dJ = torch.zeros((S, X.shape[0], cfg["d_out"]), device=X.device)
        return None, backward_raw((X, P, scratch, cfg, spec, S), dJ), None, None, None


def dp_tail_a(saved, work, grad, fop, total=None, losses=None, c_first=0, gextra=None, rows=0, lpart=None,
              n_lblocks=None, half=None):
    """Data-parallel step before the all-reduce: slab pass 1 + loss reduction (one launch), then
    slab pass 2 into ``grad`` (csrc/jet_bf3.hip ``tdq_dp_tail_a_bf3``).  ``total`` (a 1-element
    view): also write the summed loss there; ``losses`` (an ``n_terms`` view, default
    ``fop.losses``): where the per-term losses go - both can point into the all-reduce bucket."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    losses = fop.losses if losses is None else losses
    rc = lib.tdq_dp_tail_a_bf3(_lib.ptr(work), _lib.ptr(grad), X.shape[0], cfg["d_in"], _warg(cfg), cfg["d_out"],
                               cfg["n_hidden"], S, *_lo_args(cfg), _lib.ptr(fop.partials if lpart is None else lpart),
                               fop.n_blocks if n_lblocks is None else int(n_lblocks), fop.n_terms,
                               fop.n_scal, _lib.ptr(losses), _lib.ptr(fop.dscal), _lib.ptr(total), int(c_first),
                               _lib.ptr(gextra), int(rows), -1 if half is None else int(bool(half)),
                               _lib.stream_ptr(X.device))
    _lib.check(rc, "tdq_dp_tail_a_bf3")


def dp_tail_b(saved, group_array, n_groups, improved, snapshot):
    """Data-parallel step after the all-reduce and the bookkeeping: Adam over every group (theta's
    gradient = the all-reduced bucket slice in ``group_array[0].g``), best-weights snapshot and the
    next step's weight images (``tdq_dp_tail_b_bf3``)."""
    lib = _lib.load()
    X, P, scratch, cfg, spec, S = saved
    rc = lib.tdq_dp_tail_b_bf3(_lib.ptr(scratch), X.shape[0], cfg["d_in"], _warg(cfg), cfg["d_out"],
                               cfg["n_hidden"], S, ctypes.cast(group_array, ctypes.c_void_p), n_groups,
                               _lib.ptr(improved), _lib.ptr(snapshot), _lib.stream_ptr(X.device))
    _lib.check(rc, "tdq_dp_tail_b_bf3")
