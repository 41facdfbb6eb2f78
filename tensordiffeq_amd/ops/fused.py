"""Fused optimizer-side kernels (HIP on GPU, torch reference otherwise).

``adam_multi``  one launch updates every tensor of a step (flat theta, or all SA lambdas with
                ``sign=-1`` for gradient ascent, reference fit.py:136-141) with the Keras Adam
                formula; the bias-corrected step size is computed in-kernel from the device step
                counter, so the launch is graph-capturable.  ``adam_multi_opts``: the same for
                several optimizers (own counters / hyper-parameters) in ONE launch.
``best_track``  device-side "keep the best weights" (reference fit.py:51-55 stored an alias of
                the live model, B8): copies the flat buffer to the snapshot iff loss < best.
``step_book``   the per-step scalar bookkeeping in one single-thread launch (history row,
                best loss/epoch + "improved" flag, every Adam step counter, epoch); the snapshot
                of the best weights then rides on the Adam launch (``adam_multi(snapshot=...)``).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ..optimizers.adam import torch_update

_MAX_GROUPS = 16


class _Group(ctypes.Structure):
    _fields_ = [("p", ctypes.c_void_p), ("g", ctypes.c_void_p), ("m", ctypes.c_void_p),
                ("v", ctypes.c_void_p), ("n", ctypes.c_int64), ("sign", ctypes.c_float),
                ("lr", ctypes.c_float), ("b1", ctypes.c_float), ("b2", ctypes.c_float),
                ("eps", ctypes.c_float), ("pad", ctypes.c_float), ("t", ctypes.c_void_p)]


def _native(t):
    return t.is_cuda and _lib.available()


def _group_array(flat):
    arr = (_Group * len(flat))()
    for i, (p, g, m, v, sign, t, lr, b1, b2, eps) in enumerate(flat):
        arr[i] = _Group(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                        float(sign), float(lr), float(b1), float(b2), float(eps), 0.0, t.data_ptr())
    return arr


def flatten_opt_groups(opt_groups):
    """``[(groups, t, lr, b1, b2, eps), ...]`` -> one row per tensor."""
    return [(p, g, m, v, sign, t, lr, b1, b2, eps)
            for groups, t, lr, b1, b2, eps in opt_groups for (p, g, m, v, sign) in groups]


def group_array(opt_groups):
    """ctypes ``AdamGroup`` array (csrc/optim_common.h) for ONE launch, or ``None`` when the
    tensors do not fit it (more than 16, or not contiguous float32)."""
    flat = flatten_opt_groups(opt_groups)
    if not flat or len(flat) > _MAX_GROUPS or not all(
            x.dtype == torch.float32 and x.is_contiguous() for gr in flat for x in gr[:4]):
        return None
    return _group_array(flat), len(flat)


def adam_multi(groups, t, lr, b1, b2, eps, snapshot=None):
    """groups: list of (param, grad, m, v, sign) sharing one optimizer.  ``t``: float64 device step
    counter (already +1).  ``snapshot=(best, improved)``: copy group 0's parameters into ``best``
    before the update when the int32 device flag ``improved`` is set."""
    adam_multi_opts([(groups, t, lr, b1, b2, eps)], snapshot)


def adam_multi_opts(opt_groups, snapshot=None):
    """One launch for several optimizers: ``opt_groups`` = list of ``(groups, t, lr, b1, b2, eps)``
    (e.g. Adam descent on theta and Adam ascent on the SA weights, each with its own step
    counter and hyper-parameters).  ``snapshot`` applies to the first tensor of the first group."""
    flat = flatten_opt_groups(opt_groups)
    if not flat:
        return
    if snapshot is not None and snapshot[0].numel() != flat[0][0].numel():
        # the kernel copies group 0's parameters into the snapshot buffer: a stale (smaller)
        # snapshot would be an out-of-bounds device write
        raise ValueError(f"best-weights snapshot has {snapshot[0].numel()} elements, parameters "
                         f"{flat[0][0].numel()}")
    if _native(flat[0][0]) and all(x.dtype == torch.float32 and x.is_contiguous()
                                   for gr in flat for x in gr[:4]):
        lib = _lib.load()
        for lo in range(0, len(flat), _MAX_GROUPS):
            chunk = flat[lo:lo + _MAX_GROUPS]
            snap = snapshot if lo == 0 else None
            arr = _group_array(chunk)
            rc = lib.tdq_adam_multi(ctypes.cast(arr, ctypes.c_void_p), len(chunk),
                                    _lib.ptr(snap[1]) if snap else None, _lib.ptr(snap[0]) if snap else None,
                                    _lib.stream_ptr(flat[0][0].device))
            _lib.check(rc, "tdq_adam_multi")
        return
    _lib.require_on_gpu() if flat[0][0].is_cuda else None
    with torch.no_grad():
        if snapshot is not None:
            best, improved = snapshot
            best.copy_(torch.where(improved.bool(), flat[0][0], best))
        for (p, g, m, v, sign, t, lr, b1, b2, eps) in flat:
            torch_update(p, g, m, v, t, lr, b1, b2, eps, sign)


def step_book(loss, terms, state, counters, sum_terms=False):
    """Per-step bookkeeping on device (see module doc).  ``terms``: contiguous float32 vector.
    ``sum_terms``: the loss buffer is (over)written with the sum of ``terms`` first (fused loss)."""
    hist = state["hist"]
    if _native(hist):
        lib = _lib.load()
        arr = (ctypes.c_void_p * max(1, len(counters)))(*[c.data_ptr() for c in counters])
        rc = lib.tdq_step_book(_lib.ptr(loss), _lib.ptr(terms) if terms.numel() else None, int(terms.numel()),
                               int(bool(sum_terms)),
                               _lib.ptr(hist), int(hist.shape[0]), _lib.ptr(state["epoch"]),
                               _lib.ptr(state["best_loss"]), _lib.ptr(state["best_epoch"]),
                               _lib.ptr(state["improved"]), ctypes.cast(arr, ctypes.c_void_p), len(counters),
                               _lib.stream_ptr(hist.device))
        _lib.check(rc, "tdq_step_book")
        return
    if hist.is_cuda:
        _lib.require_on_gpu()
    with torch.no_grad():
        ep = state["epoch"]
        if sum_terms:
            s = torch.zeros((), device=terms.device)
            for t in terms.reshape(-1):
                s = s + t
            loss.copy_(s.reshape(loss.shape))
        lv = loss.reshape(()).float()
        row = torch.cat([lv.reshape(1), terms.reshape(-1).float()])
        hist.index_copy_(0, ep.reshape(1), row.unsqueeze(0))
        imp = lv < state["best_loss"]
        state["improved"].copy_(imp.to(state["improved"].dtype))
        state["best_epoch"].copy_(torch.where(imp, ep, state["best_epoch"]))
        state["best_loss"].copy_(torch.where(imp, lv, state["best_loss"]))
        for c in counters:
            c.add_(1.0)
        ep.add_(1)


def best_track(loss, best_loss, flat, best_flat, best_epoch, epoch):
    """if loss < best_loss: best_flat <- flat, best_loss <- loss, best_epoch <- epoch (on device)."""
    if _native(flat):
        lib = _lib.load()
        rc = lib.tdq_best_track(_lib.ptr(loss.reshape(1).float().contiguous()), _lib.ptr(best_loss),
                                _lib.ptr(flat), _lib.ptr(best_flat), _lib.ptr(best_epoch),
                                _lib.ptr(epoch), flat.numel(), _lib.stream_ptr(flat.device))
        _lib.check(rc, "tdq_best_track")
        return
    if flat.is_cuda:
        _lib.require_on_gpu()
    with torch.no_grad():
        improved = loss.reshape(()).to(best_loss.dtype) < best_loss
        best_flat.copy_(torch.where(improved, flat, best_flat))
        best_epoch.copy_(torch.where(improved, epoch, best_epoch))
        best_loss.copy_(torch.where(improved, loss.reshape(()).to(best_loss.dtype), best_loss))
