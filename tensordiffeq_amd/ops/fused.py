"""Fused optimizer-side kernels (HIP on GPU, torch reference otherwise).

``adam_multi``  one launch updates every tensor of a step (flat theta, or all SA lambdas with
                ``sign=-1`` for gradient ascent, reference fit.py:136-141) with the Keras Adam
                formula; the bias-corrected step size is computed in-kernel from the device step
                counter, so the launch is graph-capturable.
``best_track``  device-side "keep the best weights" (reference fit.py:51-55 stored an alias of
                the live model, B8): copies the flat buffer to the snapshot iff loss < best.
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
                ("pad", ctypes.c_float)]


def _native(t):
    return t.is_cuda and _lib.available()


def adam_multi(groups, t, lr, b1, b2, eps):
    """groups: list of (param, grad, m, v, sign).  ``t``: float64 device step counter (already +1)."""
    if not groups:
        return
    if _native(groups[0][0]) and all(x.dtype == torch.float32 and x.is_contiguous()
                                     for gr in groups for x in gr[:4]):
        lib = _lib.load()
        for lo in range(0, len(groups), _MAX_GROUPS):
            chunk = groups[lo:lo + _MAX_GROUPS]
            arr = (_Group * len(chunk))()
            for i, (p, g, m, v, sign) in enumerate(chunk):
                arr[i] = _Group(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), p.numel(),
                                float(sign), 0.0)
            rc = lib.tdq_adam_multi(ctypes.cast(arr, ctypes.c_void_p), len(chunk), _lib.ptr(t),
                                    float(lr), float(b1), float(b2), float(eps),
                                    _lib.stream_ptr(p.device))
            _lib.check(rc, "tdq_adam_multi")
        return
    _lib.require_on_gpu() if groups[0][0].is_cuda else None
    with torch.no_grad():
        for (p, g, m, v, sign) in groups:
            torch_update(p, g, m, v, t, lr, b1, b2, eps, sign)


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
