"""Host side of the high-order jet kernels (``csrc/jet_hi.hip``).

A loss program whose callables need derivatives beyond the fused kernels' order 2 (the reference's
AC-baseline / AC-dist-new periodic BC on u_xxx and u_xxxx, ``examples/AC-baseline.py:23-29``)
keeps every point in the fused step: the fused jet kernels compute the order <= 2 streams of
ALL points, :class:`HiJetOp` computes the extra streams of the few high-order points into extra
rows of the same jet buffer ``J`` (the fused loss reads them like any other stream), and after the
loss the parameter gradient of their adjoints, which the fused step tail adds to theta's gradient.

Stream table (``spec_i`` / ``spec_c``): the high-order plan's streams in canonical order with their
order / variable / output row, then the Faa di Bruno terms of every stream
(``jet.faa_terms``: tanh derivative order, coefficient, factor streams).
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ..jet import faa_terms

MAX_S, MAX_T, MAX_W = 8, 48, 128


def build_spec(plan_hi, out_rows):
    """``(spec_i, spec_c)`` lists for ``plan_hi``; ``out_rows[mi]`` = J row of stream ``mi`` (only the
    streams written / seeded by the kernels).  Raises ValueError outside the kernel's table limits."""
    streams = plan_hi.streams
    S = len(streams)
    if S > MAX_S:
        raise ValueError(f"high-order plan has {S} streams > {MAX_S}")
    idx = plan_hi.index
    order = [len(m) for m in streams]
    if max(order) > 4:
        raise ValueError("derivative order > 4")
    var = [m[0] if len(m) == 1 else 0 for m in streams]
    out = [int(out_rows.get(m, -1)) for m in streams]
    terms, coefs = [], []
    for s, mi in enumerate(streams):
        if s == 0:
            continue
        for k, blocks, c in faa_terms(mi):
            bl = [idx[b] for b in blocks]
            terms.append([s, k, len(bl)] + bl + [0] * (4 - len(bl)))
            coefs.append(float(c))
    if len(terms) > MAX_T:
        raise ValueError(f"{len(terms)} Faa di Bruno terms > {MAX_T}")
    spec_i = [S] + order + var + out + [len(terms)] + [v for t in terms for v in t]
    return spec_i, coefs


def eligible(net, plan_hi):
    """Whether the kernels take this network / high-order plan (split-bf16 MFMA layer GEMMs, widths <= 128)."""
    from ..models.networks import TanhMLP
    if not isinstance(net, TanhMLP):
        return False, "network is not a TanhMLP"
    sizes = net.layer_sizes
    if max(sizes[1:-1]) > MAX_W or sizes[0] > 8 or sizes[-1] > 4 or len(sizes) - 2 > 16:
        return False, "network outside the high-order kernel's envelope"
    try:
        build_spec(plan_hi, {})
    except ValueError as e:
        return False, str(e)
    try:
        lib = _lib.load()
    except _lib.NativeUnavailable:
        lib = None
    if lib is not None and not lib.tdq_jet_hi_lds_ok(len(plan_hi.streams), sizes[0], sizes[-1], len(sizes) - 2):
        return False, "streams x input / output width beyond the high-order kernels' LDS"
    return True, ""


class HiJetOp:
    """Extra (high-order) streams of the points ``[0, n_hi)`` of ``X_all``.

    ``rows``: J rows of the streams the kernels write (and whose adjoints they seed) - the
    high-order streams the fused kernels do not carry.  ``grad``: the parameter gradient of the
    last :meth:`backward` (persistent buffer: captured graphs replay the same pointers)."""

    def __init__(self, net, plan_hi, out_rows, X_all, n_hi, device):
        self.lib = _lib.load(required=True)
        self.net = net
        self.sizes = list(net.layer_sizes)
        self.widths = self.sizes[1:-1]
        self.n_hi = int(n_hi)
        self.X = X_all
        self.ldJ = X_all.shape[0]
        si, sc = build_spec(plan_hi, out_rows)
        self._si = (ctypes.c_int * len(si))(*si)
        self._sc = (ctypes.c_float * max(1, len(sc)))(*sc)
        self._w = (ctypes.c_int * len(self.widths))(*self.widths)
        nz = self.lib.tdq_jet_hi_scratch_floats(self.n_hi, len(self.widths))
        nw = self.lib.tdq_jet_hi_work_floats(self.n_hi, self.sizes[0], self._w, self.sizes[-1], len(self.widths))
        if nz < 0 or nw < 0:
            raise ValueError("high-order jet kernels cannot serve this network")
        self.Z = torch.empty(max(1, int(nz)), dtype=torch.float32, device=device)
        self.work = torch.empty(max(1, int(nw)), dtype=torch.float32, device=device)
        self.grad = torch.zeros(net.flat.numel(), dtype=torch.float32, device=device)

    def _args(self):
        return (self.sizes[0], self._w, self.sizes[-1], len(self.widths), self._si, self._sc)

    def forward(self, J, P):
        """Extra stream rows of ``J`` (``(S_total, N, d_out)``, N = the X_all rows) for the high-order
        points, on the current stream."""
        rc = self.lib.tdq_jet_hi_fwd(_lib.ptr(self.X), self.n_hi, _lib.ptr(P), *self._args(), _lib.ptr(J), self.ldJ, 0,
                                     _lib.ptr(self.Z), _lib.stream_ptr(self.X.device))
        _lib.check(rc, "tdq_jet_hi_fwd")

    def backward(self, dJ, P, part=0):
        """Parameter gradient of the adjoints in the extra rows of ``dJ`` -> :attr:`grad`.  ``part``:
        0 everything; 1 the adjoint chain only; 2 the weight-gradient tiles + reduction only (after a
        part-1 call; ``dJ`` unused) - the halves may run on different graph branches."""
        rc = self.lib.tdq_jet_hi_bwd_part(_lib.ptr(self.X), self.n_hi, _lib.ptr(P), *self._args(), _lib.ptr(dJ),
                                          self.ldJ, 0, _lib.ptr(self.Z), _lib.ptr(self.work), _lib.ptr(self.grad),
                                          int(part), _lib.stream_ptr(self.X.device))
        _lib.check(rc, "tdq_jet_hi_bwd_part")
        return self.grad
