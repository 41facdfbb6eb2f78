"""Forward-mode Taylor jets through a tanh MLP (pure-torch engine + stream planning).

Replaces the reference's nested reverse-mode ``tf.gradients`` by
propagating derivative *streams* alongside the value: for a multi-index ``mi`` (sorted tuple of
input-variable indices, e.g. ``(0, 0)`` = d2/dx2) every layer carries ``z_mi``.  Linear layers map
every stream with the same weights (bias only on the value stream); tanh maps them with
Faa di Bruno's formula over set partitions of the multi-index positions::

    d_mi tanh(z) = sum_{partitions P of mi} tanh^(|P|)(z) * prod_{B in P} z_B

where ``tanh^(k)`` is a polynomial in ``h = tanh(z)`` (``P_{k+1}(h) = P_k'(h) (1 - h^2)``).
The input layer is exact: ``z_(i) = W1[i, :]`` and every order >= 2 stream is 0.

This module is the numerical reference for the HIP jet kernels (:mod:`.ops.jet_mlp`), and the
backend used on CPU and for stream sets the kernels do not cover.
"""
from __future__ import annotations

import itertools
from functools import lru_cache

import torch

MAX_ORDER = 4


def closure(requests):
    """All sub-multisets of every requested multi-index, plus the value stream; canonical order."""
    out = {()}
    for mi in requests:
        mi = tuple(sorted(mi))
        for r in range(1, len(mi) + 1):
            for comb in itertools.combinations(mi, r):
                out.add(tuple(sorted(comb)))
    return sorted(out, key=lambda m: (len(m), m))


def _set_partitions(items):
    if not items:
        yield []
        return
    first, rest = items[0], items[1:]
    for part in _set_partitions(rest):
        yield [[first]] + part
        for i in range(len(part)):
            yield part[:i] + [[first] + part[i]] + part[i + 1:]


@lru_cache(maxsize=None)
def faa_terms(mi):
    """{(k, (block_mi, ...)): integer coefficient} for d_mi tanh(z)."""
    terms = {}
    for part in _set_partitions(list(range(len(mi)))):
        blocks = tuple(sorted(tuple(sorted(mi[p] for p in b)) for b in part))
        key = (len(part), blocks)
        terms[key] = terms.get(key, 0) + 1
    return tuple((k, blocks, c) for (k, blocks), c in sorted(terms.items()))


@lru_cache(maxsize=None)
def tanh_poly(k):
    """Coefficients (ascending powers of h) of d^k tanh / dz^k as a polynomial in h."""
    p = [0.0, 1.0]  # tanh itself: h
    for _ in range(k):
        dp = [i * p[i] for i in range(1, len(p))] or [0.0]
        # multiply by (1 - h^2)
        q = [0.0] * (len(dp) + 2)
        for i, c in enumerate(dp):
            q[i] += c
            q[i + 2] -= c
        while len(q) > 1 and q[-1] == 0.0:
            q.pop()
        p = q
    return tuple(p)


def tanh_derivs(h, kmax):
    """[h, tanh', tanh'', ...] up to order kmax evaluated from h."""
    out = [h]
    for k in range(1, kmax + 1):
        coeffs = tanh_poly(k)
        acc = torch.zeros_like(h) + coeffs[-1]
        for c in reversed(coeffs[:-1]):
            acc = acc * h + c
        out.append(acc)
    return out


class JetPlan:
    """Stream set for one evaluation: ``streams[0] == ()`` then by (order, multi-index)."""

    def __init__(self, requests, d_in):
        self.streams = closure(requests)
        self.index = {m: i for i, m in enumerate(self.streams)}
        self.order = max(len(m) for m in self.streams)
        self.d_in = d_in
        if any(v >= d_in for m in self.streams for v in m):
            raise ValueError("multi-index refers to a variable beyond the network input width")

    @property
    def S(self):
        return len(self.streams)

    def hip_supported(self):
        return self.order <= 2

    def __repr__(self):
        return f"JetPlan(streams={self.streams})"


def jet_forward(X, weights, plan):
    """Evaluate the jet.  ``weights``: list of ``(kernel (in,out), bias (out,))`` per dense layer.

    Returns a tensor ``J`` of shape ``(S, N, d_out)`` (stream-major), differentiable w.r.t. the
    weights through ordinary autograd.
    """
    streams = plan.streams
    N = X.shape[0]
    (K1, b1) = weights[0]
    z = {(): torch.addmm(b1, X, K1)}
    for mi in streams[1:]:
        if len(mi) == 1:
            z[mi] = K1[mi[0]].unsqueeze(0).expand(N, -1)
        else:
            z[mi] = None  # identically zero
    for (K, b) in weights[1:]:
        h = _tanh_jet(z, streams, plan.order)
        z = {}
        for mi in streams:
            hm = h[mi]
            if hm is None:
                z[mi] = None
            elif mi == ():
                z[mi] = torch.addmm(b, hm, K)
            else:
                z[mi] = hm @ K
    d_out = weights[-1][0].shape[1]
    out = [z[mi] if z[mi] is not None else X.new_zeros(N, d_out) for mi in streams]
    out = [o if o.shape[0] == N else o.expand(N, -1) for o in out]
    return torch.stack(out, dim=0)


def _tanh_jet(z, streams, order):
    h0 = torch.tanh(z[()])
    s = tanh_derivs(h0, order)
    h = {(): h0}
    for mi in streams[1:]:
        acc = None
        for (k, blocks, c) in faa_terms(mi):
            prod = None
            zero = False
            for blk in blocks:
                zb = z[blk]
                if zb is None:
                    zero = True
                    break
                prod = zb if prod is None else prod * zb
            if zero:
                continue
            term = s[k] * prod
            if c != 1:
                term = term * float(c)
            acc = term if acc is None else acc + term
        h[mi] = acc
    return h


def jet_dict(J, plan):
    return {mi: J[i] for i, mi in enumerate(plan.streams)}
