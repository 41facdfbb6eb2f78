"""Derivative API for user PDE callables and the planning / jet execution contexts.

Users write residuals the way the reference does with ``tf.gradients`` (reference call sites:
examples/AC-SA.py:36-44, examples/burgers-new.py:26-32, examples/steady-state.py:19-40)::

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x); u_xx = tdq.grad(u_x, x); u_t = tdq.grad(u, t)
        return u_t - 1e-4 * u_xx + 5 * u**3 - 5 * u

``tdq.grad`` is context dependent:

* no context (plain / generic backend): nested ``torch.autograd.grad`` with ``create_graph`` -
  works for any network and any derivative order, this is the correctness oracle.
* :class:`RecordContext` (one-off planning pass on a handful of points): runs real autograd *and*
  records which derivative multi-indices of the network output are requested.  If every request
  is a derivative of the network output w.r.t. one of the coordinate columns, the callable is
  "jet-able" and its stream set is the closure of the requests.
* :class:`JetContext` (fast path): ``u_model(...)`` returns the precomputed jet value stream and
  ``tdq.grad`` returns the precomputed derivative stream, so the residual costs only elementwise
  torch ops on top of one fused jet evaluation (torch or HIP kernels, :mod:`.ops.jet_mlp`).
"""
from __future__ import annotations

import threading

import torch

_TLS = threading.local()


class JetMiss(RuntimeError):
    """A derivative stream was requested that the current jet plan did not compute."""


class NotJetable(RuntimeError):
    pass


def _current():
    return getattr(_TLS, "ctx", None)


class _use:
    def __init__(self, ctx):
        self.ctx = ctx

    def __enter__(self):
        self.prev = _current()
        _TLS.ctx = self.ctx
        return self.ctx

    def __exit__(self, *exc):
        _TLS.ctx = self.prev
        return False


def _unwrap(y):
    while isinstance(y, (list, tuple)):
        if len(y) != 1:
            raise ValueError("grad() expects a single tensor")
        y = y[0]
    return y


def grad(y, x):
    """dy/dx per point (sum over network outputs when y has several columns, like tf.gradients)."""
    y = _unwrap(y)
    x = _unwrap(x)
    ctx = _current()
    if ctx is not None:
        return ctx.grad(y, x)
    return _autograd(y, x)


def gradients(ys, xs):
    """TF-style: returns a one-element list."""
    return [grad(ys, xs)]


def _autograd(y, x):
    # d(sum y)/dx == the VJP with ones (each point's outputs depend on its own coordinates only).
    # A scalar output also keeps torch.autograd.grad off its grad_outputs check, whose first call
    # imports torch.fx.experimental.symbolic_shapes (sympy): ~0.8 s of every program build on the
    # GPU box (tools/prof_program.py).
    g = torch.autograd.grad(y.sum(), x, create_graph=True, allow_unused=True)[0]
    if g is None:
        g = torch.zeros_like(x)
    return g


class _Ctx:
    def __init__(self, columns):
        self.var_of = {id(c): i for i, c in enumerate(columns)}
        self._reg = {}
        self._keep = []

    def register(self, t, mi, summed):
        self._reg[id(t)] = (tuple(mi), bool(summed))
        self._keep.append(t)

    def lookup(self, t):
        return self._reg.get(id(t))


class RecordContext(_Ctx):
    """Planning pass: real autograd on leaf columns + request recording."""

    def __init__(self, columns, model):
        super().__init__(columns)
        self.columns = columns
        self.model = model
        self.requests = set()
        self.jetable = True
        self.reasons = []
        self.d_out = None
        self._full = torch.cat([c.detach() for c in columns], dim=1)

    def proxy(self):
        def u_model(*args, **kw):
            out = self.model(*args, **kw)
            inp = args[0] if len(args) == 1 else torch.cat(args, dim=1)
            if kw or inp.shape != self._full.shape or not torch.equal(inp.detach(), self._full):
                self.jetable = False
                self.reasons.append("u_model called on inputs other than the coordinate columns")
            self.d_out = out.shape[1]
            self.register(out, (), False)
            return out
        return u_model

    def grad(self, y, x):
        g = _autograd(y, x)
        info = self.lookup(y)
        var = self.var_of.get(id(x))
        if info is None or var is None:
            self.jetable = False
            self.reasons.append("grad() of a tensor that is not a derivative stream of u_model")
            return g
        mi, summed = info
        mi2 = tuple(sorted(mi + (var,)))
        summed = summed or (self.d_out or 1) > 1
        self.register(g, mi2, summed)
        self.requests.add(mi2)
        return g


class JetContext(_Ctx):
    """Fast-path execution: serve u and its derivatives from a precomputed jet."""

    def __init__(self, columns, jet):
        super().__init__(columns)
        self.jet = jet  # dict: multi-index tuple -> (n, d_out) tensor

    def proxy(self):
        def u_model(*args, **kw):
            out = self.jet[()]
            self.register(out, (), False)
            return out
        return u_model

    def grad(self, y, x):
        info = self.lookup(y)
        var = self.var_of.get(id(x))
        if info is None or var is None:
            raise NotJetable("grad() of a tensor that is not a derivative stream of u_model")
        mi, summed = info
        mi2 = tuple(sorted(mi + (var,)))
        t = self.jet.get(mi2)
        if t is None:
            raise JetMiss(str(mi2))
        if summed or t.shape[1] > 1:
            t = t.sum(dim=1, keepdim=True)
            summed = True
        self.register(t, mi2, summed)
        return t


def use(ctx):
    return _use(ctx)


def record_callable(fn, model, points, extra_args=()):
    """Run ``fn(u_model_proxy, *extra_args, *columns)`` under a RecordContext on ``points``.

    Returns ``(requests, jetable, reasons, d_out)``.
    """
    cols = [points[:, j:j + 1].detach().clone().requires_grad_(True) for j in range(points.shape[1])]
    ctx = RecordContext(cols, model)
    with use(ctx):
        try:
            fn(ctx.proxy(), *extra_args, *cols)
        except (NotJetable, JetMiss) as e:  # pragma: no cover - defensive
            ctx.jetable = False
            ctx.reasons.append(str(e))
    return ctx.requests, ctx.jetable, ctx.reasons, ctx.d_out
