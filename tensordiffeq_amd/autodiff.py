"""Derivative API for user PDE callables and the planning / jet execution contexts.

Users write residuals the way the reference does with ``tf.gradients`` (reference call sites:
examples/AC-SA.py:36-44, examples/burgers-new.py:26-32, examples/steady-state.py:19-40)::

    def f_model(u_model, x, t):
        u = u_model(torch.cat([x, t], 1))
        u_x = tdq.grad(u, x); u_xx = tdq.grad(u_x, x); u_t = tdq.grad(u, t)
        return u_t - 1e-4 * u_xx + 5 * u**3 - 5 * u

``torch.autograd.grad(u, x, grad_outputs=torch.ones_like(u), create_graph=True)`` - the natural
PyTorch spelling of the reference's ``tf.gradients(u, x)`` (examples/burgers-new.py:26-32) - is
served the same way: while a planning / jet / trace context is active, ``torch.autograd.grad`` is
routed through :func:`_routed_autograd_grad`, which hands calls of the form "derivative stream of
u_model w.r.t. coordinate columns, unit cotangent" to the context (like ``tdq.grad``) and passes
every other call through to torch.  The planning pass checks the cotangent really is all ones, and
``LossProgram`` re-runs every jet-planned callable in a :class:`JetContext` on the probe points and
falls back to the autograd backend on any exception or mismatch.

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


_ORIG_AUTOGRAD_GRAD = torch.autograd.grad
_PATCH_LOCK = threading.Lock()
_PATCH_DEPTH = 0


def _as_seq(v):
    if v is None:
        return None
    return list(v) if isinstance(v, (list, tuple)) else [v]


def _routed_autograd_grad(outputs, inputs, grad_outputs=None, retain_graph=None, create_graph=False,
                          only_inputs=True, allow_unused=None, is_grads_batched=False,
                          materialize_grads=False):
    """``torch.autograd.grad`` while a derivative context is active (see module docstring)."""
    ctx = _current()
    ys, xs, gos = _as_seq(outputs), _as_seq(inputs), _as_seq(grad_outputs)
    if ctx is not None and ys is not None and len(ys) == 1 and xs and not is_grads_batched \
            and ctx.lookup(ys[0]) is not None and all(ctx.var_of.get(id(x)) is not None for x in xs) \
            and (gos is None or len(gos) == 1):
        go = gos[0] if gos is not None else None
        if ctx.accepts_cotangent(ys[0], go):
            return tuple(ctx.grad(ys[0], x) for x in xs)
    kw = dict(grad_outputs=grad_outputs, retain_graph=retain_graph, create_graph=create_graph,
              only_inputs=only_inputs, allow_unused=allow_unused, is_grads_batched=is_grads_batched)
    if materialize_grads:
        kw["materialize_grads"] = True
    if ctx is not None and isinstance(ctx, RecordContext):
        ctx.note_foreign_grad(ys, xs)
    return _ORIG_AUTOGRAD_GRAD(outputs, inputs, **kw)


class _use:
    """Activate a derivative context (and route ``torch.autograd.grad`` through it)."""

    def __init__(self, ctx):
        self.ctx = ctx

    def __enter__(self):
        global _PATCH_DEPTH
        self.prev = _current()
        _TLS.ctx = self.ctx
        with _PATCH_LOCK:
            if _PATCH_DEPTH == 0:
                torch.autograd.grad = _routed_autograd_grad
            _PATCH_DEPTH += 1
        return self.ctx

    def __exit__(self, *exc):
        global _PATCH_DEPTH
        _TLS.ctx = self.prev
        with _PATCH_LOCK:
            _PATCH_DEPTH -= 1
            if _PATCH_DEPTH == 0:
                torch.autograd.grad = _ORIG_AUTOGRAD_GRAD
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
    g = _ORIG_AUTOGRAD_GRAD(y.sum(), x, create_graph=True, allow_unused=True)[0]
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

    def accepts_cotangent(self, y, go):
        """``torch.autograd.grad(y, x, go)`` equals ``tdq.grad(y, x)`` when ``go`` is all ones
        (or absent for a single-element ``y``).  Execution contexts trust the planning pass,
        which checked the values (:meth:`RecordContext.accepts_cotangent`)."""
        return True


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

    def accepts_cotangent(self, y, go):
        if go is None:
            ok = y.numel() == 1
        else:
            ok = torch.is_tensor(go) and go.shape == y.shape and bool((go == 1).all())
        if not ok:
            self.jetable = False
            self.reasons.append("torch.autograd.grad with a cotangent other than ones_like(u)")
        return True   # the recording pass itself still returns the real derivative

    def note_foreign_grad(self, ys, xs):
        """A ``torch.autograd.grad`` call the jet cannot serve (not a stream w.r.t. coordinates)."""
        if any(self.lookup(y) is None for y in ys or []) or any(self.var_of.get(id(x)) is None for x in xs or []):
            self.jetable = False
            self.reasons.append("torch.autograd.grad of a tensor that is not a derivative stream of u_model")

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


def record_callable(fn, model, points, extra_args=(), return_outputs=False):
    """Run ``fn(u_model_proxy, *extra_args, *columns)`` under a RecordContext on ``points``.

    Returns ``(requests, jetable, reasons, d_out)`` (plus the callable's detached outputs with
    ``return_outputs=True``: the reference values of the plan validation in ``LossProgram``).
    """
    cols = [points[:, j:j + 1].detach().clone().requires_grad_(True) for j in range(points.shape[1])]
    ctx = RecordContext(cols, model)
    outs = None
    with use(ctx):
        try:
            out = fn(ctx.proxy(), *extra_args, *cols)
            outs = [o.detach() if torch.is_tensor(o) else o for o in
                    (out if isinstance(out, (tuple, list)) else (out,))]
        except (NotJetable, JetMiss) as e:  # pragma: no cover - defensive
            ctx.jetable = False
            ctx.reasons.append(str(e))
    if return_outputs:
        return ctx.requests, ctx.jetable, ctx.reasons, ctx.d_out, outs
    return ctx.requests, ctx.jetable, ctx.reasons, ctx.d_out
