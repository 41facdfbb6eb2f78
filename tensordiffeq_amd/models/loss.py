"""Loss assembly for collocation PINNs (reference ``CollocationSolverND.update_loss``,
models.py:116-218, and ``DiscoveryModel.loss``, models.py:343-350).

A :class:`LossProgram` is built once at compile time from the domain, BCs and user callables:

* every point set (collocation shard, IC/Dirichlet faces, periodic upper/lower faces, Neumann
  faces, assimilation data) becomes a *segment* of one device matrix ``X_all``;
* every user callable (``f_model``, each ``deriv_model``) is run once under a
  :class:`~tensordiffeq_amd.autodiff.RecordContext` on a few points to learn which derivative
  streams it needs; the union is one :class:`~tensordiffeq_amd.jet.JetPlan`;
* at run time ONE jet evaluation of the network over ``X_all`` (HIP kernels on MI355X, torch
  elsewhere) feeds every term, and the user callables only add elementwise ops.  Callables that
  cannot be served from a jet run on the generic nested-autograd path instead.

Loss definitions (SURVEY.md §2.5 "Exact numerics to match"):
  Dirichlet / IC / data   mean((u - val)^2), SA: mean((lam (u - val))^2)   (type 2: lam*mean(...))
  periodic                sum_k mean((d_k u(upper) - d_k u(lower))^2)  over every output of
                          every deriv_model (reference enforced only u, B12 - ``periodic_legacy``)
  Neumann                 sum_k mean((val - d_k u)^2)
  residual                mean(f^2), SA type 1 mean((lam f)^2), with g: mean(g(lam) f^2),
                          type 2 lam*mean(f^2); one lambda per residual (B11 fixed).
Adaptive periodic / Neumann terms, which the reference rejects (B13), take per-point weights.

Mixed plans: when some callables need derivatives beyond the fused kernels' order-2 envelope (e.g.
the periodic u_xxx, u_xxxx of AC-baseline on 2 x 201 boundary points) every point still runs on the
fused kernels with the order <= 2 plan, and the few high-order points get their extra streams from
the high-order jet kernels (``ops/jet_hi.py``) in extra rows of the same jet buffer, so the fused loss,
the fused step tail and the K-step graphs stay on (``hi_op``).  Where those kernels or the fused loss
cannot serve the program, the high-order segments run through the differentiable torch jet engine and
the loss is composed with autograd.

Data parallel: the collocation segment is this rank's shard; residual means divide by the global
count and every replicated term is scaled by ``1/world``, so per-rank losses sum to the global one.
"""
from __future__ import annotations

import math

import torch

from .. import autodiff
from ..jet import JetPlan, jet_dict
from ..utils.numerics import MSE, g_MSE


class Segment:
    def __init__(self, name, X):
        self.name = name
        self.X = X
        self.offset = 0
        self.hi = False       # mixed mode: needs the high-order plan (also in X_hi, at hi_offset)
        self.hi_offset = 0

    @property
    def n(self):
        return self.X.shape[0]


class JetParts:
    """Jets of a mixed program: ``lo`` over ``X_all`` (main plan), ``hi`` over ``X_hi``."""

    def __init__(self, lo, hi):
        self.lo, self.hi = lo, hi


class Term:
    def __init__(self, name, kind, **kw):
        self.name = name
        self.kind = kind
        self.lam = None          # index into the lambda list or None
        self.scale = 1.0         # 1/world for replicated terms
        self.denom = None        # global denominator override for sharded means
        self.__dict__.update(kw)


class LossProgram:
    def __init__(self, net, d_in, device, dtype=torch.float32, backend="auto", world=1,
                 weight_outside_sum=False, g=None, periodic_legacy=False, precision=None):
        self.net = net
        self.precision = precision   # HIP jet GEMM precision (None: ops.jet_mlp default)
        self.d_in = d_in
        self.device = torch.device(device)
        self.dtype = dtype
        self.requested_backend = backend
        self.world = world
        self.weight_outside_sum = weight_outside_sum
        self.g = g
        self.periodic_legacy = periodic_legacy
        self.segments = []
        self.terms = []
        self.callables = []   # (fn, segment names, extra_args)
        self.plan = None
        self.plan_hi = None   # mixed mode: plan of the high-order segments (torch jet engine)
        self.backend = None
        self.X_all = None
        self.X_hi = None
        self.reasons = []
        self.fused_op = None
        self.hi_op = None     # ops.jet_hi.HiJetOp: high-order streams of the X_hi points, fused path
        self.n_hi = 0

    # ---------------------------------------------------------------- building -------
    def add_segment(self, name, X):
        X = torch.as_tensor(X, dtype=self.dtype).to(self.device).reshape(-1, self.d_in).contiguous()
        seg = Segment(name, X)
        self.segments.append(seg)
        return len(self.segments) - 1

    def add_term(self, term):
        self.terms.append(term)
        return term

    def register_callable(self, fn, seg_idx, extra_args=()):
        self.callables.append((fn, seg_idx, extra_args))

    def finalize(self):
        """Plan, then lay out ``X_all``: every segment (high-order ones FIRST, so the high-order jet
        kernels see one contiguous block ``[0, n_hi)``); mixed mode also keeps ``X_hi``."""
        self._plan()
        hi = [s for s in self.segments if s.hi]
        order = hi + [s for s in self.segments if not s.hi]
        off = 0
        for s in order:
            s.offset = off
            off += s.n
        off = 0
        for s in hi:
            s.hi_offset = off
            off += s.n
        self.n_hi = off
        cat = lambda segs: torch.cat([s.X for s in segs], dim=0).contiguous() if segs \
            else torch.zeros(0, self.d_in, device=self.device)
        self.X_all = cat(order)
        self.X_hi = cat(hi) if hi else None

    @property
    def mixed(self):
        return self.plan_hi is not None

    def _plan(self):
        from ..models.networks import TanhMLP
        from ..ops import jet_mlp
        requests, jetable = set(), True
        seg_req = {}
        reasons = []
        if not isinstance(self.net, TanhMLP):
            jetable = False
            reasons.append("u_model is not a TanhMLP")
        recorded = []
        for fn, si, extra in self.callables:
            if not jetable:
                break
            X = self.segments[si].X
            probe = X[: min(8, X.shape[0])].detach().double() if X.shape[0] else X.double()
            net64 = _Float64View(self.net)
            req, ok, why, _, outs = autodiff.record_callable(fn, net64, probe, extra_args=extra,
                                                              return_outputs=True)
            requests |= req
            seg_req.setdefault(si, set()).update(req)
            recorded.append((fn, extra, probe, outs))
            if not ok:
                jetable = False
                reasons.extend(why)
        if jetable and recorded:
            ok, why = self._validate_jet(recorded, requests)
            if not ok:
                jetable = False
                reasons.append(why)
        backend = self.requested_backend
        for s in self.segments:
            s.hi = False
        if backend in ("auto", "hip") and jetable:
            plan = JetPlan(requests, self.d_in)
            ok, why = jet_mlp.hip_eligible(self.net, plan, self.device)
            if not ok and plan.order > 2:
                lo_req, hi_req, hi = self._split_by_order(seg_req)
                if hi and lo_req is not None:
                    ok_lo, why_lo = jet_mlp.hip_eligible(self.net, JetPlan(lo_req, self.d_in), self.device)
                    n_hi = sum(self.segments[i].n for i in hi)
                    n_lo = sum(sg.n for sg in self.segments) - n_hi
                    if ok_lo and n_lo >= n_hi:
                        for i in hi:
                            self.segments[i].hi = True
                        self.plan = JetPlan(lo_req, self.d_in)
                        self.plan_hi = JetPlan(hi_req, self.d_in)
                        self.backend = "hip"
                        self.reasons = reasons + [f"mixed: order-{self.plan_hi.order} segments "
                                                  f"{[self.segments[i].name for i in sorted(hi)]} on the torch jet"]
                        return
        if backend == "auto":
            if not jetable:
                backend = "autograd"
            else:
                plan = JetPlan(requests, self.d_in)
                ok, why = jet_mlp.hip_eligible(self.net, plan, self.device)
                backend = "hip" if ok else "jet"
                if not ok:
                    reasons.append(why)
        elif backend in ("jet", "hip") and not jetable:
            raise ValueError("backend %r requested but the callables are not jet-able: %s"
                             % (backend, "; ".join(reasons)))
        if backend in ("jet", "hip"):
            self.plan = JetPlan(requests, self.d_in)
            if backend == "hip":
                ok, why = jet_mlp.hip_eligible(self.net, self.plan, self.device)
                if not ok:
                    raise RuntimeError("HIP jet backend unavailable: " + why)
        self.backend = backend
        self.reasons = reasons
        if backend == "autograd" and self.requested_backend == "auto" and isinstance(self.net, TanhMLP):
            _warn_once("the loss callables run on the nested-autograd path (one to two orders of magnitude "
                       "slower than the jet kernels): " + "; ".join(reasons or ["not jet-expressible"]))

    def _validate_jet(self, recorded, requests):
        """Re-run every recorded callable in a :class:`~tensordiffeq_amd.autodiff.JetContext` on
        its float64 probe points, served by the torch jet engine with the union plan, and compare
        with the autograd values of the recording pass.  Any exception or mismatch means the jet
        path would not compute what the user wrote (e.g. a derivative taken through a name the
        recorder cannot see), so the program falls back to the autograd backend."""
        from ..jet import jet_forward
        if not requests and not any(outs for *_, outs in recorded):
            return True, ""
        plan = JetPlan(requests, self.d_in)
        w64 = [(k.detach().double(), b.detach().double()) for k, b in self.net.weights()]
        for fn, extra, probe, ref in recorded:
            if ref is None or probe.shape[0] == 0:
                continue
            try:
                with torch.no_grad():
                    J = jet_forward(probe, w64, plan)
                    cols = [probe[:, j:j + 1] for j in range(self.d_in)]
                    ctx = autodiff.JetContext(cols, jet_dict(J, plan))
                    with autodiff.use(ctx):
                        out = fn(ctx.proxy(), *extra, *cols)
                outs = list(out) if isinstance(out, (tuple, list)) else [out]
                if len(outs) != len(ref):
                    return False, f"jet validation: {getattr(fn, '__name__', fn)} returned {len(outs)} outputs, " \
                                  f"autograd {len(ref)}"
                for a, b in zip(outs, ref):
                    a = torch.as_tensor(a, dtype=torch.float64).reshape(-1)
                    b = torch.as_tensor(b, dtype=torch.float64).reshape(-1)
                    if a.numel() != b.numel() and a.numel() != 1 and b.numel() != 1:
                        return False, f"jet validation: output shape mismatch in {getattr(fn, '__name__', fn)}"
                    if not torch.allclose(a, b, rtol=1e-6, atol=1e-8 * (1.0 + float(b.abs().max()))):
                        return False, f"jet validation: {getattr(fn, '__name__', fn)} differs from autograd " \
                                      f"(max |diff| {float((a - b).abs().max()):.3e})"
            except Exception as e:  # noqa: BLE001 - any failure means "not servable from a jet"
                return False, f"jet validation: {getattr(fn, '__name__', fn)} raised {type(e).__name__}: {e}"
        return True, ""

    def _split_by_order(self, seg_req):
        """Partition segments by the order their callables need: (lo requests, hi requests, hi
        segment indices); segments without callables only need the value stream."""
        lo, hi_req, hi = {()}, set(), set()
        for si, req in seg_req.items():
            if any(len(m) > 2 for m in req):
                hi.add(si)
                hi_req |= req
            else:
                lo |= req
        return lo, hi_req, hi

    # ---------------------------------------------------------------- evaluation -----
    def seg_view(self, J, si):
        s = self.segments[si]
        if isinstance(J, JetParts):
            src, plan, off = (J.hi, self.plan_hi, s.hi_offset) if s.hi else (J.lo, self.plan, s.offset)
            return jet_dict(src[:, off:off + s.n], plan)
        return jet_dict(J[:, s.offset:s.offset + s.n], self.plan)

    def jet(self, params, X=None, plan=None):
        from ..ops import jet_mlp
        from ..jet import jet_forward
        if X is None and self.mixed:
            lo = jet_mlp.jet_eval(self.X_all, self.net, params, self.plan, self.backend, self.precision) \
                if self.X_all.shape[0] else None
            hi = jet_forward(self.X_hi, self.net.weights(params), self.plan_hi)
            return JetParts(lo, hi)
        X = self.X_all if X is None else X
        if plan is not None and plan is self.plan_hi:
            return jet_forward(X, self.net.weights(params), plan)
        return jet_mlp.jet_eval(X, self.net, params, self.plan, self.backend, self.precision)

    def plan_for(self, fn):
        """Plan that serves callable ``fn`` (the high-order one if ``fn`` runs on a hi segment)."""
        if self.mixed:
            for f, si, _ in self.callables:
                if f is fn and self.segments[si].hi:
                    return self.plan_hi
        return self.plan

    def call(self, fn, si, extra=(), J=None, X=None):
        """Evaluate a user callable on segment ``si`` (or explicit points ``X``)."""
        if self.backend == "autograd":
            Xs = self.segments[si].X if X is None else X
            cols = [Xs[:, j:j + 1].detach().clone().requires_grad_(True) for j in range(self.d_in)]
            return fn(getattr(self, "_cur_net", self.net), *extra, *cols)
        Xs = self.segments[si].X if X is None else X
        jd = self.seg_view(J, si) if X is None else jet_dict(J, self.plan_for(fn))
        cols = [Xs[:, j:j + 1] for j in range(self.d_in)]
        ctx = autodiff.JetContext(cols, jd)
        with autodiff.use(ctx):
            return fn(ctx.proxy(), *extra, *cols)

    def u_on(self, si, J=None, params=None):
        if self.backend == "autograd":
            return getattr(self, "_cur_net", self.net)(self.segments[si].X)
        s = self.segments[si]
        if isinstance(J, JetParts):
            if s.hi:
                return J.hi[0, s.hi_offset:s.hi_offset + s.n]
            J = J.lo
        return J[0, s.offset:s.offset + s.n]

    def evaluate(self, params=None, lambdas=None, extras=None):
        """Return ``(total, {term_name: value})`` (differentiable w.r.t. ``params``, ``lambdas``
        and ``extras``).  ``extras`` replaces the extra callable arguments of residual terms
        (the DiscoveryModel's coefficients)."""
        params = self.net.flat if params is None else params
        J = None
        self._cur_net = self.net
        if self.backend != "autograd":
            J = self.jet(params)
        elif params is not self.net.flat:
            self._cur_net = _ParamView(self.net, params)
        vals = {}
        total = None
        cache = {}
        self._extras = extras
        for t in self.terms:
            v = self._term(t, J, lambdas, cache)
            if t.scale != 1.0:
                v = v * t.scale
            vals[t.name] = v
            total = v if total is None else total + v
        if total is None:
            total = torch.zeros((), device=self.device)
        self._cur_net = self.net
        self._extras = None
        return total, vals

    def _lam(self, t, lambdas):
        if t.lam is None or lambdas is None:
            return None
        lam = lambdas[t.lam]
        rng = getattr(t, "lam_range", None)
        return lam if rng is None else lam[rng[0]:rng[1]]

    def _term(self, t, J, lambdas, cache):
        lam = self._lam(t, lambdas)
        osum = self.weight_outside_sum
        if t.kind in ("dirichlet", "ic", "data"):
            u = self.u_on(t.seg, J)
            val = t.val
            if lam is not None:
                return MSE(u, val, lam, osum, denom=t.denom)
            return MSE(u, val, denom=t.denom)
        if t.kind == "residual":
            key = ("res", t.seg)
            if key not in cache:
                extra = self._extras if getattr(self, "_extras", None) is not None else t.extra
                out = self.call(t.fn, t.seg, extra, J)
                cache[key] = out if isinstance(out, (tuple, list)) else (out,)
            f = cache[key][t.index]
            f = f.reshape(-1, 1) if f.dim() != 2 else f
            if lam is not None:
                if self.g is not None:
                    return g_MSE(f, 0.0, self.g(lam), denom=t.denom)
                return MSE(f, 0.0, lam, osum, denom=t.denom)
            return MSE(f, 0.0, denom=t.denom)
        if t.kind == "periodic":
            loss = None
            for (si_up, si_lo) in t.pairs:
                outs_u, outs_l = [], []
                for fn in t.fns:
                    ou = self.call(fn, si_up, (), J)
                    ol = self.call(fn, si_lo, (), J)
                    outs_u.extend(_as_list(ou))
                    outs_l.extend(_as_list(ol))
                    if self.periodic_legacy:
                        break
                if self.periodic_legacy:
                    outs_u, outs_l = outs_u[:1], outs_l[:1]
                for a, b in zip(outs_u, outs_l):
                    m = MSE(a, b, lam, osum) if lam is not None else MSE(a, b)
                    loss = m if loss is None else loss + m
            return loss
        if t.kind == "neumann":
            loss = None
            for si in t.segs:
                for fn in t.fns:
                    for o in _as_list(self.call(fn, si, (), J)):
                        m = MSE(t.val, o, lam, osum) if lam is not None else MSE(t.val, o)
                        loss = m if loss is None else loss + m
            return loss
        raise ValueError(f"unknown term kind {t.kind}")

    # ---------------------------------------------------------------- fusion ---------
    def enable_fusion(self, lambdas, extras=None):
        """Compile every term into the fused HIP loss kernel (HIP backend only).  Returns True
        when the program runs fused; otherwise the autograd-composed loss stays in use."""
        import os
        from .. import fusion
        self.fused_op = None
        self.hi_op = None
        if self.backend != "hip" or os.environ.get("TDQ_FUSED_LOSS", "1") == "0":
            return False
        if self.mixed:
            ok, why = self._hi_kernels_ok()
            if not ok:
                self.reasons.append(f"high-order segments on the torch jet: {why}")
                return False
        fl = fusion.build(self, lambdas)
        if fl is None:
            return False
        from ..ops.loss_fused import FusedLossOp
        scalars = fusion.scalar_values(fl, lambdas, extras)
        try:
            self.fused_op = FusedLossOp(fl, self, lambdas, scalars, fl.lam_offsets)
        except ValueError:
            return False
        if self.mixed:
            from ..ops.jet_hi import HiJetOp
            idx, _ = self.fused_streams()
            extra = {m: idx[m] for m in self.plan_hi.streams if m not in self.plan.index}
            self.hi_op = HiJetOp(self.net, self.plan_hi, extra, self.X_all, self.n_hi, self.device)
        return True

    def fused_streams(self):
        """``(stream -> J row, rows)`` of the fused loss: the main plan's streams, then (mixed mode)
        the high-order plan's streams the main plan lacks - the rows :class:`~..ops.jet_hi.HiJetOp`
        fills for the high-order points."""
        idx = dict(self.plan.index)
        if self.mixed:
            for m in self.plan_hi.streams:
                if m not in idx:
                    idx[m] = len(idx)
        return idx, len(idx)

    def _hi_kernels_ok(self):
        """Mixed mode on the fused path: the main plan on the split-bf16 kernels and the high-order
        plan within ops/jet_hi.py's envelope (``TDQ_HI_KERNEL=0`` keeps the torch jet)."""
        import os
        from ..ops import jet_hi, jet_hip
        from ..ops.jet_mlp import hip_config
        if os.environ.get("TDQ_HI_KERNEL", "1") == "0":
            return False, "TDQ_HI_KERNEL=0"
        if self.device.type != "cuda":
            return False, "not on a GPU"
        try:
            cfg = hip_config(self.net, self.plan, self.precision)
        except ValueError as e:
            return False, str(e)
        if not jet_hip.is_split_bf16(cfg):
            return False, f"main kernels {cfg['precision']}/{cfg.get('engine', 'fused')} (needs the split-bf16 kernels)"
        return jet_hi.eligible(self.net, self.plan_hi)

    # ---------------------------------------------------------------- prediction -----
    def residual_on(self, fn, X, params=None, extra=(), chunk=65536, values=None):
        """Evaluate residual(s) of ``fn`` on arbitrary points (no parameter gradients).

        ``values``: a list that receives the network output of every chunk - the jet's value
        stream (``streams[0] == ()``) of the same kernel launch that computed the derivatives, or
        None per chunk on the autograd backend."""
        outs = []
        for lo in range(0, X.shape[0], chunk):
            Xc = X[lo:lo + chunk]
            if self.backend == "autograd":
                cols = [Xc[:, j:j + 1].detach().clone().requires_grad_(True) for j in range(self.d_in)]
                with torch.enable_grad():
                    o = fn(_ParamView(self.net, params), *extra, *cols)
                if values is not None:
                    values.append(None)
            else:
                with torch.no_grad():
                    plan = self.plan_for(fn)
                    J = self.jet(params if params is not None else self.net.flat, X=Xc, plan=plan)
                    if values is not None:
                        values.append(J[0].reshape(Xc.shape[0], -1).detach())
                    cols = [Xc[:, j:j + 1] for j in range(self.d_in)]
                    ctx = autodiff.JetContext(cols, jet_dict(J, plan))
                    with autodiff.use(ctx):
                        o = fn(ctx.proxy(), *extra, *cols)
            o = o if isinstance(o, (tuple, list)) else (o,)
            outs.append([x.detach().reshape(Xc.shape[0], -1) for x in o])
        return [torch.cat([c[i] for c in outs], dim=0) for i in range(len(outs[0]))] if outs else []


_WARNED = set()


def _warn_once(msg):
    """One warning per distinct message per process (a fallback is decided once per program,
    but solvers rebuild programs per precision / minibatch)."""
    import warnings
    if msg not in _WARNED:
        _WARNED.add(msg)
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def _as_list(o):
    return list(o) if isinstance(o, (tuple, list)) else [o]


class _Float64View:
    """Network wrapper evaluating in float64 for the planning pass (exact request recording)."""

    def __init__(self, net):
        self.net = net

    def __call__(self, *xs, **kw):
        ws = [(k.double(), b.double()) for k, b in self.net.weights()]
        x = xs[0] if len(xs) == 1 else torch.cat(xs, dim=1)
        h = x.double()
        for i, (k, b) in enumerate(ws):
            h = torch.addmm(b, h, k)
            if i < len(ws) - 1:
                h = torch.tanh(h)
        return h


class _ParamView:
    """A TanhMLP evaluated at an explicit flat parameter tensor."""

    def __init__(self, net, params):
        self.net, self.params = net, params

    def __call__(self, *xs, **kw):
        if self.params is None:
            return self.net(*xs)
        return self.net(*xs, params=self.params)


def global_count(n_local, ctx):
    if ctx is None or not ctx.is_distributed:
        return n_local
    t = torch.tensor([float(n_local)], dtype=torch.float64, device=ctx.device)
    ctx.all_reduce_(t)
    return int(round(t.item()))


def is_finite(x):
    return math.isfinite(float(x))
