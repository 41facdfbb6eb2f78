"""Line-search L-BFGS with the iterate and history on the device (``newton_eager=False``).

The reference's graph-mode L-BFGS is ``tfp.optimizer.lbfgs_minimize`` (tensordiffeq/fit.py:107-122:
10 correction pairs, ``tolerance=1e-20``, a Wolfe line search, ``max_iterations`` = newton_iter).
Here every vector - the iterate, the gradient, the direction, the 10 (s, y) pairs - stays on the
GPU and one L-BFGS iteration is a handful of graph replays:

* **direction** (one graph): the two-loop recursion over a fixed 10-slot history (newest last; an
  empty slot has rho = 0 and changes nothing, so the graph never changes shape), ``H0 = s.y / y.y``
  of the newest pair, then ``g.d``, ``max|g|`` and ``sum|g|`` copied to pinned host memory -
  one host read.
* **trial** (one graph): ``x = x0 + t d`` with ``t`` read from pinned host memory at replay time,
  the fused objective ``[grad | loss]`` (``LossGradEngine.evaluate_fg``: the fused training step's
  kernels), ``[DP: all-reduce]``, then ``f`` and ``g.d`` copied back - ONE host read per line-search
  trial, the only data the host-side line search needs.
* **update** (one graph): shift the history, insert ``s = x1 - x0``, ``y = g1 - g0``, ``rho``.

The line search is the strong-Wolfe bracketing / zoom of Nocedal & Wright (Alg. 3.5 / 3.6,
``c1 = 1e-4``, ``c2 = 0.9``) with safeguarded cubic interpolation, plus the approximate Wolfe
conditions of Hager & Zhang (TFP's default line search; ``delta = 0.1``, ``sigma = 0.9``,
``epsilon = 1e-6``): near the minimum the loss changes only at its rounding level, where the
sufficient-decrease test is noise - a trial within ``epsilon |f0|`` of ``f0`` whose slope satisfies
``sigma g0.d <= g.d <= (2 delta - 1) g0.d`` is accepted.  It runs on the host on the two scalars of
each trial.  A line search that finds no decrease along the L-BFGS direction drops the history and
retries along steepest descent (as for a non-descent direction); only when that fails too does the
run stop.  Stops: ``max_iterations``, ``max|g| <= tolerance``, no decrease along steepest descent
either, or an unchanged loss (TFP's zero x / f tolerances).

On a CPU (or without graphs) the same operations run eagerly; that path is the oracle of the tests
(tests/test_lbfgs_wolfe.py).
"""
from __future__ import annotations

import math

import torch

from ..graphs import capture_graph

C1, C2 = 1e-4, 0.9
HZ_DELTA, HZ_SIGMA, HZ_EPS = 0.1, 0.9, 1e-6   # approximate Wolfe (Hager & Zhang 2005, TFP's defaults)
# approximate-Wolfe loss tolerance per objective precision.  HZ's epsilon must cover the noise of
# f: with the split-bf16 objective (hi + lo operands, gradient 3.4e-6 vs fp64) TFP's 1e-6 makes
# the line search fail on AC-SA after ~1.2k of 10k iterations (L2 0.106), 1e-5 / 1e-4 after
# 1.3k / 3.8k, while 1e-3 runs all 10k (L2 4.9e-2, loss 0.061 -> 0.0044); the same start on the
# fp32 / fp64 objectives (N_f 5k) runs the full schedule at 1e-6 (tools/wolfe_diag.py,
# profiles/r6g_wolfe_diag.jsonl, r6h_wolfe_eps_sweep.jsonl)
HZ_EPS_BY_PRECISION = {"fp32": HZ_EPS, "bf16x3": 1e-3, "bf16": 1e-2}


def hz_eps_for(precision):
    """The approximate-Wolfe tolerance for an objective evaluated in ``precision``
    (``TDQ_WOLFE_EPS`` overrides)."""
    import os
    env = os.environ.get("TDQ_WOLFE_EPS")
    if env:
        return float(env)
    return HZ_EPS_BY_PRECISION.get(precision, HZ_EPS)


def _cubic(x1, f1, g1, x2, f2, g2, lo, hi):
    """Minimizer in [lo, hi] of the cubic through (x1, f1, f1') and (x2, f2, f2'), else the middle."""
    try:
        d1 = g1 + g2 - 3.0 * (f1 - f2) / (x1 - x2)
        disc = d1 * d1 - g1 * g2
        if disc >= 0 and math.isfinite(disc):
            d2 = math.copysign(math.sqrt(disc), x2 - x1)
            t = x2 - (x2 - x1) * (g2 + d2 - d1) / (g2 - g1 + 2.0 * d2)
            if math.isfinite(t):
                return min(max(t, lo), hi)
    except ZeroDivisionError:
        pass
    return 0.5 * (lo + hi)


class WolfeLBFGS:
    """State and graphs of one run (see the module docstring).  ``evaluate()`` returns
    ``[grad | loss]`` at the current ``x`` (it reads ``x`` itself, like the device L-BFGS)."""

    def __init__(self, evaluate, x, m=10, tolerance=1e-20, max_ls=25, all_reduce=None, capture_all_reduce=False,
                 use_graph=None, hz_eps=HZ_EPS):
        # float64: the diagnostic runs on a float64 objective (tools/wolfe_diag.py)
        if x.dtype not in (torch.float32, torch.float64) or not x.is_contiguous() or x.dim() != 1:
            raise ValueError("x must be a contiguous 1-D float32 / float64 tensor")
        self.evaluate, self.x, self.m = evaluate, x, int(m)
        self.tolerance, self.max_ls = float(tolerance), int(max_ls)
        self.hz_eps = float(hz_eps)   # approximate-Wolfe loss tolerance (relative to |f0|)
        self.all_reduce, self.capture_all_reduce = all_reduce, bool(capture_all_reduce)
        dev = x.device
        self.cuda = x.is_cuda
        self.use_graph = self.cuda if use_graph is None else (bool(use_graph) and self.cuda)
        p = x.numel()
        dt = x.dtype
        z = lambda *s: torch.zeros(*s, dtype=dt, device=dev)  # noqa: E731
        self.x0, self.g0, self.d, self.q = x.detach().clone(), z(p), z(p), z(p)
        self.xl, self.gl, self.gt = z(p), z(p), z(p)
        self.S, self.Y = z(self.m, p), z(self.m, p)
        self.rho, self.ys, self.yy, self.alpha = z(self.m), z(self.m), z(self.m), z(self.m)
        pin = self.cuda
        self.t_host = torch.zeros(1, dtype=dt, pin_memory=pin)
        self.t_dev = z(1)
        self.out_host = torch.zeros(4, dtype=dt, pin_memory=pin)
        self.out_dev = z(4)
        self.graphs = {}
        self.n_iter = self.func_eval = 0
        self.n_restarts = 0       # line searches retried along steepest descent
        self.reason = "running"
        self.f_hist = []

    # ------------------------------------------------------------------ device pieces -------
    def _read(self):
        """The one host read of a replay: ``out_dev`` -> pinned -> floats."""
        if self.cuda:
            torch.cuda.current_stream(self.x.device).synchronize()
        return [float(v) for v in self.out_host.tolist()]

    def _post(self):
        self.out_host.copy_(self.out_dev, non_blocking=self.cuda)

    def _op_eval(self, with_reduce=True):
        fg = self.evaluate()
        if with_reduce and self.all_reduce is not None:
            self.all_reduce(fg)
        return fg

    def _op_trial_a(self):
        self.t_dev.copy_(self.t_host, non_blocking=self.cuda)
        torch.addcmul(self.x0, self.d, self.t_dev, out=self.x)
        self._fg = self._op_eval(with_reduce=self.capture_all_reduce or not self.use_graph)

    def _op_trial_b(self):
        fg = self._fg
        self.gt.copy_(fg[:-1])
        self.out_dev[0:1].copy_(fg[-1:])
        self.out_dev[1:2].copy_(torch.dot(self.gt, self.d).reshape(1))
        self._post()

    def _op_direction(self):
        q = self.q
        q.copy_(self.g0)
        for i in reversed(range(self.m)):
            a = self.alpha[i:i + 1]
            a.copy_(self.rho[i:i + 1] * torch.dot(self.S[i], q).reshape(1))
            q.addcmul_(self.Y[i], a, value=-1.0)
        last = self.m - 1
        ok = self.rho[last:last + 1] > 0
        gamma = torch.where(ok, self.ys[last:last + 1] / torch.where(ok, self.yy[last:last + 1],
                                                                     torch.ones_like(self.yy[:1])),
                            torch.ones_like(self.ys[:1]))
        q.mul_(gamma)
        for i in range(self.m):
            b = self.rho[i:i + 1] * torch.dot(self.Y[i], q).reshape(1)
            q.addcmul_(self.S[i], self.alpha[i:i + 1] - b)
        torch.neg(q, out=self.d)
        self.out_dev[0:1].copy_(torch.dot(self.g0, self.d).reshape(1))
        self.out_dev[1:2].copy_(self.g0.abs().max().reshape(1))
        self.out_dev[2:3].copy_(self.g0.abs().sum().reshape(1))
        self.out_dev[3:4].copy_(self.d.abs().max().reshape(1))
        self._post()

    def _op_update(self):
        s = self.xl - self.x0
        y = self.gl - self.g0
        for buf, v in ((self.S, s), (self.Y, y)):
            buf[:-1].copy_(buf[1:].clone())
            buf[-1].copy_(v)
        ys = torch.dot(y, s).reshape(1)
        yy = torch.dot(y, y).reshape(1)
        for buf, v in ((self.rho, 1.0 / ys), (self.ys, ys), (self.yy, yy)):
            buf[:-1].copy_(buf[1:].clone())
            buf[-1:].copy_(v)
        self._op_accept()

    def _op_accept(self):
        self.x0.copy_(self.xl)
        self.g0.copy_(self.gl)

    def _run(self, name, fn, idempotent=True):
        """``fn`` eagerly, or its graph: at the first call one eager run (lazy initialisation),
        the capture, and - for ops that may run twice - a replay, so tensors the capture produced
        (the trial's ``[grad | loss]``) hold this call's values."""
        if not self.use_graph:
            fn()
            return
        g = self.graphs.get(name)
        if g is None:
            dev = self.x.device
            side = torch.cuda.Stream(device=dev)
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                fn()
            torch.cuda.current_stream(dev).wait_stream(side)
            torch.cuda.synchronize(dev)
            g = torch.cuda.CUDAGraph()
            with capture_graph(g, pool=self._pool()):
                fn()
            self.graphs[name] = g
            if not idempotent:
                return   # the eager run above did the work
        g.replay()

    def _pool(self):
        if getattr(self, "_gpool", None) is None:
            self._gpool = torch.cuda.graph_pool_handle()
        return self._gpool

    def _trial(self, t):
        self.t_host[0] = t
        self._run("trial_a", self._op_trial_a)
        if self.use_graph and self.all_reduce is not None and not self.capture_all_reduce:
            self.all_reduce(self._fg)
        self._run("trial_b", self._op_trial_b)
        self.func_eval += 1
        f, gtd = self._read()[:2]
        return f, gtd

    def _keep(self):
        """The last trial becomes the line search's low point (device copies, no sync)."""
        self.xl.copy_(self.x)
        self.gl.copy_(self.gt)

    # ------------------------------------------------------------------ line search ---------
    def _search(self, t, f0, gtd0, dmax):
        """Strong-Wolfe step from x0 along d: ``(t, f, gtd)`` of the accepted point (its x / g in
        ``xl`` / ``gl``), or ``None`` when no point below f0 was found."""
        best = None   # (t, f, gtd) of the low point (held in xl / gl)
        tp, fp, gp = 0.0, f0, gtd0
        bracket = None
        n = 0

        def approx_wolfe(f, gtd):
            return f <= f0 + self.hz_eps * abs(f0) and HZ_SIGMA * gtd0 <= gtd <= (2.0 * HZ_DELTA - 1.0) * gtd0

        while n < self.max_ls:
            f, gtd = self._trial(t)
            n += 1
            if not math.isfinite(f):
                bracket = ((tp, fp, gp), (t, math.inf, math.nan))
                break
            if f > f0 + C1 * t * gtd0 or (n > 1 and f >= fp):
                if approx_wolfe(f, gtd):
                    self._keep()
                    return (t, f, gtd)
                bracket = ((tp, fp, gp), (t, f, gtd))
                break
            self._keep()
            best = (t, f, gtd)
            if abs(gtd) <= -C2 * gtd0:
                return best
            if gtd >= 0:
                bracket = ((t, f, gtd), (tp, fp, gp))
                break
            t_new = _cubic(tp, fp, gp, t, f, gtd, t + 0.01 * (t - tp), 10.0 * t)
            tp, fp, gp = t, f, gtd
            t = t_new
        if bracket is None:
            return best
        (tl, fl, gl), (th, fh, gh) = bracket
        while n < self.max_ls:
            if abs(th - tl) * dmax < 1e-9 * max(1.0, abs(tl)):
                break
            lo, hi = min(tl, th), max(tl, th)
            if math.isfinite(fh) and math.isfinite(gh):
                t = _cubic(tl, fl, gl, th, fh, gh, lo, hi)
            else:
                t = 0.5 * (lo + hi)
            w = 0.1 * (hi - lo)      # keep the trial off the bracket's ends
            t = min(max(t, lo + w), hi - w)
            f, gtd = self._trial(t)
            n += 1
            if not math.isfinite(f) or f > f0 + C1 * t * gtd0 or f >= fl:
                if math.isfinite(f) and approx_wolfe(f, gtd):
                    self._keep()
                    return (t, f, gtd)
                th, fh, gh = t, (f if math.isfinite(f) else math.inf), gtd
                continue
            self._keep()
            best = (t, f, gtd)
            if abs(gtd) <= -C2 * gtd0:
                return best
            if gtd * (th - tl) >= 0:
                th, fh, gh = tl, fl, gl
            tl, fl, gl = t, f, gtd
        return best

    # ------------------------------------------------------------------ driver --------------
    def minimize(self, max_iter, on_iter=None):
        x = self.x
        fg = self._op_eval()
        self.func_eval += 1
        self.g0.copy_(fg[:-1])
        self.x0.copy_(x)
        self.out_dev[0:1].copy_(fg[-1:])
        self._post()
        f0 = self._read()[0]
        self.f_hist.append(f0)
        if not math.isfinite(f0):
            self.reason = "NaN loss"
            return self
        restarted = False
        while self.n_iter < max_iter:
            self._run("direction", self._op_direction)
            gtd0, gmax, g1, dmax = self._read()
            if gmax <= self.tolerance:
                self.reason = "gradient tolerance"
                break
            if not gtd0 < 0:
                if restarted:
                    self.reason = "no descent direction"
                    break
                self.rho.zero_()     # drop the history and take steepest descent
                restarted = True
                continue
            t = min(1.0, 1.0 / g1) if self.n_iter == 0 or restarted else 1.0
            res = self._search(t, f0, gtd0, dmax)
            if res is None:
                if not restarted:
                    # drop the history and retry along steepest descent (x0, g0 are untouched by
                    # a failed search) before giving up - ADVICE r5
                    self.rho.zero_()
                    restarted = True
                    self.n_restarts += 1
                    continue
                self.reason = "line search found no decrease"
                break
            t, f1, gtd1 = res
            ys = t * (gtd1 - gtd0)
            if ys > 1e-10:
                self._run("update", self._op_update, idempotent=False)
            else:
                self._run("accept", self._op_accept)
            restarted = False
            self.n_iter += 1
            self.f_hist.append(f1)
            if on_iter is not None:
                on_iter(self.n_iter, f1)
            if f1 == f0:
                f0 = f1
                self.reason = "no change in loss"
                break
            f0 = f1
        else:
            self.reason = "max_iterations"
        x.copy_(self.x0)
        self.min_loss = f0
        return self


def minimize(evaluate, x, max_iter, m=10, tolerance=1e-20, all_reduce=None, capture_all_reduce=False,
             use_graph=None, on_iter=None, hz_eps=HZ_EPS):
    """Line-search L-BFGS on ``x`` (in place; left at the final iterate).  Returns the
    :class:`WolfeLBFGS` (``n_iter``, ``func_eval``, ``reason``, ``min_loss``, ``f_hist``)."""
    opt = WolfeLBFGS(evaluate, x, m=m, tolerance=tolerance, all_reduce=all_reduce,
                     capture_all_reduce=capture_all_reduce, use_graph=use_graph, hz_eps=hz_eps)
    return opt.minimize(max_iter, on_iter=on_iter)
