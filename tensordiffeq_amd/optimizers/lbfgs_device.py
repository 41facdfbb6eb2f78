"""Device-resident L-BFGS (build plan step 6).

Same algorithm as :func:`tensordiffeq_amd.optimizers.lbfgs.eager_lbfgs` - the reference's lua
port (tensordiffeq/optimizers.py:107-308; history 50, fixed step 0.8 after a first step of
``min(1, 1/|g|_1)``, pairs kept only when ``y.s > 1e-10``, ``H0 = y.s / y.y``, tolFun / tolX /
maxEval tests, NaN stop, best-iterate tracking with the B9 fixes) - but every piece of state lives
on the GPU and one iteration is a fixed sequence of kernel launches (``csrc/lbfgs.hip``)::

    axpy(x += t d)  ->  evaluate fg = [grad | loss] at x  ->  [DP: all-reduce fg]  ->  update(fg)

so the whole iteration is captured once as a HIP graph and replayed.  By default the update is TWO
launches (``tdq_lbfgs_update_fused``: dots + logic, then direction + descent test + the step
itself, each finished by the block that arrives last on a counter tree) instead of five (dots, logic,
direction, step, axpy); ``TDQ_LBFGS_FUSED=0`` keeps the five-launch path - both give the same
trajectory bit for bit (GPU test).  The host reads one flag
every ``poll_every`` iterations instead of ~6 scalars per iteration (reference host syncs at
optimizers.py:173,224,256-276,290); once a stopping test fires every kernel turns into a no-op,
so replays past convergence change nothing.  Under DP every rank runs the identical deterministic
update on the all-reduced ``fg``, so the replicas stay equal without further communication.

:class:`DeviceLBFGS` holds the state and exposes ``update(fg)`` / ``axpy()``; on CPU (or without
the native library, where that is allowed) the same state machine runs in torch ops, which is
also the oracle of the kernel tests.
"""
from __future__ import annotations

import ctypes
import math

import torch

from ..config import DEFAULT_LBFGS_STOP as DEFAULT_STOP

from ..graphs import capture_graph
from ..ops import _lib

# scalar-state layout (mirrors the LB_* enum of csrc/lbfgs.hip)
ACTIVE, NITER, FEVAL, K, HEAD, PUSHED, SLOT, BEST, F, FOLD, MINLOSS, BESTEP, HDIAG, T, DT1, G1, \
    REASON, GTD = range(18)
NST = 24
MAXM = 64
REASONS = {0: "running", 1: "tolFun at start", 2: "NaN loss", 3: "maxIter / maxEval",
           4: "tolFun / tolX / function change", 5: "no descent direction"}
# function-change stopping test: "fixed" |f - f_old| < tolX (what the reference evidently meant);
# "legacy" |f| < tolX - what its `tf.abs(f, f_old) < tolX` computes (optimizers.py:273, the second
# argument of tf.abs is the op name), i.e. in practice never: the run goes on to maxIter
STOP_MODES = ("fixed", "legacy")


def _ceil(a, b):
    return (a + b - 1) // b


def _f32(v):
    return float(torch.tensor(v, dtype=torch.float32))


class DeviceLBFGS:
    """L-BFGS state for a flat fp32 parameter vector ``x`` (updated in place by :meth:`axpy`)."""

    def __init__(self, x, m=50, max_iter=100, lr=0.8, tol_fun=1e-12, tol_x=1e-12, max_eval=None,
                 record_history=True, stop=DEFAULT_STOP, img_target=None):
        if not (1 <= m <= MAXM):
            raise ValueError(f"history size must be in [1, {MAXM}]")
        if stop not in STOP_MODES:
            raise ValueError(f"stop must be one of {STOP_MODES}")
        self.stop = stop
        if x.dtype != torch.float32 or not x.is_contiguous() or x.dim() != 1:
            raise ValueError("x must be a contiguous 1-D float32 tensor")
        self.x = x
        self.p = p = x.numel()
        self.m = int(m)
        self.max_iter = int(max_iter)
        self.max_eval = float(max_eval if max_eval is not None else 1.25 * max_iter)
        self.lr = float(lr)
        self.tol_fun = float(tol_fun)
        self.tol_x = float(tol_x)
        dev = x.device
        self.native = x.is_cuda and _lib.available()
        if x.is_cuda and not self.native:
            _lib.require_on_gpu()
        import os
        self.fused = self.native and os.environ.get("TDQ_LBFGS_FUSED", "1") != "0"
        f32 = dict(device=dev, dtype=torch.float32)
        f64 = dict(device=dev, dtype=torch.float64)
        self.g_old = torch.zeros(p, **f32)
        self.d = torch.zeros(p, **f32)
        self.S = torch.zeros(self.m, p, **f32)
        self.Y = torch.zeros(self.m, p, **f32)
        self.best_x = x.detach().clone()
        self.st = torch.zeros(NST, **f64)
        self.SY = torch.zeros(self.m, self.m, **f64)
        self.YY = torch.zeros(self.m, self.m, **f64)  # Y^T Y and R^{-1} (lbfgs.hip lbfgs_logic_lds)
        self.coef = torch.zeros(2 * self.m + 1, **f64)
        self.nchunks = max(1, min(64, _ceil(p, 4096)))
        self.nblk = max(1, min(2048, _ceil(p, 64)))  # direction blocks: 64 elements x 4 history quarters
        self.part = torch.zeros(self.nchunks * (self.m + 1) * 5, **f64)
        self.part2 = torch.zeros(2 * self.nblk, **f64)
        self.fhist = torch.full((self.max_iter + 1,), float("nan"), **f32) if record_history else None
        self.x_prev = torch.empty(p, **f32) if self.fused else None
        # two arrival-counter trees (lbfgs.hip last_block), zero at the start, re-armed by the kernels
        self.ticket = (torch.zeros(2 * _lib.load().tdq_lbfgs_ticket_ints(), dtype=torch.int32, device=dev)
                       if self.fused else None)
        # the objective's weight-image target (jet_hip.img_target): the fused update writes the new
        # x's images too, so the objective skips its pack launch
        self.img_target = img_target if self.fused else None
        self.reset()

    def reset(self):
        """Start a fresh run from the current ``x`` (history cleared)."""
        st = torch.zeros(NST, dtype=torch.float64)
        st[ACTIVE] = 1.0
        st[FEVAL] = 1.0
        st[MINLOSS] = math.inf
        st[BESTEP] = -1.0
        st[HDIAG] = 1.0
        st[SLOT] = -1.0
        self.st.copy_(st)
        self.SY.zero_()
        self.YY.zero_()
        self.g_old.zero_()
        self.d.zero_()
        if self.fhist is not None:
            self.fhist.fill_(float("nan"))

    # ------------------------------------------------------------------ launches ----------
    def update(self, fg):
        """Consume an evaluation ``fg = [grad (p) | loss]`` at the current ``x``: stopping tests,
        history push and the next direction / step (no host synchronisation on the GPU path)."""
        if fg.numel() != self.p + 1 or fg.dtype != torch.float32 or not fg.is_contiguous():
            raise ValueError(f"fg must be a contiguous float32 vector of {self.p + 1} elements")
        if fg.device != self.x.device:
            raise ValueError("fg and x must live on the same device")
        if self.fused:
            lib = _lib.load()
            rc = lib.tdq_lbfgs_update_fused(
                _lib.ptr(self.x), _lib.ptr(fg), _lib.ptr(self.g_old), _lib.ptr(self.d), _lib.ptr(self.S),
                _lib.ptr(self.Y), _lib.ptr(self.best_x), _lib.ptr(self.x_prev), _lib.ptr(self.st), _lib.ptr(self.SY),
                _lib.ptr(self.YY), _lib.ptr(self.coef), _lib.ptr(self.part), _lib.ptr(self.part2),
                _lib.ptr(self.fhist), _lib.ptr(self.ticket),
                self.p, self.m, self.max_iter, self.nchunks, self.nblk,
                0 if self.fhist is None else self.fhist.numel(), self.max_eval, self.lr, self.tol_fun,
                self.tol_x, 1 if self.stop == "legacy" else 0,
                None if self.img_target is None else ctypes.cast(self.img_target, ctypes.c_void_p),
                _lib.stream_ptr(self.x.device))
            _lib.check(rc, "tdq_lbfgs_update_fused")
            return
        if self.native:
            lib = _lib.load()
            rc = lib.tdq_lbfgs_update(
                _lib.ptr(self.x), _lib.ptr(fg), _lib.ptr(self.g_old), _lib.ptr(self.d), _lib.ptr(self.S),
                _lib.ptr(self.Y), _lib.ptr(self.best_x), _lib.ptr(self.st), _lib.ptr(self.SY), _lib.ptr(self.YY),
                _lib.ptr(self.coef), _lib.ptr(self.part), _lib.ptr(self.part2), _lib.ptr(self.fhist),
                self.p, self.m, self.max_iter, self.nchunks, self.nblk,
                0 if self.fhist is None else self.fhist.numel(), self.max_eval, self.lr, self.tol_fun,
                self.tol_x, 1 if self.stop == "legacy" else 0, _lib.stream_ptr(self.x.device))
            _lib.check(rc, "tdq_lbfgs_update")
            return
        with torch.no_grad():
            self._update_torch(fg)

    def axpy(self):
        """``x += t d`` (no-op once stopped; also a no-op on the fused path, whose update already
        took the step)."""
        if self.fused:
            return
        if self.native:
            lib = _lib.load()
            rc = lib.tdq_lbfgs_axpy(_lib.ptr(self.x), _lib.ptr(self.d), _lib.ptr(self.st), self.p,
                                    self.nblk, _lib.stream_ptr(self.x.device))
            _lib.check(rc, "tdq_lbfgs_axpy")
            return
        with torch.no_grad():
            if float(self.st[ACTIVE]) != 0.0:
                self.x.add_(self.d, alpha=_f32(float(self.st[T])))

    # ------------------------------------------------------------------ torch mirror ------
    def _update_torch(self, fg):
        """Host-scalar mirror of the four update kernels (CPU path and test oracle)."""
        st = self.st
        s_ = [float(v) for v in st.tolist()]
        m = self.m
        if s_[ACTIVE] == 0.0:
            st[BEST] = 0.0
            return
        g = fg[:-1].double()
        f = float(fg[-1])
        t32 = _f32(s_[T])
        s_vec = (t32 * self.d).double()
        y_vec = (fg[:-1] - self.g_old).double()
        n_iter = int(s_[NITER])
        g1 = float(g.abs().sum())
        st[G1] = g1
        best = done = 0
        reason = 0
        minloss = s_[MINLOSS]
        fh = self.fhist
        if n_iter == 0:
            if fh is not None and fh.numel() > 0:
                fh[0] = f
            if math.isfinite(f):
                best, minloss = 1, f
                st[BESTEP] = -1.0
            if g1 <= self.tol_fun:
                done, reason = 1, 1
        else:
            fe = s_[FEVAL] + 1.0
            st[FEVAL] = fe
            if fh is not None and n_iter < fh.numel():
                fh[n_iter] = f
            if math.isnan(f):
                done, reason = 1, 2
            else:
                if f < minloss:
                    best, minloss = 1, f
                    st[BESTEP] = float(n_iter - 1)
                if n_iter >= self.max_iter or fe >= self.max_eval:
                    done, reason = 1, 3
                elif g1 <= self.tol_fun or s_[DT1] <= self.tol_x or \
                        (abs(f) if self.stop == "legacy" else abs(f - s_[FOLD])) < self.tol_x:
                    done, reason = 1, 4
        st[F] = f
        st[MINLOSS] = minloss
        if best:
            self.best_x.copy_(self.x)
        st[BEST] = 0.0
        k, head = int(s_[K]), int(s_[HEAD])
        pushed, slot = 0, -1
        if done:
            st[ACTIVE] = 0.0
            st[REASON] = float(reason)
            st[PUSHED] = 0.0
            return
        n_iter += 1
        st[NITER] = float(n_iter)
        if n_iter > 1:
            ys = float(s_vec @ y_vec)
            yy = float(y_vec @ y_vec)
            if ys > 1e-10:
                if k == m:
                    slot, head = head, (head + 1) % m
                else:
                    slot, k = (head + k) % m, k + 1
                st[K], st[HEAD], st[HDIAG] = float(k), float(head), ys / yy
                self.S[slot].copy_(s_vec.float())
                self.Y[slot].copy_(y_vec.float())
                pushed = 1
        st[PUSHED], st[SLOT] = float(pushed), float(slot)
        gam = 1.0 if n_iter == 1 else float(st[HDIAG])
        if n_iter == 1 or k == 0:
            dn = -gam * g
        else:
            idx = [(head + i) % m for i in range(k)]
            Sk = self.S[idx].double()
            Yk = self.Y[idx].double()
            SY = Sk @ Yk.T
            R = torch.triu(SY)
            a = Sk @ g
            b = Yk @ g
            u = torch.linalg.solve_triangular(R, a.unsqueeze(1), upper=True).squeeze(1)
            rhs = torch.diagonal(SY) * u + gam * ((Yk @ Yk.T) @ u) - gam * b
            p1 = torch.linalg.solve_triangular(R.T, rhs.unsqueeze(1), upper=False).squeeze(1)
            dn = -gam * g - Sk.T @ p1 + gam * (Yk.T @ u)
        d = dn.float()
        self.g_old.copy_(fg[:-1])
        self.d.copy_(d)
        gtd = float(g @ d.double())
        st[GTD] = gtd
        if gtd > -self.tol_x:
            st[ACTIVE] = 0.0
            st[REASON] = 5.0
            return
        t = min(1.0, 1.0 / g1) if n_iter == 1 else self.lr
        st[T] = t
        st[DT1] = float(d.double().abs().sum()) * t
        st[FOLD] = f

    # ------------------------------------------------------------------ host queries ------
    def active(self):
        return float(self.st[ACTIVE]) != 0.0

    @property
    def n_iter(self):
        return int(self.st[NITER])

    @property
    def func_eval(self):
        return int(self.st[FEVAL])

    @property
    def min_loss(self):
        return float(self.st[MINLOSS])

    @property
    def best_epoch(self):
        return int(self.st[BESTEP])

    @property
    def reason(self):
        return REASONS.get(int(self.st[REASON]), "?")

    def history(self):
        """Loss after every evaluation (index 0 = initial point)."""
        if self.fhist is None:
            return []
        n = min(self.fhist.numel(), self.n_iter + 1)
        return self.fhist[:n].tolist()


def minimize(evaluate, x, max_iter, m=50, lr=0.8, tol_fun=1e-12, tol_x=1e-12, all_reduce=None,
             use_graph=None, poll_every=32, on_poll=None, capture_all_reduce=False, stop=DEFAULT_STOP,
             images=None):
    """Run device L-BFGS on ``x`` (in place) for at most ``max_iter`` iterations.

    ``evaluate()`` returns ``fg = [grad | loss]`` at the current ``x`` (a float32 device vector;
    it must read ``x`` itself).  ``all_reduce(buf)`` (optional, DP) sums ``fg`` over ranks in
    place between the evaluation and the update.  ``on_poll(opt)`` is called at every host poll
    (progress bars / metrics).  Returns the :class:`DeviceLBFGS` (``best_x``, ``st``,
    ``fhist``); ``x`` is left at the LAST iterate - callers restore ``best_x``.  ``stop``: the
    function-change test, see :data:`STOP_MODES`.  ``images``: ``(img_target, evaluate_nopack)``
    of a one-launch objective (``LossGradEngine.image_target``) - the fused update writes the
    next x's weight images and every evaluation after the first skips its pack launch."""
    opt = DeviceLBFGS(x, m=m, max_iter=max_iter, lr=lr, tol_fun=tol_fun, tol_x=tol_x, stop=stop,
                      img_target=images[0] if images is not None else None)
    graph_ok = x.is_cuda and opt.native
    use_graph = graph_ok if use_graph is None else (bool(use_graph) and graph_ok)
    # the first evaluation packs the images of the starting x; later ones read what the update wrote
    ev_next = images[1] if (images is not None and opt.img_target is not None) else evaluate

    def one():
        opt.axpy()
        fg = ev_next()
        if all_reduce is not None:
            all_reduce(fg)
        opt.update(fg)

    fg = evaluate()
    if all_reduce is not None:
        all_reduce(fg)
    opt.update(fg)
    if not use_graph:
        while opt.active():
            one()
            if on_poll is not None and opt.n_iter % poll_every == 0:
                on_poll(opt)
        if on_poll is not None:
            on_poll(opt)
        return opt
    dev = x.device
    # the collective between evaluation and update: captured in the iteration graph (RCCL), or a
    # host launch between two graphs (gloo)
    split = all_reduce is not None and not capture_all_reduce
    # one eager iteration on a side stream (lazy allocations / kernel loads), then capture
    side = torch.cuda.Stream(device=dev)
    side.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(side):
        one()
    torch.cuda.current_stream(dev).wait_stream(side)
    torch.cuda.synchronize(dev)
    # iterations per graph (TDQ_LBFGS_UNROLL, default 8): back-to-back replays of a one-iteration
    # graph leave the GPU idle ~9 us between graphs (tools/timeline.py); past a stopping test the
    # extra captured iterations are no-ops, so a replay may run over the end by up to K - 1
    import os
    K = 1 if split else max(1, int(os.environ.get("TDQ_LBFGS_UNROLL", "8")))
    if opt.active():
        pool = torch.cuda.graph_pool_handle()
        ga = torch.cuda.CUDAGraph()
        with capture_graph(ga, pool=pool):
            for _ in range(K):
                opt.axpy()
                fg_static = ev_next()
                if all_reduce is not None and not split:
                    all_reduce(fg_static)
                if not split:
                    opt.update(fg_static)
        gb = None
        if split:
            gb = torch.cuda.CUDAGraph()
            with capture_graph(gb, pool=pool):
                opt.update(fg_static)
        # Host polls are pipelined one batch behind the GPU: after queueing batch b's replays, the
        # host copies the scalar state (active, n_iter, f) to pinned memory behind them and only then
        # waits for batch b - 1's copy, which finished while batch b runs - so the GPU never idles
        # across a poll.  (A synchronous poll every 32 iterations left the GPU idle for the host's
        # read-back, callback and the next graph launches: AC-SA bf16x3 L-BFGS 0.377 ms per iteration
        # wall vs 0.327 ms of kernels, gpurun_out r6d.)  Batch sizes follow the host's own count of
        # launched iterations, so a run that ends at maxIter launches no extra iteration; a run that
        # stops early (a test fired) runs at most one queued batch of no-op updates.
        pin = x.is_cuda
        bufs = [torch.zeros(3, dtype=torch.float64, pin_memory=pin) for _ in range(2)]
        evs = [torch.cuda.Event(), torch.cuda.Event()]
        cur = torch.cuda.current_stream(dev)
        sel = torch.tensor([ACTIVE, NITER, F], device=dev)
        expected = opt.n_iter
        pending, b = None, 0
        launched = 1

        hostprof = os.environ.get("TDQ_LBFGS_HOSTPROF", "0") == "1"   # host enqueue vs wait split
        opt.host_times = {"enqueue_s": 0.0, "wait_s": 0.0, "batches": 0}

        def consume(i):
            if hostprof:
                import time
                t = time.perf_counter()
                evs[i].synchronize()
                opt.host_times["wait_s"] += time.perf_counter() - t
            evs[i].synchronize()
            a, it, f = bufs[i].tolist()
            opt.polled = {"active": a != 0.0, "n_iter": int(it), "f": f}
            if on_poll is not None:
                on_poll(opt)
            return a != 0.0

        while launched <= 2 * max_iter + 8 * K:   # the maxIter test always fires first
            remaining = max_iter - expected + 1
            if remaining <= 0:
                break
            n = max(1, min(poll_every, remaining))
            reps = (n + K - 1) // K
            if hostprof:
                import time
                t_enq = time.perf_counter()
            for _ in range(reps):
                ga.replay()
                if gb is not None:
                    all_reduce(fg_static)
                    gb.replay()
            if hostprof:
                opt.host_times["enqueue_s"] += time.perf_counter() - t_enq
                opt.host_times["batches"] += 1
            launched += reps * K
            expected += reps * K
            bufs[b].copy_(torch.index_select(opt.st, 0, sel), non_blocking=pin)
            evs[b].record(cur)
            if pending is not None and not consume(pending):
                pending = None
                break
            pending, b = b, b ^ 1
        if pending is not None:
            consume(pending)
        opt.polled = None
    if on_poll is not None:
        on_poll(opt)
    return opt
